"""bench.py's own rank launcher (`python bench.py --gpus N` without torchrun).

CPU: with fewer visible GPUs than --gpus (none here) it stops before touching any GPU with a clear
message and exit status 2.  GPU: two ranks rehearsed on cuda:0 over gloo
(SPHRT_BENCH_ONE_DEVICE=1) print one JSON line with n_gpus 2 and a final all-gather of the
2 x 50-view stack that matches each rank's own shard.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_spawn_refuses_missing_gpus():
    env = dict(os.environ)
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'SPHRT_BENCH_ONE_DEVICE'):
        env.pop(k, None)
    env['HIP_VISIBLE_DEVICES'] = ''       # (on a GPU box too: no device visible)
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2'], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 2, (p.returncode, p.stderr[-2000:])
    assert 'GPU(s) visible' in p.stderr
    assert p.stdout.strip() == ''


def _rehearse(*args, timeout=600):
    """bench.py with two ranks on cuda:0 over gloo (SPHRT_BENCH_ONE_DEVICE=1) -> its JSON line."""
    env = dict(os.environ, SPHRT_BENCH_ONE_DEVICE='1')
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK'):
        env.pop(k, None)
    p = subprocess.run([sys.executable, '-u', os.path.join(ROOT, 'bench.py'), '--gpus', '2']
                       + list(args), env=env, capture_output=True, text=True, timeout=timeout,
                       cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_strong_args_refused_for_static_headline():
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--scaling', 'strong'],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 2 and 'c4 and c5' in p.stderr


@pytest.mark.gpu
def test_spawned_two_rank_rehearsal(gpu):
    rec = _rehearse('--steps', '5', '--warmup', '2')
    assert rec['n_gpus'] == 2 and rec['steps'] == 5 and rec['scaling'] == 'weak'
    assert rec['final_gather']['matches_local_shard']
    assert rec['final_gather']['stack_shape'][0] == 100
    assert rec['value'] > 0
    # the strong-scaled C4 / C5 legs every default run carries (BASELINE configs[3], [4])
    c4, c5 = rec['strong']['c4'], rec['strong']['c5_retrieval']
    assert c4.get('matches_1gpu') is True, c4
    assert c4['views_this_rank'] == 25 and c4['stack_shape'] == [50, 100, 50], c4
    assert c5.get('matches_1gpu') is True, c5
    assert c5['views_this_rank'] == 32 and c5['iterations'] == 100, c5


@pytest.mark.gpu
def test_strong_c4_two_rank_rehearsal(gpu):
    """One 50-slice dynamic volume over 2 ranks: each rank forwards its 25 views / slices and
    back-projects its residual into them; the gathered stack and gradient equal one GPU's."""
    rec = _rehearse('--config', 'c4', '--scaling', 'strong', '--steps', '5', '--warmup', '2',
                    '--no-cpu-baseline')
    assert rec['scaling'] == 'strong' and rec['n_gpus'] == 2
    s = rec['strong']
    assert s['matches_1gpu'] is True, s
    assert s['stack_rel_diff_vs_1gpu'] <= 1e-5 and s['grad_rel_diff_vs_1gpu'] <= 1e-5, s
    assert s['rays'] == 250000 and s['views_this_rank'] == 25
    assert rec['roofline']['frac'] > 0


@pytest.mark.gpu
def test_strong_c5_two_rank_rehearsal(gpu):
    """The static_retrieval.py loop with its 64 views over 2 ranks (distributed.gd: one gradient
    all_reduce per iteration): the iterates and losses equal retrieval.gd on one GPU."""
    rec = _rehearse('--config', 'c5', '--scaling', 'strong', '--steps', '30', '--warmup', '1',
                    '--no-cpu-baseline')
    s = rec['strong']
    assert rec['scaling'] == 'strong' and s['iterations'] == 30
    assert s['matches_1gpu'] is True, s
    assert s['coeffs_max_abs_diff_vs_1gpu'] <= 1e-9 and s['fidelity_last'] < s['fidelity_first']
