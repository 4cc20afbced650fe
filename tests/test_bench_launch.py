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


@pytest.mark.gpu
def test_spawned_two_rank_rehearsal(gpu):
    env = dict(os.environ, SPHRT_BENCH_ONE_DEVICE='1')
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK'):
        env.pop(k, None)
    p = subprocess.run([sys.executable, '-u', os.path.join(ROOT, 'bench.py'), '--gpus', '2',
                        '--steps', '5', '--warmup', '2'], env=env, capture_output=True, text=True,
                       timeout=600, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert rec['n_gpus'] == 2 and rec['steps'] == 5
    assert rec['final_gather']['matches_local_shard']
    assert rec['final_gather']['stack_shape'][0] == 100
    assert rec['value'] > 0
