#!/usr/bin/env python3
"""rocprofv3 PMC passes over the bare forward (the bench config's dtype) (tools/prof_forward.py --only) and the
per-launch numbers the bench roofline uses.  Runs rocprofv3 as a child process (this driver never
touches the GPU itself); one counter group per pass (MI355X_MICROARCH.md § rocprofv3 PMC slots).

    python tools/pmc_forward.py --out profiles/r01_forward_c2_pmc.json [--config c2]

HBM traffic per launch = 2 * FETCH_SIZE + WRITE_SIZE (KB = 1024 B): gfx950 FETCH_SIZE counts half
the bytes of wide streaming reads (MI355X_MICROARCH.md § HBM); WRITE_SIZE is exact.
"""
import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PASSES = [
    ['FETCH_SIZE'],
    ['WRITE_SIZE'],
    ['SQ_WAVES', 'SQ_INSTS_VALU', 'SQ_INSTS_SALU', 'SQ_INSTS_LDS', 'SQ_INSTS_VMEM_RD',
     'SQ_INSTS_VMEM_WR', 'SQ_WAVE_CYCLES', 'SQ_BUSY_CYCLES'],
    ['SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_WAIT_INST_LDS',
     'GRBM_GUI_ACTIVE'],
]


def adjoint_kernel_name(config, dtype='f32'):
    """The transposed CSR's forward instantiation (the adjoint / dynamic gradient), with that
    CSR's row (voxel) and segment counts."""
    code = ('import sys, torch, json; sys.path.insert(0, %r); import bench; '
            'from sph_raytracer_amd import Operator; cfg = bench.CONFIGS[%r]; '
            'g, v = bench.build_geometry(cfg, 0, 1); dev = torch.device("cuda", 0); '
            'op = Operator(g, v, device=dev, dynamic=g.dynamic); '
            'x = torch.rand(cfg[0], device=dev, dtype=torch.%s); '
            'y = torch.rand(tuple(v.shape), device=dev, dtype=x.dtype); '
            'op._apply_adjoint(y, tuple(x.shape), x.dtype, dev); '
            'n_chan, div, _ = op._layout(x.shape); '
            'T = op._paired(x.shape[0], div)["transposed"] if div else op._transposed(); '
            'c = T["desc"]; '
            'print(json.dumps([op._adjoint_kernel_name(x), c.n_rays, c.n_segments]))'
            % (ROOT, config, 'float32' if dtype == 'f32' else 'float64'))
    out = subprocess.run([sys.executable, '-c', code], check=True, capture_output=True, text=True)
    name, rows, segs = json.loads(out.stdout.strip().splitlines()[-1])
    return name, rows, segs


def kernel_name(config, dtype='f32'):
    """The forward instantiation for a config and dtype, from a child process (this driver never
    touches the GPU itself)."""
    code = ('import sys, torch; sys.path.insert(0, %r); sys.path.insert(0, %r); import bench; '
            'from sph_raytracer_amd import Operator; cfg = bench.CONFIGS[%r]; '
            'g, v = bench.build_geometry(cfg, 0, 1); op = Operator(g, v, device=torch.device("cuda", 0), dynamic=g.dynamic); '
            'x = torch.rand(cfg[0], device="cuda", dtype=torch.%s); import json; '
            'print(json.dumps([op._forward_kernel_name(x), op._csr["n"], op._csr["total"]]))'
            % (ROOT, os.path.join(ROOT, 'tools'), config,
               'float32' if dtype == 'f32' else 'float64'))
    out = subprocess.run([sys.executable, '-c', code], check=True, capture_output=True, text=True)
    return json.loads(out.stdout.strip().splitlines()[-1])


def run_pass(counters, workdir, config, reps, kernel, dtype='f32', adjoint=False):
    d = os.path.join(workdir, '_'.join(c.lower() for c in counters[:2]))
    shutil.rmtree(d, ignore_errors=True)
    cmd = ['rocprofv3', '--pmc', *counters, '-d', d, '-o', 'pmc', '--output-format', 'csv', '--',
           sys.executable, os.path.join(ROOT, 'tools', 'prof_forward.py'), '--only', '--reps',
           str(reps), '--config', config, '--dtype', dtype] + (['--adjoint'] if adjoint else [])
    subprocess.run(cmd, check=True, cwd=ROOT, stdout=subprocess.DEVNULL, timeout=90)
    files = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
    if not files:
        raise RuntimeError(f'no counter_collection.csv under {d}')
    vals = {}
    disp = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            if kernel not in row['Kernel_Name']:
                continue
            name = row['Counter_Name']
            vals.setdefault(name, []).append(float(row['Counter_Value']))
            disp.setdefault(name, set()).add(row['Dispatch_Id'])
    return {k: sum(v) / len(disp[k]) for k, v in vals.items()}, {k: len(v) for k, v in disp.items()}, files


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--out', required=True)
    ap.add_argument('--config', default='c2')
    ap.add_argument('--reps', type=int, default=10)
    ap.add_argument('--dtype', default=None, choices=['f32', 'f64'],
                    help='forward dtype (default: the bench config\'s)')
    ap.add_argument('--kernel', default=None,
                    help='kernel name substring (default: the instantiation the f32 forward runs)')
    ap.add_argument('--workdir', default=os.path.join(ROOT, 'gpurun_out', 'pmc'))
    ap.add_argument('--adjoint', action='store_true',
                    help='the adjoint\'s kernel (the transposed CSR\'s forward; a dynamic grid\'s '
                         'time-paired gradient); rays / segments are that CSR\'s rows / segments')
    ap.add_argument('--extra', action='append', default=[],
                    help='one more counter group (space-separated names) per use')
    args = ap.parse_args()
    if args.dtype is None:
        sys.path.insert(0, ROOT)
        import bench
        import torch
        args.dtype = 'f64' if bench.CONFIGS[args.config][4] == torch.float64 else 'f32'
    name, rays, segments = (adjoint_kernel_name if args.adjoint else kernel_name)(args.config,
                                                                                  args.dtype)
    if args.kernel is None:
        args.kernel = name
    per_launch, dispatches, raw = {}, {}, []
    passes = PASSES + [e.split() for e in args.extra]
    for counters in passes:
        v, n, files = run_pass(counters, args.workdir, args.config, args.reps, args.kernel,
                               args.dtype, args.adjoint)
        per_launch.update(v)
        dispatches.update(n)
        raw += files
    rec = {
        'kernel': args.kernel, 'config': args.config, 'dtype': args.dtype,
        'adjoint': args.adjoint, 'rays': rays, 'segments': segments,
        'dispatches': dispatches,
        'per_launch': per_launch,
        'correction': 'MI355X_MICROARCH.md §HBM: FETCH_SIZE reads 1/2 of wide streaming reads on '
                      'gfx950 -> doubled; WRITE_SIZE exact; KB = 1024 B; one counter group per pass',
        'traffic_bytes_per_launch': (2 * per_launch['FETCH_SIZE'] + per_launch['WRITE_SIZE']) * 1024,
        'commands': [f'rocprofv3 --pmc {" ".join(c)} -d ... -- python tools/prof_forward.py --only '
                     f'--reps {args.reps} --config {args.config} --dtype {args.dtype}'
                     + (' --adjoint' if args.adjoint else '')
                     for c in passes],
    }
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, 'w') as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == '__main__':
    main()
