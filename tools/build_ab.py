#!/usr/bin/env python3
"""Build libsphrt.so from the csrc/ of another git revision, for A/B timing against this tree.

The variant embeds this tree's source hash (so _lib's integrity check accepts it: same ABI,
other kernels) and lands in sph_raytracer_amd/lib/variants/libsphrt_<name>.so.

    python tools/build_ab.py NAME REV [-DFLAG ...]     # e.g. base HEAD
    SPHRT_LIB=sph_raytracer_amd/lib/variants/libsphrt_base.so python tools/trace_time.py c3
"""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from sph_raytracer_amd import build  # noqa: E402

VDIR = os.path.join(ROOT, 'sph_raytracer_amd', 'lib', 'variants')


def main(name, rev, *extra):
    os.makedirs(VDIR, exist_ok=True)
    out = os.path.join(VDIR, f'libsphrt_{name}.so')
    tmp = tempfile.mkdtemp(prefix='sphrt_ab_')
    try:
        rel = os.path.relpath(build.CSRC, ROOT)
        files = subprocess.run(['git', 'ls-tree', '--name-only', rev, rel + '/'], cwd=ROOT,
                               check=True, capture_output=True, text=True).stdout.split()
        for f in files:
            blob = subprocess.run(['git', 'show', f'{rev}:{f}'], cwd=ROOT, check=True,
                                  capture_output=True).stdout
            with open(os.path.join(tmp, os.path.basename(f)), 'wb') as fh:
                fh.write(blob)
        cmd = build.command(out, extra)
        i = cmd.index('-o')
        flags = [c.replace(build.CSRC, tmp) for c in cmd[1:i] if c != '-shared']
        srcs = [os.path.join(tmp, os.path.basename(s)) for s in cmd[i + 2:]]
        objs = []
        for src in srcs:
            obj = src + '.o'
            subprocess.run([cmd[0], *flags, '-c', src, '-o', obj], check=True)
            objs.append(obj)
        subprocess.run([cmd[0], f'--offload-arch={build.ARCH}', '-shared', '-fPIC', *objs, '-o',
                        out], check=True)
    finally:
        shutil.rmtree(tmp)
    print(out)


if __name__ == '__main__':
    main(*sys.argv[1:])
