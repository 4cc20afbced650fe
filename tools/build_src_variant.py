#!/usr/bin/env python3
"""Build libsphrt.so from this tree's csrc/ with some source files replaced (A/B of kernel
experiments without committing them).  The variant embeds this tree's source hash, so _lib's
integrity check accepts it (same ABI), and lands in sph_raytracer_amd/lib/variants/.

    python tools/build_src_variant.py NAME trace.hip=/tmp/trace_variant.hip [...]
    SPHRT_LIB=sph_raytracer_amd/lib/variants/libsphrt_NAME.so python tools/trace_time.py c3
"""
import os
import shutil
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from sph_raytracer_amd import build  # noqa: E402

VDIR = os.path.join(ROOT, 'sph_raytracer_amd', 'lib', 'variants')


def main(name, *repl):
    os.makedirs(VDIR, exist_ok=True)
    out = os.path.join(VDIR, f'libsphrt_{name}.so')
    tmp = tempfile.mkdtemp(prefix='sphrt_var_')
    try:
        for f in os.listdir(build.CSRC):
            shutil.copy(os.path.join(build.CSRC, f), tmp)
        for r in repl:
            dst, src = r.split('=', 1)
            shutil.copy(src, os.path.join(tmp, dst))
        cmd = build.command(out)
        i = cmd.index('-o')
        flags = [c.replace(build.CSRC, tmp) for c in cmd[1:i] if c != '-shared']
        srcs = [os.path.join(tmp, os.path.basename(s)) for s in cmd[i + 2:]]

        def comp(src):
            subprocess.run([cmd[0], *flags, '-c', src, '-o', src + '.o'], check=True)
            return src + '.o'
        with ThreadPoolExecutor(4) as pool:
            objs = list(pool.map(comp, srcs))
        subprocess.run([cmd[0], f'--offload-arch={build.ARCH}', '-shared', '-fPIC', *objs, '-o',
                        out], check=True)
    finally:
        shutil.rmtree(tmp)
    print(out)


if __name__ == '__main__':
    main(*sys.argv[1:])
