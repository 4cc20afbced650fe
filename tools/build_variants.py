#!/usr/bin/env python3
"""Build A/B variants of libsphrt.so (same ABI, different -D switches) next to the product build.

    python tools/build_variants.py NAME=-DFLAG=1,-DOTHER=0 ...
    SPHRT_LIB=sph_raytracer_amd/lib/variants/libsphrt_NAME.so python tools/prof_forward.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from sph_raytracer_amd import build  # noqa: E402

VDIR = os.path.join(ROOT, 'sph_raytracer_amd', 'lib', 'variants')


def main(specs):
    os.makedirs(VDIR, exist_ok=True)
    for spec in specs:
        name, _, flags = spec.partition('=')
        out = os.path.join(VDIR, f'libsphrt_{name}.so')
        build.build_lib(out, [f for f in flags.split(',') if f])
        print(out)


if __name__ == '__main__':
    main(sys.argv[1:])
