"""Build libsphrt.so in-tree for gfx950 with hipcc (no torch extension, no JIT cache).

    python -m sph_raytracer_amd.build [--verbose]

The library goes to sph_raytracer_amd/lib/libsphrt.so, which travels with the repo snapshot to
the GPU box (it is git-ignored, not gpurun-ignored).  Device code is compiled with
-ffp-contract=off: the solver's fused multiply-adds are explicit (csrc/solve.hpp).
"""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, 'csrc')
OUT = os.path.join(HERE, 'lib', 'libsphrt.so')
FAST_OUT = os.path.join(HERE, 'lib', '_sphrt_fast.so')   # CPython entry for steady-state calls
SOURCES = ['api.hip', 'trace.hip', 'apply.hip', 'transpose.hip', 'rays.hip', 'loss.hip']
HEADERS = ['common.hpp', 'solve.hpp', 'introsort.hpp', 'stage.hpp']
ARCH = os.environ.get('SPHRT_ARCH', 'gfx950')


def hipcc():
    for cand in (os.environ.get('HIPCC'), '/opt/rocm/bin/hipcc', shutil.which('hipcc')):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError('hipcc not found (ROCm 7.x expected under /opt/rocm)')


def command(out=OUT, extra=()):
    return [hipcc(), f'--offload-arch={ARCH}', '-O3', '-std=c++17', '-fPIC', '-shared',
            '-ffp-contract=off', '-munsafe-fp-atomics',
            '-I', os.path.join(ROOT, 'include'), '-I', CSRC,
            *extra, '-o', out] + [os.path.join(CSRC, s) for s in SOURCES]


def _stale(out):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(ROOT, 'include', 'sphrt.h'),
                                                                   os.path.abspath(__file__)]
    return any(os.path.getmtime(d) > t for d in deps)


def fast_command(out=FAST_OUT):
    """g++ for csrc/fastpath.cpp: host code against torch's C++ / CPython API (torch headers of the
    interpreter that builds it), linked to the torch libraries it is loaded next to."""
    import sysconfig
    import torch
    tdir = os.path.dirname(torch.__file__)
    return ['g++', '-O2', '-std=c++17', '-fPIC', '-shared', '-D__HIP_PLATFORM_AMD__=1',
            '-DUSE_ROCM=1', '-I', os.path.join(tdir, 'include'),
            '-I', os.path.join(tdir, 'include', 'torch', 'csrc', 'api', 'include'),
            '-I', '/opt/rocm/include', '-I', os.path.join(ROOT, 'include'),
            '-I', sysconfig.get_paths()['include'],
            os.path.join(CSRC, 'fastpath.cpp'), '-L', os.path.join(tdir, 'lib'),
            '-ltorch_python', '-ltorch', '-ltorch_cpu', '-lc10', '-lc10_hip',
            f'-Wl,-rpath,{os.path.join(tdir, "lib")}', '-o', out]


def build_fast(force=False, verbose=False):
    src = os.path.join(CSRC, 'fastpath.cpp')
    if not force and os.path.exists(FAST_OUT) and \
            os.path.getmtime(FAST_OUT) >= max(os.path.getmtime(src), os.path.getmtime(__file__),
                                              os.path.getmtime(os.path.join(ROOT, 'include', 'sphrt.h'))):
        return FAST_OUT
    tmp = f'{FAST_OUT}.tmp{os.getpid()}'   # per process: ranks that start together never share it
    cmd = fast_command(tmp)
    if verbose:
        print(' '.join(cmd))
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f'g++ (fastpath.cpp) failed ({res.returncode}):\n{res.stderr[-4000:]}')
    os.replace(tmp, FAST_OUT)
    return FAST_OUT


def build(force=False, verbose=False):
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    build_fast(force, verbose)
    if not force and not _stale(OUT):
        return OUT
    cmd = command()
    if verbose:
        print(' '.join(cmd))
    tmp = f'{OUT}.tmp{os.getpid()}'
    cmd[cmd.index(OUT)] = tmp
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f'hipcc failed ({res.returncode}):\n{res.stderr[-4000:]}')
    os.replace(tmp, OUT)
    return OUT


if __name__ == '__main__':
    print(build(force='--force' in sys.argv, verbose='--verbose' in sys.argv))
