"""Build libsphrt.so in-tree for gfx950 with hipcc (no torch extension, no JIT cache).

    python -m sph_raytracer_amd.build [--verbose]

The library goes to sph_raytracer_amd/lib/libsphrt.so, which travels with the repo snapshot to
the GPU box (it is git-ignored, not gpurun-ignored).  Device code is compiled with
-ffp-contract=off: the solver's fused multiply-adds are explicit (csrc/solve.hpp).
"""
import hashlib
import os
import re
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


_FLAGS = ['-O3', '-std=c++17', '-fPIC', '-shared', '-ffp-contract=off', '-munsafe-fp-atomics']
FAST_SOURCES = ['fastpath.cpp', 'construct.cpp']
_FAST_FLAGS = ['-O2', '-std=c++17', '-fPIC', '-shared', '-ffp-contract=off']
# sphrt_version() ends in "src <hash>"; the same text is in the library file (host rodata), so a
# build's hash can be read without loading it
_HASH_RE = re.compile(rb'sph_raytracer_amd [^\x00]*? src ([0-9a-f]{16})')


def _hash(files, flags):
    h = hashlib.sha256()
    for name, path in [(f, os.path.join(CSRC, f)) for f in sorted(files)] + \
            [('sphrt.h', os.path.join(ROOT, 'include', 'sphrt.h'))]:
        with open(path, 'rb') as fh:
            data = fh.read()
        h.update(name.encode() + b'\0' + str(len(data)).encode() + b'\0' + data)
    h.update(' '.join(flags).encode())
    return h.hexdigest()[:16]


def source_hash():
    """Hash of everything libsphrt.so is built from: the HIP sources and headers, the C ABI
    header, the target and the compile flags (16 hex digits).  Embedded into the library at build
    time (-DSPHRT_SOURCE_HASH); _lib.load() refuses a library whose hash differs from the tree's,
    and build() rebuilds on a mismatch (not on file times)."""
    return _hash(SOURCES + HEADERS, [ARCH] + _FLAGS)


def fast_hash():
    """The same for _sphrt_fast.so (the CPython entry): its C++ sources, the C ABI header and its
    flags; checked by _lib.load_fast()."""
    return _hash(FAST_SOURCES, _FAST_FLAGS)


def have_sources():
    return all(os.path.exists(os.path.join(CSRC, f)) for f in SOURCES + HEADERS + FAST_SOURCES)


def embedded_hash(path):
    """The source hash a built library carries (None: not built, or built without one)."""
    if not os.path.exists(path):
        return None
    with open(path, 'rb') as fh:
        m = _HASH_RE.search(fh.read())
    return m.group(1).decode() if m else None


def command(out=OUT, extra=()):
    return [hipcc(), f'--offload-arch={ARCH}', *_FLAGS, f'-DSPHRT_SOURCE_HASH="{source_hash()}"',
            '-I', os.path.join(ROOT, 'include'), '-I', CSRC,
            *extra, '-o', out] + [os.path.join(CSRC, s) for s in SOURCES]


def _stale(out):
    want = fast_hash() if os.path.basename(out).startswith('_sphrt_fast') else source_hash()
    return embedded_hash(out) != want


def fast_command(out=FAST_OUT):
    """g++ for csrc/fastpath.cpp + construct.cpp: host code against torch's C++ / CPython API (torch
    headers of the interpreter that builds it), linked to the torch libraries it is loaded next
    to.  -ffp-contract=off: construct.cpp's host arithmetic (start voxels) is the exact IEEE
    products and sums numpy does."""
    import sysconfig
    import torch
    tdir = os.path.dirname(torch.__file__)
    return ['g++', *_FAST_FLAGS, '-D__HIP_PLATFORM_AMD__=1',
            '-DUSE_ROCM=1', f'-DSPHRT_SOURCE_HASH="{fast_hash()}"',
            '-I', os.path.join(tdir, 'include'),
            '-I', os.path.join(tdir, 'include', 'torch', 'csrc', 'api', 'include'),
            '-I', '/opt/rocm/include', '-I', os.path.join(ROOT, 'include'),
            '-I', sysconfig.get_paths()['include'],
            *[os.path.join(CSRC, f) for f in FAST_SOURCES], '-L', os.path.join(tdir, 'lib'),
            '-ltorch_python', '-ltorch', '-ltorch_cpu', '-lc10', '-lc10_hip',
            '-L', '/opt/rocm/lib', '-lamdhip64', '-ldl',
            f'-Wl,-rpath,{os.path.join(tdir, "lib")}', '-o', out]


def build_fast(force=False, verbose=False):
    if not force and not _stale(FAST_OUT):
        return FAST_OUT
    tmp = f'{FAST_OUT}.tmp{os.getpid()}'   # per process: ranks that start together never share it
    cmd = fast_command(tmp)
    if verbose:
        print(' '.join(cmd))
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f'g++ (fastpath.cpp, construct.cpp) failed ({res.returncode}):\n{res.stderr[-4000:]}')
    os.replace(tmp, FAST_OUT)
    return FAST_OUT


def _run(cmd, what, verbose):
    if verbose:
        print(' '.join(cmd))
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f'{what} failed ({res.returncode}):\n{res.stderr[-4000:]}')


def build_lib(out=OUT, extra=(), verbose=False):
    """hipcc every source to an object in parallel (the translation units share no device code),
    then link them: the same command() flags, a fraction of the wall time of one serial hipcc."""
    from concurrent.futures import ThreadPoolExecutor
    cmd = command(out, extra)
    i = cmd.index('-o')
    flags, srcs = [c for c in cmd[1:i] if c != '-shared'], cmd[i + 2:]
    tag = f'{os.getpid()}_{abs(hash(tuple(extra))) % 10**8}'
    objs = [f'{out}.{os.path.splitext(os.path.basename(src))[0]}.{tag}.o' for src in srcs]
    try:
        with ThreadPoolExecutor(max_workers=min(len(srcs), 8)) as pool:
            for f in [pool.submit(_run, [cmd[0], *flags, '-c', src, '-o', obj], f'hipcc {src}',
                                  verbose) for src, obj in zip(srcs, objs)]:
                f.result()
        tmp = f'{out}.tmp{os.getpid()}'   # per process: ranks that start together never share it
        _run([cmd[0], f'--offload-arch={ARCH}', '-shared', '-fPIC', *objs, '-o', tmp], 'hipcc link',
             verbose)
        os.replace(tmp, out)
    finally:
        for obj in objs:
            if os.path.exists(obj):
                os.remove(obj)
    return out


def build(force=False, verbose=False):
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    build_fast(force, verbose)
    if not force and not _stale(OUT):
        return OUT
    return build_lib(OUT, verbose=verbose)


if __name__ == '__main__':
    print(build(force='--force' in sys.argv, verbose='--verbose' in sys.argv))
