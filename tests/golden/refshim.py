"""Load the read-only Python reference (/root/reference/sph_raytracer) in THIS container only.

Used exclusively by ``make_golden.py`` to capture golden input/output vectors.  Nothing under
``tests/`` imports this at test time, and the GPU box never sees /root/reference.

The reference does not import under Python 3.10: ``raytracer.py:204`` uses a PEP-646 star
subscript (``all_regs_s[..., *debug_los, :]``) inside its ``debug`` branch.  We read the module
source as text, rewrite that one expression to the equivalent tuple subscript, and compile it
with the *real* file path as filename so TorchScript can still fetch ``forward_fill_jit``'s source
through ``inspect``/``linecache``.  No reference source is stored anywhere.
"""
import importlib.util
import os
import sys
import types

REF_ROOT = '/root/reference'
PKG = 'sph_raytracer'


def available():
    return os.path.isdir(os.path.join(REF_ROOT, PKG))


def load():
    """Return the reference package modules as a namespace (geometry, raytracer, loss, model)."""
    if 'refpkg_sph' in sys.modules:
        return sys.modules['refpkg_sph']
    os.environ.setdefault('PYTHONDONTWRITEBYTECODE', '1')
    sys.dont_write_bytecode = True
    pkgdir = os.path.join(REF_ROOT, PKG)
    pkg = types.ModuleType(PKG)
    pkg.__path__ = [pkgdir]
    sys.modules[PKG] = pkg
    mods = {}
    for name in ('geometry', 'raytracer', 'loss', 'model', 'retrieval'):
        path = os.path.join(pkgdir, name + '.py')
        with open(path) as f:
            src = f.read()
        # the only Python>=3.11 construct, in the debug-print branch
        src = src.replace('all_regs_s[..., *debug_los, :]',
                          'all_regs_s[(Ellipsis, *debug_los, slice(None))]')
        mod = types.ModuleType(f'{PKG}.{name}')
        mod.__file__ = path
        mod.__package__ = PKG
        sys.modules[mod.__name__] = mod
        code = compile(src, path, 'exec')
        exec(code, mod.__dict__)
        setattr(pkg, name, mod)
        mods[name] = mod
    ns = types.SimpleNamespace(**mods)
    sys.modules['refpkg_sph'] = ns
    return ns
