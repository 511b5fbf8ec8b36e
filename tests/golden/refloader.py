"""Load the read-only tlslite-ng reference *in the build container only*.

Test infrastructure, never shipped: the GPU box has no ``/root/reference``.
Used by ``make_golden.py`` to generate the committed fixtures, and by the
optional ``tests/test_reference_crosscheck.py`` (skipped where the reference is
absent).

``tlslite/__init__.py`` imports the whole API, which pulls ``ecdsa`` (not
installed, no network).  ``tlslite/utils/compat.py:14`` imports ``ecdsa`` too,
and ``tlslite/x509.py:9`` does ``from ecdsa.keys import ...``.  We therefore
(1) register ``tlslite`` and ``tlslite.utils`` as bare namespace packages so
the package ``__init__`` never runs, and (2) install a meta-path finder that
fabricates ``ecdsa`` / ``ecdsa.*`` with dummy attributes.  ``NIST192p`` raises
``AttributeError`` so ``compat.py:231-237`` sets ``ecdsaAllCurves = False``.
Nothing is written under ``/root/reference`` (``dont_write_bytecode``).
"""
import importlib.abc
import importlib.machinery
import os
import sys
import types

REF_ROOT = os.environ.get("TLSGPU_REFERENCE", "/root/reference")


def available():
    return os.path.isfile(os.path.join(REF_ROOT, "tlslite", "utils", "aesgcm.py"))


class _Dummy(object):
    def __init__(self, *a, **k):
        pass

    def __call__(self, *a, **k):
        return _Dummy()


class _FakeModule(types.ModuleType):
    def __getattr__(self, name):
        if name.startswith("__") or name == "NIST192p":
            raise AttributeError(name)
        return type(name, (_Dummy,), {})


class _EcdsaFinder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    def find_spec(self, fullname, path, target=None):
        if fullname == "ecdsa" or fullname.startswith("ecdsa."):
            return importlib.machinery.ModuleSpec(fullname, self, is_package=True)
        return None

    def create_module(self, spec):
        mod = _FakeModule(spec.name)
        mod.__path__ = []
        return mod

    def exec_module(self, module):
        pass


_loaded = False


def load():
    """Make ``import tlslite.utils.X`` resolve to the reference sources."""
    global _loaded
    if _loaded:
        return
    if not available():
        raise RuntimeError("reference not present at %s" % REF_ROOT)
    sys.dont_write_bytecode = True
    if not any(isinstance(f, _EcdsaFinder) for f in sys.meta_path):
        sys.meta_path.insert(0, _EcdsaFinder())
    for name, sub in (("tlslite", "tlslite"), ("tlslite.utils", "tlslite/utils")):
        if name not in sys.modules:
            pkg = types.ModuleType(name)
            pkg.__path__ = [os.path.join(REF_ROOT, sub)]
            sys.modules[name] = pkg
    if os.path.join(REF_ROOT, "unit_tests") not in sys.path:
        sys.path.append(os.path.join(REF_ROOT, "unit_tests"))
    _loaded = True
