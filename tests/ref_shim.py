"""Load the reference's Python sources for parity tests.

``autograd`` is not installed (no network), so a NumPy shim stands in for
``autograd.numpy`` / ``autograd.scipy`` (the reference only uses them as NumPy).
The reference package is imported under the name ``ref_normflows`` so it never
collides with this repository's ``normflows`` compatibility shim.
Only reference *source* files are executed; nothing serialized is unpickled.
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types

import numpy as np

os.environ.setdefault("MPLBACKEND", "Agg")


def _install_autograd_shim():
    if "autograd" in sys.modules and getattr(sys.modules["autograd"], "_vinf_shim", False):
        return
    ag = types.ModuleType("autograd")
    ag._vinf_shim = True
    agnp = types.ModuleType("autograd.numpy")
    agnp.__dict__.update(np.__dict__)
    agnp.random = np.random
    sys.modules["autograd.numpy.random"] = np.random
    import scipy

    ag.numpy = agnp
    ag.scipy = scipy
    ag.grad = lambda f: (lambda *a, **k: (_ for _ in ()).throw(NotImplementedError("grad")))
    misc = types.ModuleType("autograd.misc")
    opt = types.ModuleType("autograd.misc.optimizers")
    for name in ("adam", "rmsprop", "sgd"):
        setattr(opt, name, lambda *a, **k: None)
    misc.optimizers = opt
    ag.misc = misc
    sys.modules.update({"autograd": ag, "autograd.numpy": agnp, "autograd.scipy": scipy,
                        "autograd.misc": misc, "autograd.misc.optimizers": opt})


def load_reference(root):
    """Import /root/reference/normflows/normflows as package ``ref_normflows``."""
    _install_autograd_shim()
    if "ref_normflows" in sys.modules:
        return sys.modules["ref_normflows"]
    pkg_dir = os.path.join(str(root), "normflows", "normflows")
    spec = importlib.util.spec_from_file_location(
        "ref_normflows", os.path.join(pkg_dir, "__init__.py"), submodule_search_locations=[pkg_dir])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["ref_normflows"] = mod
    spec.loader.exec_module(mod)
    return mod


def ref_module(root, name):
    load_reference(root)
    return importlib.import_module(f"ref_normflows.{name}")


def load_defs(path, names=None):
    """Execute only the top-level function/lambda/import definitions of a reference *script*
    (e.g. get_data.py parses sys.argv at import time, so it cannot be imported)."""
    import ast

    _install_autograd_shim()
    src = open(path).read()
    tree = ast.parse(src)
    keep = []
    for node in tree.body:
        if isinstance(node, (ast.FunctionDef, ast.Import, ast.ImportFrom)):
            keep.append(node)
        elif isinstance(node, ast.Assign) and isinstance(node.value, ast.Lambda):
            keep.append(node)
    mod = ast.Module(body=[n for n in keep if not (isinstance(n, (ast.Import, ast.ImportFrom))
                                                 and any(a.name.startswith(("pandas", "statsmodels",
                                                                            "normflows", "tqdm",
                                                                            "matplotlib"))
                                                         for a in n.names if hasattr(a, "name"))
                                                 or (isinstance(n, ast.ImportFrom) and
                                                     (n.module or "").startswith(
                                                         ("normflows", "matplotlib", "tqdm",
                                                          "statsmodels", "pandas"))))],
                     type_ignores=[])
    ns: dict = {}
    exec(compile(mod, path, "exec"), ns)
    return ns if names is None else {k: ns[k] for k in names}
