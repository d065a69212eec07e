"""Load the ``unity-raytracer_amd/`` package (hyphenated directory) as the
module ``unity_raytracer_amd``, and the CPU oracle wrapper as ``rt_oracle``
(the latter for tests / smoke / bench cpu_baseline only)."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "unity-raytracer_amd")


def load():
    name = "unity_raytracer_amd"
    if name in sys.modules:
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(
        name, os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def load_oracle():
    """Test infrastructure only (tests/, __graft_entry__.smoke, bench cpu_baseline)."""
    name = "rt_oracle"
    if name in sys.modules:
        return sys.modules[name]
    load()
    path = os.path.join(ROOT, "oracle", "oracle.py")
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod
