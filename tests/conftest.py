import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
ORACLE = os.path.join(ROOT, "oracle")
if os.path.dirname(os.path.abspath(__file__)) not in sys.path:
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
if ORACLE not in sys.path:
    sys.path.insert(0, ORACLE)

import _rt_pkg  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device")


@pytest.fixture(scope="session")
def rt():
    mod = _rt_pkg.load()
    # measuring sessions only: run the suite against a library variant
    # (unity-raytracer_amd/lib/variants/<name>/librt_mi355.so)
    v = os.environ.get("RT_TEST_LIB_VARIANT")
    if v:
        mod.abi.LIB_PATH = os.path.join(ROOT, "unity-raytracer_amd", "lib", "variants", v, "librt_mi355.so")
    return mod


@pytest.fixture(scope="session")
def orc():
    return _rt_pkg.load_oracle()


@pytest.fixture(scope="session")
def gpu_ctx(rt):
    """One rt_ctx for the whole GPU session (one process, one device)."""
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a gfx950 device (run with -m 'not gpu' on CPU)")
    torch.cuda.init()
    ctx = rt.Context()
    yield ctx
    ctx.close()
