import faulthandler
import os
import sys
import threading

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
    config.addinivalue_line("markers", "fullsize: whole BASELINE-size frames against the oracle (GPU)")


# Per-test stall watchdog (GPU tests): a test that runs longer than this is
# taken to be stalled — every host thread's Python stack, the library's
# report of the blocking calls its threads sit in (rt_debug_read
# RT_DEBUG_HOST_WAITS) and each open context's stream states go to stderr,
# and the process exits (status 70), well before the GPU box's 3-minute
# silence limit would kill the run without a word.  The whole GPU suite takes
# about a minute; no single test takes more than a few seconds.
WATCHDOG_S = float(os.environ.get("RT_TEST_WATCHDOG_S", "100"))


def _task_states():
    """Every thread of this process as the kernel sees it: name, state and
    wait channel (futex, an amdgpu/kfd wait, ...)."""
    out = []
    for tid in sorted(os.listdir("/proc/self/task"), key=int):
        base = f"/proc/self/task/{tid}/"
        try:
            comm = open(base + "comm").read().strip()
            state = open(base + "stat").read().rsplit(")", 1)[1].split()[0]
            wchan = open(base + "wchan").read().strip() or "-"
            sysc = open(base + "syscall").read().split()[0]
        except OSError:
            continue
        out.append(f"  tid {tid} {comm!r} state {state} wchan {wchan} syscall {sysc}")
    return "\n".join(out)


def _stall_dump(name):
    # pytest captures fd 2 during a test: the dump goes to a file of its own
    # (gpurun_out/ travels back from the GPU box) and to the terminal writer's fd
    path = os.path.join(ROOT, "gpurun_out", f"stall_{os.getpid()}.txt")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    f = open(path, "w")

    def out(text):
        f.write(text + "\n")
        f.flush()

    out(f"=== watchdog: {name} still running after {WATCHDOG_S:.0f} s ===")
    try:
        rtmod = sys.modules.get("unity_raytracer_amd.raytracing") or _rt_pkg.load().raytracing
        out(rtmod.host_waits_report(None))
        out("threads (kernel view):\n" + _task_states())
        for c in [c for c in list(rtmod.LIVE_CONTEXTS) if getattr(c, "h", None)]:
            out(rtmod.host_waits_report(c))
    except Exception as e:  # the dump must not hide the stall itself
        out(f"(library report failed: {e!r})")
    faulthandler.dump_traceback(file=f, all_threads=True)
    f.close()
    try:
        os.write(2, open(path, "rb").read())
    except OSError:
        pass
    os._exit(70)


@pytest.fixture(autouse=True)
def _watchdog(request):
    if request.node.get_closest_marker("gpu") is None:
        yield
        return
    t = threading.Timer(WATCHDOG_S, _stall_dump, args=(request.node.nodeid,))
    t.daemon = True
    t.start()
    try:
        yield
    finally:
        t.cancel()


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
