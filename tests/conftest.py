import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "scion-xdp-br_amd")
for p in (PKG, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    # Build the checker and the product library if this checkout has not been built yet.
    if not os.path.exists(os.path.join(ROOT, "oracle", "libhfvoracle.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    if not os.path.exists(os.path.join(PKG, "lib", "libscionhfv.so")):
        subprocess.run(["make", "-C", PKG], check=True, capture_output=True)


def rerun_on_test_build(request, timeout=600):
    """A test that needs a test hook (hfv_debug_relay_delay, _publish_delay, _br_grid, _br_split:
    compiled into lib/libscionhfv_test.so only, never into the product library) runs in a child
    pytest process on the test build.  Returns True in the parent (the child ran it and passed),
    False in the child (run the test body)."""
    if os.environ.get("HFV_TEST_BUILD_CHILD") == "1":
        return False
    import scion_hfv as hfv
    env = dict(os.environ, HFV_LIB=hfv.TEST_LIB_PATH, HFV_TEST_BUILD_CHILD="1")
    r = subprocess.run([sys.executable, "-u", "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-m", "gpu or not gpu",
                        request.node.nodeid], cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, (r.stdout[-4000:], r.stderr[-2000:])
    assert " passed" in r.stdout, r.stdout[-2000:]
    return True


@pytest.fixture(scope="session")
def gpu_ctx():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import scion_hfv as hfv
    ctx = hfv.Ctx(0)
    yield ctx
    ctx.close()
