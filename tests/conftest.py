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


@pytest.fixture(scope="session")
def gpu_ctx():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import scion_hfv as hfv
    ctx = hfv.Ctx(0)
    yield ctx
    ctx.close()
