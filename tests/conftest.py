import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
# development only: run the suite against a variant build's package tree
# (tools/build_variant.sh makes build/abl/pkg_<name>/cpgisland_amd with that libcpg.so)
if os.environ.get("CPG_DEV_PKG"):
    sys.path.insert(0, os.environ["CPG_DEV_PKG"])


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests proper")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the oracle (test infrastructure) if needed; the product .so must exist."""
    if not os.path.exists(os.path.join(ROOT, "oracle", "_build", "libcpg_oracle.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    if not os.path.exists(os.path.join(ROOT, "cpgisland_amd", "libcpg.so")):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "cpgisland_amd", "csrc")],
                       check=True)


@pytest.fixture(scope="session")
def gpu_ctx():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cpgisland_amd import Context
    ctx = Context(0)
    yield ctx
    ctx.close()
