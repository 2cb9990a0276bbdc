import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Make sure the oracle and the product libraries exist (no-op when built)."""
    for d in ("oracle", "xfemm_amd"):
        so = {"oracle": os.path.join(ROOT, "oracle", "_build", "liboracle.so"),
              "xfemm_amd": os.path.join(ROOT, "xfemm_amd", "lib", "libxfemm_fsolver.so")}[d]
        if not os.path.exists(so):
            r = subprocess.run(["make", "-C", os.path.join(ROOT, d), "-j8"], capture_output=True, text=True)
            assert r.returncode == 0, r.stdout + r.stderr
    yield
