"""The FSolver's host thread pool (xfemm_amd/csrc/fsolver/hostpool.h): every
loop index once, and an exception thrown inside a loop -- on a worker or on
the calling thread -- comes back out of run() on the caller after every
claimed chunk has finished (tests/native/hostpool_check.cpp)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("threads", ["1", "4", "16"])
def test_host_pool_runs_every_index_and_rethrows(tmp_path, threads):
    exe = str(tmp_path / "hostpool_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-o", exe,
                    os.path.join(ROOT, "tests", "native", "hostpool_check.cpp")], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, XFEMM_HOST_THREADS=threads))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "hostpool ok" in r.stdout
