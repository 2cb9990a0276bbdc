"""The host path's number conversions (xfemm_amd/csrc/fsolver/fastnum.h)
against the C library they replace, bit for bit and character for character:

* parse_double vs strtod (fscanf "%lf", how the reference's FSolver::LoadMesh
  reads every coordinate) -- the value and the characters consumed -- on the
  reference-layout mesh files of the tests (Triangle's %.17g coordinates),
  3M generated strings (%.17g / %.Ng / %e of random doubles, near-midpoint
  decimal strings with 17-25 digits) and the odd tokens strtod alone accepts
  (hex floats, inf / nan, '+', huge exponents);
* put_g17 vs printf("%.17g") (the .ans columns) on 4M doubles: uniform,
  grid coordinates, wide exponents, random bit patterns, dyadic values whose
  decimal expansion ends in a tie, powers of ten, every power of two and its
  neighbours, zeros, subnormals, inf / nan.

tests/native/fastnum_check.cpp is compiled here with the image's g++.
"""
import os
import shutil
import subprocess
import tarfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_parse_and_format_match_the_c_library(tmp_path):
    exe = str(tmp_path / "fastnum_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(ROOT, "tests", "native", "fastnum_check.cpp")],
                   check=True)
    with tarfile.open(os.path.join(ROOT, "tests", "golden", "torque", "TorqueBenchmark_fine_30.tgz")) as tf:
        tf.extractall(tmp_path)
    files = [str(p) for p in tmp_path.rglob("*.node")] + [os.path.join(ROOT, "tests", "golden", "Temp.node")]
    files = [f for f in files if os.path.exists(f)]
    assert files
    r = subprocess.run([exe] + files, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "formatted" in r.stdout
