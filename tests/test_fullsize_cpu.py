"""Pins the vectorised Static2D restatement (tests/fullsize.py) that the
full-size GPU tests use as their checker: against the C oracle's assembled
system (itself bit-exact to the reference's golden .ans files) and, for the
nonlinear case, the converged oracle's answer is a fixed point of its secant
system."""
import numpy as np
import pytest

import fullsize
from oracle import oracle
from util import converged, synth_to_oracle
from xfemm_amd import synth


@pytest.mark.parametrize("cells", [40, 61])
def test_restated_system_equals_oracle(cells):
    pr, mesh, _ = synth_to_oracle(synth.magnetostatic(cells))
    K, b, _ = fullsize.assemble(pr, mesh)
    M, bo = oracle.system(pr, mesh)
    assert abs(K - M).max() <= 1e-14 * abs(M).max()
    assert np.abs(b - bo).max() <= 1e-14 * np.abs(bo).max()


def test_converged_nonlinear_answer_is_secant_fixed_point():
    pr, mesh, _ = synth_to_oracle(synth.magnetostatic(48, nonlinear=True))
    V = converged(pr, mesh) / fullsize.C_ANS
    K, b, _ = fullsize.assemble(pr, mesh, V)
    assert np.linalg.norm(b - K @ V) <= 1e-12 * np.linalg.norm(b)
    # and a plain linear solve is not (the check has teeth)
    K0, b0, _ = fullsize.assemble(pr, mesh)
    assert np.linalg.norm(b0 - K @ V) / np.linalg.norm(b0) < 1e-12
    assert np.linalg.norm(b - K0 @ V) > 1e-5 * np.linalg.norm(b)
