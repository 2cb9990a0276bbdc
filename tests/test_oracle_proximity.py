"""FSolver::GetFillFactor's proximity-effect permeability (fsolver.cpp:1083-1193)
as restated in oracle/femfile.py::get_fill_factor.  No reference fixture holds a
ProximityMu (the reference computes it inside FSolver, which needs the whole
solver build), so these pin properties of the restated closed forms: the
low-frequency limit 1, losses (Im < 0) that grow with frequency, the
rectangular-wire foil model against its own definition, the reference's 0/0 for
copper-clad aluminium, and that the .fem path and the in-memory path agree.
Parity of the product with this restatement: tests/test_gpu_harmonic.py."""
import cmath
import math

import numpy as np
import pytest

from oracle import femfile
from util import synth_to_oracle
from xfemm_amd import synth


def _prox(wt, f):
    pr, mesh, _ = synth_to_oracle(synth.harmonic(8, frequency=f, prox=wt))
    return pr, mesh, pr.labels[3].ProximityMu


@pytest.mark.parametrize("wt", [0, 1, 2, 3])
def test_low_frequency_limit_and_losses(wt):
    _, _, lo = _prox(wt, 1e-3)
    assert abs(lo - 1) < 1e-6   # the loss term is linear in f
    prev = 0.0
    for f in (1.0, 10.0, 100.0):
        _, _, pm = _prox(wt, f)
        assert pm.imag < 0 and abs(pm) <= 1 + 1e-12
        assert -pm.imag > prev   # losses grow with frequency below their peak
        prev = -pm.imag


def test_rectangular_wire_is_the_equivalent_foil():
    pr, mesh, pm = _prox(3, 2e4)
    lb, bp = pr.labels[3], pr.blocks[3]
    sel = mesh.lbl == 3
    x, y, p = mesh.x, mesh.y, mesh.p[sel]
    atot = 0.0001 * np.sum((y[p[:, 1]] - y[p[:, 2]]) * (x[p[:, 0]] - x[p[:, 2]])
                           - (y[p[:, 2]] - y[p[:, 0]]) * (x[p[:, 2]] - x[p[:, 1]])) / 2
    d = bp.WireD * 1e-3
    fill = math.sqrt(d * d * lb.Turns / atot)   # d / pitch
    muo = 4e-7 * math.pi
    k = cmath.sqrt(1j * 2 * math.pi * 2e4 * bp.Cduct * 1e6 * fill * muo) * d / 2
    assert abs(pm - (fill * cmath.tanh(k) / k + 1 - fill)) < 1e-12


def test_copper_clad_aluminium_is_undefined_as_in_the_reference():
    kw = synth.harmonic(8, frequency=2e4, prox=0)
    kw["blocks"][3]["LamType"] = 7
    pr, _, _ = synth_to_oracle(kw)
    assert cmath.isnan(pr.labels[3].ProximityMu)


def test_static_and_non_wound_labels_keep_unit_permeability():
    pr, _, _ = synth_to_oracle(synth.harmonic(8, frequency=2e4))
    assert all(lb.ProximityMu == 1.0 for lb in pr.labels)
    kw = synth.harmonic(8, frequency=2e4, prox=1)
    kw["frequency"] = 0.0
    pr, _, _ = synth_to_oracle(kw)
    assert pr.labels[3].ProximityMu == 1.0 and pr.labels[3].bIsWound


def test_file_path_matches_in_memory_path(tmp_path):
    kw = synth.harmonic(10, circuits=False, frequency=2e4, prox=2)
    kw["marker"] = None
    kw["points"] = []
    pm = synth_to_oracle(kw)[0].labels[3].ProximityMu
    base = str(tmp_path / "p")
    synth.write_problem(base, kw)
    pr, _ = femfile.load_problem(base)
    assert abs(pr.labels[3].ProximityMu - pm) <= 1e-12 * abs(pm)
