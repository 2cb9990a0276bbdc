"""Previous-solution problems ([PrevSoln] / [PrevType]) in the oracle's file
layer (oracle/femfile.py, restating fsolver.cpp:202-238, 801-1081, 1224-1320).

Pinned on the reference's own machine: TorqueBenchmark (configs[0]) solved,
its answer written as a WriteStatic2D .ans, then re-solved with that .ans as
[PrevSoln] (PrevType 0).  The reference then takes nodes, elements, periodic
pairs and air-gap elements from the .ans (no Cuthill renumbering) and -- as
its .ans element lines carry no edge markers -- boundary property 0 on every
element edge.  TorqueBenchmark's property 0 is the periodic "pbc1" (BdryType
4), which the element loop never reads, so the re-solve must reproduce the
first answer bit for bit and pass femmcli_TorqueBenchmark.lua's torque check.
The refusals are the reference's (messages included).  CPU only."""
import os

import numpy as np
import pytest

import ansfile
import torque
from oracle import femfile, gaptorque, oracle
from util import GOLDEN


def _prev_case(tmp_path, deg=30, prev_type=0):
    base = torque.write_case(tmp_path, deg)
    pr, mesh = femfile.load_problem(base)
    A, st, _ = oracle.solve(pr, mesh)
    fem = open(base + ".fem").read()
    ansfile.write_static_ans(base + ".ans", fem, pr, mesh, A)
    base2 = str(tmp_path / "again")
    with open(base2 + ".fem", "w") as fh:
        fh.write(ansfile.with_prev(fem, base + ".ans", prev_type))
    return pr, mesh, A, base2


def test_prev_mesh_comes_from_the_ans(tmp_path):
    pr, mesh, A, base2 = _prev_case(tmp_path)
    pr2, mesh2, prev = femfile.load_problem(base2, with_prev=True)
    assert prev.Aprev is None and not prev.Jprev.any()
    assert np.array_equal(mesh2.x, mesh.x) and np.array_equal(mesh2.y, mesh.y)
    assert np.array_equal(mesh2.p, mesh.p) and np.array_equal(mesh2.lbl, mesh.lbl)
    assert np.array_equal(mesh2.marker, mesh.marker) and np.array_equal(mesh2.pbc, mesh.pbc)
    assert (mesh2.e == 0).all() and mesh2.bandwidth == 0      # CElement() default e = {0, 0, 0}
    assert len(mesh2.ages) == len(mesh.ages)
    for a, b in zip(mesh2.ages, mesh.ages):
        assert np.array_equal(a["qn"], b["qn"]) and np.array_equal(a["qw"], b["qw"])
    assert pr2.bdrys[0].BdryFormat == 4


def test_prev_mesh_native_loader_matches(tmp_path):
    """The product's FSolver (libxfemm_fsolver.so, host part: no GPU) reads the
    same mesh back from the .ans as the restatement: nodes, elements with edge
    property 0, labels, periodic pairs."""
    from xfemm_amd import fsolver
    pr, mesh, A, base2 = _prev_case(tmp_path)
    _, mesh2, _ = femfile.load_problem(base2, with_prev=True)
    fs = fsolver.FSolver(delete_mesh_files=False)
    fs.PathName = base2
    assert fs.LoadProblemFile(), fs.last_error()
    assert fs.LoadMesh(), fs.last_error()
    x, y, mk = fs.nodes()
    p, lbl, e = fs.elements()
    assert np.array_equal(x, mesh2.x) and np.array_equal(y, mesh2.y) and np.array_equal(mk, mesh2.marker)
    assert np.array_equal(np.asarray(p).reshape(-1, 3), mesh2.p)
    assert np.array_equal(lbl, mesh2.lbl)
    assert np.array_equal(np.asarray(e).reshape(-1, 3), mesh2.e)
    assert np.array_equal(fs.pbcs(), mesh2.pbc)


def test_prev_solve_reproduces_the_machine(tmp_path):
    deg = 30
    pr, mesh, A, base2 = _prev_case(tmp_path, deg)
    pr2, mesh2 = femfile.load_problem(base2)
    A2, _, _ = oracle.solve(pr2, mesh2)
    assert np.array_equal(A2, A)
    age = mesh2.ages[0]
    tq = gaptorque.gap_dc_torque(age, A2, pr2.Depth, pr2.LengthUnits, 0.0)
    ok, diff, rel = torque.torque_ok(tq, deg)
    assert ok, (tq, diff, rel)


def test_prev_refusals(tmp_path):
    pr, mesh, A, base2 = _prev_case(tmp_path)
    fem = open(base2 + ".fem").read()
    prev = fem.split('[PrevSoln]    = "')[1].split('"')[0]
    cases = {
        "Cannot handle incremental permeability problems with frequency 0": ansfile.with_prev(fem, prev, 1),
        "Failed to open the specified previous solution file": ansfile.with_prev(fem, prev + ".missing", 0),
    }
    for msg, text in cases.items():
        with open(base2 + ".fem", "w") as fh:
            fh.write(text)
        with pytest.raises(femfile.PrevSolnError, match=msg):
            femfile.load_problem(base2)
    # an AC .ans as the previous solution
    ac = str(tmp_path / "ac.ans")
    with open(ac, "w") as fh:
        fh.write(open(prev).read().replace("[Frequency]   =  0", "[Frequency]   =  60", 1))
    with open(base2 + ".fem", "w") as fh:
        fh.write(ansfile.with_prev(fem, ac, 0))
    with pytest.raises(femfile.PrevSolnError, match="appears to be an AC problem"):
        femfile.load_problem(base2)
