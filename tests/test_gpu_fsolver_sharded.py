"""The drop-in FSolver sharded over ranks (xfemm_fsolver_set_comm): every
rank runs its own FSolver on the same .fem + mesh files, runSolver builds the
rank's row block (xfk_problem_create_dist / _harmonic_dist), the solve is
collective, rank 0 writes the .ans and deletes the mesh files.

Driven through the in-process transport (one host thread per rank, all ranks
on cuda:0), every communicator recording its calls so kernels.check_comm_logs
proves the issue order.  Against the single-device FSolver on the same files:
the .ans is identical line for line except the A column (the partial sums are
grouped per rank, so A differs in its last bits: within 1e-6 of max|A| for
the linear problems, 1e-5 nonlinear / harmonic -- the sharded-solve tolerances
of tests/test_gpu_sharded.py); TorqueBenchmark's torque passes the reference's
check (femmcli_TorqueBenchmark.lua) on every rank count.
"""
import os
import shutil
import threading

import numpy as np
import pytest

from oracle import femfile, gaptorque
from torque import torque_ok, write_case
from xfemm_amd import fsolver, kernels, synth

pytestmark = pytest.mark.gpu

MESH_EXT = (".node", ".ele", ".edge", ".pbc")


def _copy_case(base, dst_dir):
    os.makedirs(dst_dir, exist_ok=True)
    out = os.path.join(dst_dir, os.path.basename(base))
    for ext in (".fem",) + MESH_EXT:
        shutil.copy(base + ext, out + ext)
    return out


def _single(base):
    fs = fsolver.FSolver()
    fs.PathName = base
    assert fs.LoadProblemFile() and fs.runSolver(False), fs.last_error()
    return fs.stats()


def _sharded(base, nranks):
    comms = kernels.Comm.local_group(nranks)
    for c in comms:
        c.record(1)
    fss = [fsolver.FSolver(comm=comms[q]) for q in range(nranks)]
    ok, err, st = [None] * nranks, [None] * nranks, [None] * nranks

    def work(q):
        try:
            fss[q].PathName = base
            ok[q] = fss[q].LoadProblemFile() and fss[q].runSolver(False)
            err[q] = fss[q].last_error()
            st[q] = fss[q].stats()
        except Exception as ex:   # surfaced below
            err[q] = repr(ex)
            ok[q] = False

    th = [threading.Thread(target=work, args=(q,)) for q in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert all(ok), err
    order = kernels.check_comm_logs([c.log() for c in comms])
    sols = [fs.solution() for fs in fss]
    del fss
    for c in comms:
        c.close()
    return st, order, sols


def _ans_sections(path):
    """(lines before the node section, node rows as token lists, the rest)"""
    with open(path) as fh:
        lines = fh.read().split("\n")
    k = next(i for i, ln in enumerate(lines) if ln.strip().lower().startswith("[solution]"))
    nn = int(lines[k + 1])
    return lines[:k + 2], [ln.split("\t") for ln in lines[k + 2:k + 2 + nn]], lines[k + 2 + nn:]


def _compare_ans(a, b, tol, ncols=1):
    """ncols A columns after x, y: 1 static, 2 harmonic (re, im)"""
    ha, na, ra = _ans_sections(a)
    hb, nb_, rb = _ans_sections(b)
    assert ha == hb and ra == rb                      # .fem echo, elements, circuits, pbc, air gaps
    assert len(na) == len(nb_)
    m = 2 + ncols
    xa = np.array([[float(t) for t in r[:m]] for r in na])
    xb = np.array([[float(t) for t in r[:m]] for r in nb_])
    assert np.array_equal(xa[:, :2], xb[:, :2])
    assert [r[m:] for r in na] == [r[m:] for r in nb_]   # markers
    err = np.abs(xa[:, 2:] - xb[:, 2:]).max() / np.abs(xb[:, 2:]).max()
    assert err <= tol, err
    return err


@pytest.mark.parametrize("nranks", [2, 4])
def test_fsolver_sharded_torque_benchmark(tmp_path, nranks):
    deg = 30
    (tmp_path / "src").mkdir()
    base = write_case(tmp_path / "src", deg)
    ref = _copy_case(base, str(tmp_path / "one"))
    shr = _copy_case(base, str(tmp_path / "sh"))
    _single(ref)
    st, order, sols = _sharded(shr, nranks)
    err = _compare_ans(shr + ".ans", ref + ".ans", 1e-6)
    for ext in MESH_EXT:                               # rank 0 deleted them after the collective solve
        assert not os.path.exists(shr + ext), ext
    for A in sols[1:]:                                 # every rank holds the global solution
        assert np.array_equal(A[2], sols[0][2])
    ans = femfile.read_ans(shr + ".ans")
    pr = femfile.prepare_problem(femfile.parse_fem(shr + ".fem"))
    (age,) = ans.ages
    tq = gaptorque.gap_dc_torque(age, ans.A, pr.Depth, pr.LengthUnits)
    good, diff, rel = torque_ok(tq, deg)
    assert good, (tq, diff, rel)
    print("FSolver over %d ranks: A within %.2e of one device, torque %.7f, %d collectives" % (
        nranks, err, tq, order["calls"]))


@pytest.mark.parametrize("nranks", [2, 4])
def test_fsolver_sharded_200k_synthetic(tmp_path, nranks):
    kw = synth.magnetostatic(316)                      # 199,712 triangles
    base = str(tmp_path / "src" / "sq")
    os.makedirs(os.path.dirname(base))
    synth.write_problem(base, kw)
    ref = _copy_case(base, str(tmp_path / "one"))
    shr = _copy_case(base, str(tmp_path / "sh"))
    st1 = _single(ref)
    st, order, _ = _sharded(shr, nranks)
    _compare_ans(shr + ".ans", ref + ".ans", 1e-6)
    assert st[0]["cg_iters"] <= 1.25 * st1["cg_iters"] + 2, (st[0]["cg_iters"], st1["cg_iters"])


def test_fsolver_sharded_nonlinear(tmp_path):
    kw = synth.magnetostatic(80, nonlinear=True)
    base = str(tmp_path / "src" / "nl")
    os.makedirs(os.path.dirname(base))
    synth.write_problem(base, kw)
    ref = _copy_case(base, str(tmp_path / "one"))
    shr = _copy_case(base, str(tmp_path / "sh"))
    _single(ref)
    _sharded(shr, 2)
    _compare_ans(shr + ".ans", ref + ".ans", 1e-5)


def test_fsolver_sharded_harmonic(tmp_path):
    kw = synth.harmonic(40, circuits=False)
    base = str(tmp_path / "src" / "hm")
    os.makedirs(os.path.dirname(base))
    synth.write_problem(base, kw)
    ref = _copy_case(base, str(tmp_path / "one"))
    shr = _copy_case(base, str(tmp_path / "sh"))
    _single(ref)
    _sharded(shr, 2)
    _compare_ans(shr + ".ans", ref + ".ans", 1e-6, ncols=2)
