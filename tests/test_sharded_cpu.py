"""The sharded solve's host side on CPU: the row-block partition plan
(xfk_partition_plan, the same code xfk_problem_create_dist uses) and the
distributed PCG it drives, run as 2 gloo ranks (tests/dist_worker.py)."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from xfemm_amd import kernels, synth

import dist_worker


def _plans(N, p, world):
    return [kernels.partition_plan(N, p, r, world) for r in range(world)]


def _check_plans(N, p, plans):
    p = np.asarray(p).reshape(-1, 3)
    world = len(plans)
    # owned blocks tile [0, N)
    starts = [pl["row0"] for pl in plans]
    assert starts == sorted(starts) and starts[0] == 0
    assert sum(pl["n_own"] for pl in plans) == N
    owner = np.zeros(N, int)
    for q, pl in enumerate(plans):
        owner[pl["row0"]:pl["row0"] + pl["n_own"]] = q
    for q, pl in enumerate(plans):
        # local elements = every element touching an owned row
        touch = np.where((owner[p] == q).any(axis=1))[0]
        assert np.array_equal(np.sort(pl["elems"]), touch)
        # every node of a local element is local; owned rows come first
        l2g = pl["l2g"]
        assert np.array_equal(l2g[:pl["n_own"]], np.arange(pl["row0"], pl["row0"] + pl["n_own"]))
        assert set(np.unique(p[touch])) <= set(l2g.tolist())
        # receive ranges are contiguous slices of one peer's rows, placed after the owned block
        off = pl["n_own"]
        for peer, loff, ln, g0 in pl["recv"]:
            assert loff == off and (owner[g0:g0 + ln] == peer).all()
            assert np.array_equal(l2g[loff:loff + ln], np.arange(g0, g0 + ln))
            off += ln
            # the peer sends exactly this range
            snd = [s for s in plans[peer]["send"] if s[0] == q]
            assert len(snd) == 1 and snd[0][2] == ln and snd[0][3] == g0
            assert snd[0][1] == g0 - plans[peer]["row0"]
        assert off == pl["n_own"] + pl["n_halo"]


@pytest.mark.parametrize("world", [2, 3, 5])
def test_partition_plan_banded(world):
    kw = synth.magnetostatic(20)
    N = len(kw["x"])
    plans = _plans(N, kw["p"], world)
    _check_plans(N, kw["p"], plans)
    # row-major numbering: interior ranks talk to their two neighbours only
    for q, pl in enumerate(plans):
        assert {int(r[0]) for r in pl["recv"]} == {x for x in (q - 1, q + 1) if 0 <= x < world}


def test_partition_plan_scrambled_numbering():
    kw = synth.magnetostatic(16)
    N = len(kw["x"])
    perm = np.random.default_rng(7).permutation(N)
    p = perm[np.asarray(kw["p"])]
    plans = _plans(N, p, 3)
    _check_plans(N, p, plans)
    assert all(len(pl["recv"]) == 2 for pl in plans)


def _check_coupled(N, p, X, plans):
    """Coupled-node plans: every element touching a coupled node is local on
    every rank, the coupled nodes owned elsewhere are the first n_extra halo
    nodes, and each peer sends the ranges a rank receives from it in the same
    order (coupled ranges first)."""
    p = np.asarray(p).reshape(-1, 3)
    world = len(plans)
    isx = np.zeros(N, bool)
    isx[X] = True
    owner = np.zeros(N, int)
    for q, pl in enumerate(plans):
        owner[pl["row0"]:pl["row0"] + pl["n_own"]] = q
    for q, pl in enumerate(plans):
        touch = np.where((owner[p] == q).any(axis=1) | isx[p].any(axis=1))[0]
        assert np.array_equal(np.sort(pl["elems"]), touch)
        l2g = pl["l2g"]
        assert len(set(l2g.tolist())) == len(l2g)
        assert set(np.unique(p[touch])) <= set(l2g.tolist())
        n0, ne = pl["n_own"], pl["n_extra"]
        extra = set(np.where(isx & (owner != q))[0].tolist())
        assert set(l2g[n0:n0 + ne].tolist()) == extra
        off = n0
        for peer, loff, ln, g0 in pl["recv"]:
            assert loff == off and (owner[g0:g0 + ln] == peer).all()
            assert np.array_equal(l2g[loff:loff + ln], np.arange(g0, g0 + ln))
            off += ln
        assert off == n0 + pl["n_halo"]
        for peer in range(world):
            if peer == q:
                continue
            mine = [(int(r[2]), int(r[3])) for r in pl["recv"] if r[0] == peer]
            theirs = [(int(t[2]), int(t[3])) for t in plans[peer]["send"] if t[0] == q]
            assert mine == theirs


@pytest.mark.parametrize("world", [2, 3, 4])
def test_partition_plan_coupled_nodes(world):
    kw = synth.bc_showcase(12)
    N = len(kw["x"])
    X = np.unique(np.asarray(kw["pbc"]).reshape(-1, 3)[:, :2])
    plans = [kernels.partition_plan(N, kw["p"], r, world, coupled=X) for r in range(world)]
    _check_coupled(N, kw["p"], X, plans)
    assert sum(pl["n_extra"] for pl in plans) == (world - 1) * len(X)
    # without coupled nodes the plan is the ordinary one
    plain = _plans(N, kw["p"], world)
    _check_plans(N, kw["p"], plain)
    assert all(pl["n_extra"] == 0 for pl in plain)


def test_partition_plan_rejects_bad_sizes():
    kw = synth.magnetostatic(4)
    with pytest.raises(kernels.XfkError):
        kernels.partition_plan(len(kw["x"]), kw["p"], 3, 3)
    with pytest.raises(kernels.XfkError):
        kernels.partition_plan(len(kw["x"]), kw["p"], 0, len(kw["x"]) + 1)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2])
def test_sharded_pcg_gloo(world):
    """2 gloo ranks: halo slices + all-reduced partials reproduce the global solve."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(dist_worker.run, args=(world, _free_port(), 24, d), nprocs=world, join=True)
        it, err, npeers = open(os.path.join(d, "result.txt")).read().split()
    assert int(npeers) == 1 and int(it) > 10
    assert float(err) <= 1e-6


def test_comm_log_checker_rejects_a_mismatched_sequence():
    """The checker itself: a rank that posts an all-reduce where its peer
    posts an exchange, or a send without its receive, is reported."""
    a = [dict(seq=0, op="allreduce", stream=0, waited=0, peer=-1, bytes=8, g0=0)]
    b = [dict(seq=0, op="exchange", stream=0, waited=0, peer=-1, bytes=0, g0=0)]
    with pytest.raises(AssertionError):
        kernels.check_comm_logs([a, b])
    e0 = [dict(seq=0, op="exchange", stream=1, waited=1, peer=-1, bytes=0, g0=1),
          dict(seq=0, op="send", stream=1, waited=1, peer=1, bytes=80, g0=5)]
    e1 = [dict(seq=0, op="exchange", stream=1, waited=1, peer=-1, bytes=0, g0=0)]
    with pytest.raises(AssertionError):
        kernels.check_comm_logs([e0, e1])
