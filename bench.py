"""Bench: solved DoF/s of the fsolver static-2D hot path on MI355X.

One step = FSolver::Static2D from a device-resident mesh: symbolic phase
(node -> element lists, CSR pattern, Dirichlet row lists), row-gather element
assembly, boundary conditions, the AMG setup (built fresh every step) and the
PCG solve to the problem's Precision (1e-8), plus the Newton loop for
nonlinear problems.  Inputs (mesh + property tables) are uploaded before the
timed region.

N = 1 workload: BASELINE configs[2], synthetic 2M-triangle square-domain
magnetostatic problem with linear mu (1000 x 1000 cells -> 2,000,000
triangles, 1,002,001 nodes), synthetic data.

N > 1 (one process per GPU, torchrun), default --mode sharded: BASELINE
configs[4], ONE synthetic 20M-triangle mesh (3162 x 3162 cells, 10.0M DoF)
split in row blocks over the N ranks (xfk_problem_create_dist): each rank
assembles its rows, the PCG exchanges halo slices (RCCL send/recv) before
every SpMV and all-reduces its inner-product partials once per iteration
(RCCL all-reduce over xGMI).  "scaling": "strong" (the mesh is fixed).  After
the timed region rank 0 solves the same mesh alone on its GPU, so the line
carries the measured same-mesh speedup.  --mode replicas instead solves one
independent 2M-tri problem per GPU (parameter sweep; no collective, "weak").
The host barrier / max-over-ranks and the RCCL unique-id broadcast use
torch.distributed (gloo) on scalars only.

Output: one JSON line (rank 0) with
  roofline       the PCG SpMV (k_cg_spmv): HIP-event timing inside the timed
                 region, algorithmic bytes per launch, PMC traffic from the
                 committed rocprof summary; roofline.phases = every AMG setup
                 step and every launch of one PCG iteration (xfk_phase_profile,
                 after the timed region), annotated with the rocprof duration,
                 the PMC traffic and the bound (cache / hbm / latency) of the
                 same launch from the newest profiles/*_phase_pmc.json;
  cpu_baseline   the reference's spars.cpp via oracle/_ref, single core,
                 bounded sample;
  secondary      configs[3] (nonlinear M-19, Newton loop) and configs[4] on
                 one GPU (20M triangles, 10.0M DoF);
  cold_first_solve  the first solve of a fresh problem object (no capacity or
                 round-count hints from an earlier setup), and the next fresh
                 problem of the process (hints of the previous one, checked);
  fsolver_end_to_end  the product path: FSolver .fem -> .ans wall time on
                 configs[1] and configs[2], split into LoadMesh / Cuthill /
                 create / solve / write;
  fsolver_cold_process  bin/fsolver as a fresh child process per analysis
                 (the reference's command-line use), start to exit;
  sharded_diagnosis  (sharded runs) time inside each kind of collective on
                 every rank, the per-rank phases and their maximum over ranks.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
R_OVERRIDE = None       # tools/lab/rank0_probe.py: ranks of the compute-only probe


def _hip_sync():
    lib = ctypes.CDLL("libamdhip64.so")
    lib.hipDeviceSynchronize()


def spmv_bytes(n_rows, nnz, amg=False, col_bytes=4.0):
    """Algorithmic HBM bytes of one CSR SpMV launch of the PCG (k_cg_spmv,
    xfemm_amd/csrc/xfk_pcg.hip): val 8 B + the column index per nonzero (4 B,
    or 2 B with the AMG's 16-bit tile offsets: col_bytes as the library
    reports it), rowptr 4 B per row (+1), u read once 8 B per row, w written
    8 B per row (the fused u.w partial re-reads u from cache).  With the AMG
    preconditioner the r.u partial comes from the V-cycle's last level-0 sweep
    (which holds r and u), so the SpMV does not read r either."""
    return (8 + col_bytes) * nnz + 4 * (n_rows + 1) + 16 * n_rows


class stdout_to_stderr:
    """fd-level redirect: native code printing to stdout (the reference's
    PCGSolve printf, RCCL's init banner) must not mix into the JSON line."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        os.dup2(self.saved, 1)
        os.close(self.saved)


def host_cpu():
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(n_cells, nonlinear):
    """Reference CPU solver on the same workload as the GPU line (configs[2]:
    the 1000 x 1000-cell, 2M-triangle mesh by default): the reference's own
    CBigLinProb (spars.cpp: linked-list matrix, SSOR-PCG, SetValue) compiled
    into oracle/_ref, driven by the restated Static2D element loop
    (oracle/static2d_oracle.c).  Single thread, as the reference runs."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle import oracle
    from util import synth_to_oracle
    from xfemm_amd import synth
    kind = "reference" if oracle.ref_available() else "port"
    kw = synth.magnetostatic(n_cells, nonlinear=nonlinear)
    pr, mesh, _ = synth_to_oracle(kw)
    with stdout_to_stderr():
        t0 = time.perf_counter()
        _, st, _ = oracle.solve(pr, mesh, "reference" if kind == "reference" else "oracle")
        dt = time.perf_counter() - t0
    dof = len(mesh.x)
    iters = (", %d PCG iters" % st["cg_iters"]) if st["cg_iters"] >= 0 else ""
    return {
        "value": dof / dt,
        "unit": "DoF/s",
        "cores": 1,
        "kind": kind,
        "host_cpu": host_cpu(),
        "sample": "%dx%d-cell square (%d tri, %d DoF)%s: one full Static2D (assembly + SSOR-PCG to 1e-8%s) "
                  "in %.1f s on one core of the GPU box's host%s"
                  % (n_cells, n_cells, 2 * n_cells * n_cells, dof, " M-19" if nonlinear else "", iters, dt,
                     "; the same mesh as the GPU line" if n_cells == 1000 else "; a smaller mesh than the GPU line"),
    }


def nonlinear_secondary(device, args):
    """BASELINE configs[3] (the same 2M-tri mesh with M-19 B-H steel, full
    Newton loop with re-assembly every iteration) measured after the main
    timed region, same step definition (symbolic phase included).  The
    default solver runs the passes before the last to an Eisenstat-Walker
    forcing tolerance and the last one to Precision (XFK_OPT_NEWTON_INEXACT);
    `exact_newton` is the same workload with every pass to Precision, as the
    reference's loop (static2d.cpp:997-1008), and the distance between the
    two answers."""
    from xfemm_amd import kernels, synth
    import numpy as np
    kw = synth.magnetostatic(args.cells, nonlinear=True)

    def run(inexact):
        P = kernels.Static2DProblem(device=device, precond=args.precond, amg_sweeps=args.amg_sweeps,
                                    amg_omega=args.amg_omega, amg_dense=args.amg_dense, amg_theta=args.amg_theta,
                                    newton_inexact=inexact, **kw)
        P.solve(rebuild_symbolic=True)
        _hip_sync()
        t0 = time.perf_counter()
        res = [P.solve(rebuild_symbolic=True) for _ in range(args.secondary_steps)]
        _hip_sync()
        dt = (time.perf_counter() - t0) / args.secondary_steps
        A = P.solution()
        n = P.n_nodes
        P.close()
        return n, dt, res[-1], A

    n, dt, r, A = run(True)
    n0, dt0, r0, A0 = run(False)
    return {"workload": "configs[3]: synthetic %d-tri square-domain magnetostatic, nonlinear M-19 B-H "
                        "(Newton, re-assembly every iteration), tol %g" % (2 * args.cells ** 2, kw["precision"]),
            "metric": "solved DoF/s", "value": n / dt, "unit": "DoF/s", "ms_per_step": 1e3 * dt,
            "steps": args.secondary_steps, "warmup": 1, "newton_iters": r["newton_iters"],
            "pcg_iters": r["cg_iters"], "ms_amg_setup": r["ms_amg_setup"], "ms_assemble": r["ms_assemble"],
            "ms_symbolic": r["ms_symbolic"], "ms_solve": r["ms_solve"],
            "newton": "inexact passes (Eisenstat-Walker eta 0.05 of the pass's initial residual, the first pass "
                      "to 1e-4), the last pass to Precision",
            "exact_newton": {"value": n0 / dt0, "ms_per_step": 1e3 * dt0, "newton_iters": r0["newton_iters"],
                             "pcg_iters": r0["cg_iters"],
                             "max_dA_over_maxA": float(np.abs(A - A0).max() / np.abs(A0).max()),
                             "note": "every Newton pass to Precision, as the reference's loop"}}


def configs4_secondary(device, args):
    """BASELINE configs[4]'s mesh (3162 x 3162 cells, 20M triangles, 10.0M
    DoF) solved on ONE GPU: the N = 1 anchor of the strong-scaling curve the
    sharded N > 1 lines measure on the same mesh.  Same step definition as the
    main line (symbolic phase included), after one warm-up solve."""
    from xfemm_amd import kernels, synth
    kw = synth.magnetostatic(args.shard_cells)
    P = kernels.Static2DProblem(device=device, precond=args.precond, amg_sweeps=args.amg_sweeps,
                                amg_omega=args.amg_omega, amg_dense=args.amg_dense, amg_theta=args.amg_theta, **kw)
    P.solve(rebuild_symbolic=True)
    _hip_sync()
    t0 = time.perf_counter()
    res = [P.solve(rebuild_symbolic=True) for _ in range(args.secondary_steps)]
    _hip_sync()
    dt = (time.perf_counter() - t0) / args.secondary_steps
    n = P.n_nodes
    P.close()
    r = res[-1]
    pcg = r["ms_solve"] - r["ms_amg_setup"]
    return {"workload": "configs[4] mesh on 1 GPU: synthetic %d-tri square-domain magnetostatic, linear mu, tol %g"
                        % (2 * args.shard_cells ** 2, kw["precision"]),
            "metric": "solved DoF/s", "value": n / dt, "unit": "DoF/s", "ms_per_step": 1e3 * dt,
            "steps": args.secondary_steps, "warmup": 1, "dof": n, "nnz": r["nnz"], "pcg_iters": r["cg_iters"],
            "ms_per_pcg_iteration": pcg / max(1, r["cg_iters"]), "amg_levels": r["amg_levels"],
            "ms_amg_setup": r["ms_amg_setup"], "ms_assemble": r["ms_assemble"], "ms_symbolic": r["ms_symbolic"],
            "ms_solve": r["ms_solve"]}


def configs4_rank0_of_8(device, args):
    """One rank of the 8-GPU configs[4] run, compute only: the per-rank lower
    bound of the sharded step.  The 8 ranks first solve the mesh together
    through the in-process transport on this GPU (untimed), rank 0 recording
    every byte it receives (xfk_comm_record mode 2) over a first and a repeated
    solve; rank 0's problem is then
    rebuilt on the replay transport (xfk_comm_create_replay) and solved alone:
    its own kernels on its own 1/8 of the mesh, bit-identical to the recorded
    run, each collective replaced by a device copy of the recorded bytes.  So
    the time is rank 0's compute plus device-local copies -- no xGMI
    transfer, no wait for a peer -- and the replicated coarse levels are timed
    apart (XFK_TIME_TAIL)."""
    import threading
    from xfemm_amd import kernels, synth
    R = R_OVERRIDE or 8
    kw = synth.magnetostatic(args.shard_cells)
    opts = dict(device=device, precond=args.precond, amg_sweeps=args.amg_sweeps, amg_omega=args.amg_omega,
                amg_dense=args.amg_dense, amg_theta=args.amg_theta, amg_replicate=args.amg_replicate)
    comms = kernels.Comm.local_group(R)
    comms[0].record(2)
    for c in comms[1:]:
        c.record(1)
    probs = [kernels.Static2DProblem(**kw, comm=comms[q], **opts) for q in range(R)]
    out, err = [None] * R, [None] * R

    def work(q):
        try:   # a first and a repeated solve: the replay serves each its own segment
            for _ in range(2):
                out[q] = probs[q].solve(rebuild_symbolic=True)
        except Exception as ex:   # surfaced below
            err[q] = ex

    th = [threading.Thread(target=work, args=(q,)) for q in range(R)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    info0 = probs[0].dist_info()
    for p in probs:
        p.close()
    for e in err:
        if e is not None:
            raise e
    order = kernels.check_comm_logs([c.log() for c in comms])
    rep = comms[0].replay()
    for c in comms:
        c.close()
    P = kernels.Static2DProblem(**kw, comm=rep, **opts)
    P.solve(rebuild_symbolic=True)
    _hip_sync()
    w0 = time.monotonic_ns()
    t0 = time.perf_counter()
    res = [P.solve(rebuild_symbolic=True) for _ in range(args.secondary_steps)]
    _hip_sync()
    dt = (time.perf_counter() - t0) / args.secondary_steps
    if os.environ.get("XFK_LAB_WINDOW"):   # lab: the timed replay's window in the kernel trace's clock
        print("[window] rank0 replay %d %d solves %d" % (w0, time.monotonic_ns(), args.secondary_steps),
              file=sys.stderr, flush=True)
    rt = P.solve(rebuild_symbolic=True, time_tail=True)
    P.close()
    rep.close()
    r = res[-1]
    it = max(1, r["cg_iters"])
    pcg = r["ms_solve"] - r["ms_amg_setup"]
    return {"workload": "configs[4] rank 0 of 8, compute only: synthetic %d-tri mesh row-block sharded over 8 "
                        "ranks, rank 0's solve alone on one GPU with every collective replayed from its recording "
                        "of the 8-rank run (device copies, no peers)" % (2 * args.shard_cells ** 2),
            "metric": "per-rank step time (lower bound of the 8-GPU step)", "ms_per_step": 1e3 * dt,
            "steps": args.secondary_steps, "warmup": 1, "rank0_rows": info0["n_own"], "rank0_halo": info0["n_halo"],
            "pcg_iters": r["cg_iters"], "pcg_iters_8rank_run": out[0]["cg_iters"],
            "amg_levels": r["amg_levels"], "ms_symbolic": r["ms_symbolic"], "ms_assemble": r["ms_assemble"],
            "ms_amg_setup": r["ms_amg_setup"], "ms_per_pcg_iteration": pcg / it,
            "replicated_tail": {"ms_setup": rt["ms_rep_setup"], "ms_per_vcycle": rt["ms_rep_cycle"] / max(1, rt["rep_cycles"]),
                                "vcycles": rt["rep_cycles"],
                                "note": "every rank builds and applies the coarse levels of <= 250k global rows; per "
                                        "V-cycle: the all-gather of the coarse right-hand side (replayed: a device "
                                        "copy) + the replicated cycle (HIP events, XFK_TIME_TAIL solve after the "
                                        "timed ones)"},
            "collectives_per_solve": dict(order, calls=order["calls"] / 2.0,
                                          ops={k: v / 2.0 for k, v in order["ops"].items()},
                                          note="every rank's recorded collectives over the two recorded solves "
                                               "(first + repeated), halved: per solve")}


def diagnosis_row(P, comm, rank):
    """One rank's share of a sharded step (after the timed region): one more
    solve with every collective bracketed by HIP events on its stream
    (xfk_comm_time: the interval includes the wait for the peers' matching
    call), then one with the replicated coarse levels timed apart
    (XFK_TIME_TAIL).  Rows / halo, the step's phases, PCG iterations, calls and
    microseconds inside each kind of collective."""
    comm.time(True)
    r = P.solve(rebuild_symbolic=True)
    tm = comm.timing()
    comm.time(False)
    rt = P.solve(rebuild_symbolic=True, time_tail=True)
    info = P.dist_info()
    it = max(1, r["cg_iters"])
    return {"rank": rank, "rows": info["n_own"], "halo": info["n_halo"], "pcg_iters": r["cg_iters"],
            "ms_symbolic": r["ms_symbolic"], "ms_assemble": r["ms_assemble"], "ms_amg_setup": r["ms_amg_setup"],
            "ms_pcg": r["ms_solve"] - r["ms_amg_setup"], "ms_solve": r["ms_solve"],
            "us_per_pcg_iteration": 1e3 * (r["ms_solve"] - r["ms_amg_setup"]) / it,
            "ms_in_collectives": 1e-3 * sum(v["us"] for v in tm.values()), "collectives": tm,
            "replicated_tail": {"ms_setup": rt["ms_rep_setup"],
                                "us_per_vcycle": 1e3 * rt["ms_rep_cycle"] / max(1, rt["rep_cycles"]),
                                "vcycles": rt["rep_cycles"]}}


def diagnosis_summary(rows, transport):
    """Every rank's diagnosis_row with the maxima over ranks: the N > 1 line
    says where a sharded step's time went."""
    def mx(key):
        return max(q[key] for q in rows)
    ops = {nm: {"calls_per_solve": rows[0]["collectives"][nm]["calls"],
                "us_rank0": rows[0]["collectives"][nm]["us"],
                "us_max_over_ranks": max(q["collectives"][nm]["us"] for q in rows),
                "us_longest_call": max(q["collectives"][nm]["us_max_call"] for q in rows)}
           for nm in ("allreduce", "exchange", "allgather")}
    return {"transport": transport,
            "comm": {"ops": ops, "calls_per_solve": sum(v["calls_per_solve"] for v in ops.values()),
                     "ms_in_collectives_rank0": rows[0]["ms_in_collectives"],
                     "ms_in_collectives_max_over_ranks": mx("ms_in_collectives"),
                     "note": "one diagnostic solve after the timed region, HIP events around every collective on "
                             "its stream (xfk_comm_time): transfer + wait for the peers' matching call"},
            "max_over_ranks": {k: mx(k) for k in ("ms_symbolic", "ms_assemble", "ms_amg_setup", "ms_pcg",
                                                  "ms_solve", "us_per_pcg_iteration")},
            "ranks": rows}


def sharded_diagnosis(P, comm, dist, rank, world):
    """diagnosis_row on every rank, gathered on rank 0 (gloo all_gather_object)."""
    row = diagnosis_row(P, comm, rank)
    rows = [row]
    if dist is not None:
        rows = [None] * world
        dist.all_gather_object(rows, row)
    return diagnosis_summary(rows, "rccl") if rank == 0 else None


def local_ranks_run(args):
    """--force-sharded --local-ranks R: the sharded step of R ranks through the
    in-process transport (one host thread per rank, all on device 0) -- the
    plumbing of the N > 1 line where only one GPU exists.  The ranks
    time-share one GPU, so the step time is NOT a scaling number; the line
    carries the sharded_diagnosis block of the same code path the RCCL run
    reports."""
    import threading
    from xfemm_amd import kernels, synth
    R = args.local_ranks
    kw = synth.magnetostatic(args.shard_cells, nonlinear=args.nonlinear)
    comms = kernels.Comm.local_group(R)
    probs = [kernels.Static2DProblem(device=0, comm=comms[q], precond=args.precond, amg_sweeps=args.amg_sweeps,
                                     amg_omega=args.amg_omega, amg_dense=args.amg_dense, amg_theta=args.amg_theta,
                                     amg_replicate=args.amg_replicate, **kw) for q in range(R)]
    bar = threading.Barrier(R)
    t = [0.0, 0.0]
    rows, err = [None] * R, [None] * R

    def work(q):
        try:
            for _ in range(args.warmup):
                probs[q].solve(rebuild_symbolic=True)
            _hip_sync()
            bar.wait()
            if q == 0:
                t[0] = time.perf_counter()
            for _ in range(args.steps):
                probs[q].solve(rebuild_symbolic=True)
            _hip_sync()
            bar.wait()
            if q == 0:
                t[1] = time.perf_counter()
            rows[q] = diagnosis_row(probs[q], comms[q], q)
        except Exception as ex:   # surfaced below
            err[q] = ex
            bar.abort()

    th = [threading.Thread(target=work, args=(q,)) for q in range(R)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    n = probs[0].n_nodes
    for p in probs:
        p.close()
    for c in comms:
        c.close()
    for e in err:
        if e is not None:
            raise e
    dt = (t[1] - t[0]) / args.steps
    return {"metric": "sharded step plumbing (in-process ranks time-sharing one GPU; not a scaling number)",
            "ms_per_step": 1e3 * dt, "steps": args.steps, "warmup": args.warmup, "local_ranks": R,
            "config": {"workload": "synthetic %d-tri square-domain magnetostatic, row-block sharded over %d "
                                   "in-process ranks on one GPU" % (2 * args.shard_cells ** 2, R), "dof": n},
            "sharded_diagnosis": diagnosis_summary(rows, "in-process (LocalComm)")}


def fsolver_end_to_end(device, args):
    """The drop-in product path timed whole: FSolver .fem + fmesher files ->
    .ans (fsolver.cpp:1213-1340's sequence: LoadMesh, Cuthill-McKee, problem
    creation with the host -> HBM upload, the device solve with the solution
    read-back, the .ans write), a fresh FSolver per run as femmcli's
    mi_analyze uses it.  configs[1]: the ~200k-triangle TorqueBenchmark at
    30 degrees (tests/golden/torque/TorqueBenchmark_fine_30.tgz, made by
    tools/gen_torque_fixtures.py); configs[2]: the bench's own 2M-triangle
    mesh written in the fmesher layout (synth.write_problem).  Two runs each,
    the second reported (the first also loads the process's code objects)."""
    import shutil
    import tarfile
    import tempfile
    from xfemm_amd import fsolver, synth
    out = []
    with tempfile.TemporaryDirectory() as td:
        with tarfile.open(os.path.join(ROOT, "tests", "golden", "torque", "TorqueBenchmark_fine_30.tgz")) as tf:
            tf.extractall(td)
        cases = [("configs[1]: TorqueBenchmark refined (~200k tri, periodic + air gap), 30 deg",
                  os.path.join(td, "TorqueBenchmark_fine_30"))]
        b2 = os.path.join(td, "square")
        synth.write_problem(b2, synth.magnetostatic(args.cells))
        cases.append(("configs[2]: synthetic %d-tri square" % (2 * args.cells ** 2), b2))
        for name, base in cases:
            src = base + "_src"
            os.makedirs(src, exist_ok=True)
            for ext in (".fem", ".node", ".ele", ".edge", ".pbc"):
                shutil.copy(base + ext, os.path.join(src, os.path.basename(base) + ext))
            rec = None
            for _ in range(2):
                for ext in (".node", ".ele", ".edge", ".pbc"):   # (runSolver deletes the mesh files)
                    shutil.copy(os.path.join(src, os.path.basename(base) + ext), base + ext)
                _hip_sync()
                t0 = time.perf_counter()
                fs = fsolver.FSolver(device=device)
                fs.PathName = base
                ok = fs.LoadProblemFile() and fs.runSolver(False)
                dt = time.perf_counter() - t0
                if not ok:
                    raise RuntimeError("FSolver failed on %s: %s" % (name, fs.last_error()))
                st, tm = fs.stats(), fs.times()
                rec = {"workload": name, "dof": fs.NumNodes, "ms_wall": 1e3 * dt,
                       "dof_per_s_wall": fs.NumNodes / dt, "pcg_iters": st["cg_iters"],
                       "ms_device_solve": st["ms_solve"] + st["ms_assemble"] + st["ms_symbolic"]}
                rec.update(tm)
                del fs
            out.append(rec)
    return out


def fsolver_cold_process(args):
    """The one-shot command line as the reference runs it (cfemm/fsolver/main.cpp:
    a fresh process per analysis): xfemm_amd/bin/fsolver <problem> started as a
    child process and timed from start to exit, on configs[1] and configs[2].
    Run before this process touches the GPU (the children bring it up
    themselves).  Each case twice: with the HIP bring-up on its own thread
    beside LoadMesh / Cuthill (the default, xfk_device_init) and with it left
    to the first device call (XFEMM_NO_HIP_WARMUP=1, the serial order); the two
    .ans files must be byte-identical."""
    import filecmp
    import shutil
    import tarfile
    import tempfile
    from xfemm_amd import synth
    exe = os.path.join(ROOT, "xfemm_amd", "bin", "fsolver")
    if not os.path.exists(exe):
        return {"skipped": "xfemm_amd/bin/fsolver is not built"}
    out = []
    with tempfile.TemporaryDirectory() as td:
        with tarfile.open(os.path.join(ROOT, "tests", "golden", "torque", "TorqueBenchmark_fine_30.tgz")) as tf:
            tf.extractall(td)
        cases = [("configs[1]: TorqueBenchmark refined (~200k tri, periodic + air gap), 30 deg",
                  os.path.join(td, "TorqueBenchmark_fine_30"))]
        b2 = os.path.join(td, "square")
        synth.write_problem(b2, synth.magnetostatic(args.cells))
        cases.append(("configs[2]: synthetic %d-tri square" % (2 * args.cells ** 2), b2))
        for name, base in cases:
            rec = {"workload": name}
            ans = {}
            for mode in ("overlapped", "serial"):
                run = os.path.join(td, "run_" + mode)
                os.makedirs(run, exist_ok=True)
                dst = os.path.join(run, os.path.basename(base))
                for ext in (".fem", ".node", ".ele", ".edge", ".pbc"):
                    shutil.copy(base + ext, dst + ext)
                env = dict(os.environ)
                env.pop("XFEMM_NO_HIP_WARMUP", None)
                if mode == "serial":
                    env["XFEMM_NO_HIP_WARMUP"] = "1"
                t0 = time.perf_counter()
                r = subprocess.run([exe, dst], capture_output=True, text=True, env=env, timeout=300)
                dt = time.perf_counter() - t0
                if r.returncode != 0:
                    raise RuntimeError("bin/fsolver failed on %s (%s): rc %d\n%s%s"
                                       % (name, mode, r.returncode, r.stdout[-2000:], r.stderr[-2000:]))
                rec["ms_wall_" + mode] = 1e3 * dt
                ans[mode] = dst + ".ans"
            rec["ans_byte_identical"] = filecmp.cmp(ans["overlapped"], ans["serial"], shallow=False)
            out.append(rec)
    return {"cases": out, "note": "xfemm_amd/bin/fsolver <problem> as a child process, start to exit (process start, "
                                  "HIP runtime + device bring-up, LoadMesh, Cuthill, solve, .ans write); "
                                  "'overlapped': bring-up on its own thread from LoadProblemFile (default); "
                                  "'serial': XFEMM_NO_HIP_WARMUP=1"}


def cold_first_solve(device, args, kw):
    """A first solve of a fresh problem: new Static2DProblem (host -> HBM
    upload timed apart), then its first solve() with none of the per-problem
    hints a re-solve reuses (SpGEMM slot capacities, the nested-dissection plan
    of the dense coarsest level, MIS round batch sizes, the first PCG batch).
    The process's code objects are already loaded (it runs after the timed
    region)."""
    from xfemm_amd import kernels

    def one():
        _hip_sync()
        kernels.alloc_stats(reset=True)
        t0 = time.perf_counter()
        P = kernels.Static2DProblem(device=device, precond=args.precond, amg_sweeps=args.amg_sweeps,
                                    amg_omega=args.amg_omega, amg_dense=args.amg_dense, amg_theta=args.amg_theta,
                                    **kw)
        _hip_sync()
        t1 = time.perf_counter()
        a_create = kernels.alloc_stats(reset=True)
        r = P.solve(rebuild_symbolic=True)
        _hip_sync()
        t2 = time.perf_counter()
        a_solve = kernels.alloc_stats(reset=True)
        n = P.n_nodes
        P.close()
        return {"value": n / (t2 - t1), "unit": "DoF/s", "ms_first_solve": 1e3 * (t2 - t1),
                "ms_create_upload": 1e3 * (t1 - t0), "pcg_iters": r["cg_iters"], "ms_amg_setup": r["ms_amg_setup"],
                "ms_symbolic": r["ms_symbolic"], "ms_assemble": r["ms_assemble"], "ms_solve": r["ms_solve"],
                "hip_malloc_create": a_create["n_malloc"], "hip_malloc_first_solve": a_solve["n_malloc"],
                "ms_hip_malloc_first_solve": a_solve["ms_malloc"]}

    kernels.forget_amg_hints()
    first = one()
    first["note"] = ("fresh problem object, first solve (no re-solve hints, the process's AMG hints dropped "
                     "(xfk_amg_forget_hints), no device blocks of a destroyed problem to reuse: the bench's own "
                     "problem is still alive); ms_create_upload = host -> HBM upload of the mesh and tables "
                     "(outside the step)")
    second = one()
    second["note"] = ("the next fresh problem of the same process (a session's next analysis, the next rotor "
                      "angle): the previous one was destroyed, its device blocks come from the process cache, "
                      "its AMG setup left capacities / MIS rounds / the coarsest plan for a problem of its size, "
                      "taken as speculation checked on the device")
    first["next_problem_in_process"] = second
    return first


def _tag_order(path):
    """Profile tags in the order they were made: r01 < r01b < ... < r03z <
    r03aa < r03ab ... (a longer tag of the same round is a later one)."""
    tag = os.path.basename(path).split("_")[0]
    return (tag[:3], len(tag), tag)


def pmc_traffic(algo_bytes, kernel="k_cg_spmv"):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/*_pmc_summary.json, written by tools/profile.sh from separate
    FETCH_SIZE / WRITE_SIZE rocprofv3 passes of this bench, gfx950-corrected).
    Only a summary of the same workload counts: its traffic must lie within
    [0.8, 2] x this launch's algorithmic bytes."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_summary.json")), key=_tag_order)
    for path in reversed(paths):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if kernel in d and 0.8 * algo_bytes <= d[kernel]["traffic_bytes"] <= 2.0 * algo_bytes:
            return d[kernel]["traffic_bytes"], os.path.relpath(path, ROOT)
    return None, None


# the kernel family each iteration phase launches (xfk_phase_profile names)
PHASE_KERNELS = (("PCG update", ("k_cg_axpy",)), ("sweep", ("k_amg_smooth",)), ("residual", ("k_amg_smooth",)),
                 ("restriction", ("k_csr_mv_tile", "k_csr_mv_g")), ("folded pre", ("k_fold_pre",)),
                 ("dense inverse x b", ("k_dense_mv",)), ("L0 folded post", ("k_fold_post0",)),
                 ("folded post", ("k_csr_mv_tile", "k_csr_mv_g")), ("prolongation", ("k_csr_mv_tile", "k_csr_mv_g")),
                 ("PCG SpMV", ("k_cg_spmv",)))


def _phase_rank(name):
    """Launch order of an iteration phase: update, the V-cycle down (levels
    ascending), the coarsest solve, back up (levels descending), SpMV."""
    import re
    if name.startswith("PCG update"):
        return (0, 0)
    if name.startswith("PCG SpMV"):
        return (9, 0)
    m = re.match(r"L(\d+) ", name)
    lvl = int(m.group(1)) if m else 0
    if "dense" in name:
        return (2, 0)
    if "post" in name or "prolongation" in name:
        return (3, -lvl)
    return (1, lvl)


def annotate_phases(phases):
    """Per-launch rocprof duration, HBM traffic and bound of the iteration
    phases from the newest profiles/*_phase_pmc.json (tools/phase_pmc.py: one
    PCG iteration of the same bench workload in launch order, from a kernel
    trace and separate FETCH_SIZE / WRITE_SIZE passes).  Bound: "cache" when
    the launch moves less than half its algorithmic bytes from HBM (its
    operands sit in L2 / MALL); "hbm" when it does and streams them at >= 30 %
    of the HBM peak; "latency" when it moves its bytes but far below the
    streaming rate (small coarse-level launches at the dependent-launch floor,
    short dependent load chains).  Returns the source file or None."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_phase_pmc.json")), key=_tag_order)
    if not paths:
        return None
    with open(paths[-1]) as f:
        seq = json.load(f).get("sequence", [])
    its = sorted([p for p in phases if p.get("launches_per_iteration", 0) >= 0.5],
                 key=lambda p: _phase_rank(p["phase"]))
    # each launch of the profiled iteration goes to the first phase (in
    # launch-rank order) of its kernel family with launches left: a phase
    # launched k times per iteration (the W level's coarse visits) takes k
    left = [max(1, int(round(p["launches_per_iteration"]))) for p in its]
    if sum(left) != len(seq):
        return None
    fams = [next((k for key, k in PHASE_KERNELS if key in p["phase"]), ()) for p in its]
    got = [[] for _ in its]
    for e in seq:
        q = next((q for q in range(len(its)) if left[q] > 0 and fams[q] and e["kernel"].startswith(fams[q])), None)
        if q is None:
            return None
        left[q] -= 1
        got[q].append(e)
    for ph, es in zip(its, got):
        e = {"rocprof_us": sum(x["rocprof_us"] for x in es) / len(es),
             "traffic_bytes": (sum(x["traffic_bytes"] for x in es) / len(es)
                               if all(x.get("traffic_bytes") is not None for x in es) else None)}
        ph["rocprof_us"] = e["rocprof_us"]
        if ph.get("bytes_per_launch") and e.get("traffic_bytes") is not None:
            ph["traffic_bytes"] = e["traffic_bytes"]
            ph["traffic_over_algorithmic"] = e["traffic_bytes"] / ph["bytes_per_launch"]
            ph["achieved_GBps_rocprof"] = ph["bytes_per_launch"] / (e["rocprof_us"] * 1e-6) / 1e9
            ph["frac_rocprof"] = ph["achieved_GBps_rocprof"] / HBM_PEAK_GBS
            if e["traffic_bytes"] < 0.5 * ph["bytes_per_launch"]:
                ph["bound"] = "cache"
            else:
                ph["bound"] = "hbm" if ph["frac_rocprof"] >= 0.3 else "latency"
    return os.path.relpath(paths[-1], ROOT)


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, argv):
    """`bench.py --gpus N` started without a launcher (no WORLD_SIZE in the
    environment): start the N rank processes here, one per GPU, as torchrun
    would (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR 127.0.0.1 / a free
    MASTER_PORT), before anything in this process touches the GPU -- the
    parent never imports the HIP library, it only waits.  Children are plain
    subprocesses (no exec of a GPU-initialised process).  If one rank fails,
    the others are stopped (their exact PIDs) so no rank waits forever in a
    collective.  Returns the exit code: 0 when every rank succeeded, else the
    first failing rank's code (never 0)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                    "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
        print("[bench] spawned rank %d/%d pid %d" % (r, n, procs[-1].pid), file=sys.stderr, flush=True)
    code = 0
    alive = list(range(n))
    while alive:
        time.sleep(0.2)
        for r in list(alive):
            rc = procs[r].poll()
            if rc is None:
                continue
            alive.remove(r)
            print("[bench] rank %d exited with %d" % (r, rc), file=sys.stderr, flush=True)
            if rc != 0 and code == 0:
                code = rc if rc > 0 else 128 - rc
                for q in alive:          # a failed rank: the others would block in its collectives
                    procs[q].terminate()
                deadline = time.time() + 20
                for q in alive:
                    try:
                        procs[q].wait(timeout=max(0.1, deadline - time.time()))
                    except subprocess.TimeoutExpired:
                        procs[q].kill()
    return code


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) of ONE node; without a launcher's WORLD_SIZE, N > 1 spawns the N rank "
                         "processes itself (default: WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--cells", type=int, default=1000, help="cells per side (2*cells^2 triangles)")
    ap.add_argument("--nonlinear", action="store_true", help="M-19 B-H steel (configs[3])")
    ap.add_argument("--cpu-cells", type=int, default=1000,
                    help="cells per side of the CPU-baseline sample (1000: the GPU line's own 2M-tri mesh)")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the configs[3] (nonlinear M-19) secondary measurement")
    ap.add_argument("--secondary-steps", type=int, default=3)
    ap.add_argument("--no-configs4", action="store_true",
                    help="skip the configs[4] mesh (20M tri) single-GPU secondary measurement")
    ap.add_argument("--precond", choices=["amg", "jacobi"], default="amg",
                    help="device preconditioner of the PCG (the reference uses SSOR)")
    ap.add_argument("--amg-sweeps", type=int, default=1, help="Jacobi sweeps before/after the coarse correction")
    ap.add_argument("--amg-omega", type=float, default=1.75, help="Jacobi weight factor (weight omega / rho)")
    ap.add_argument("--amg-dense", type=int, default=None, help="dense coarsest level of at most this many rows")
    ap.add_argument("--amg-theta", type=float, default=None, help="strength threshold (default 0.08)")
    ap.add_argument("--amg-replicate", type=int, default=None,
                    help="sharded solves: coarse levels of at most this many global rows are replicated")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fsolver", action="store_true", help="skip the FSolver .fem -> .ans end-to-end timing")
    ap.add_argument("--no-phases", action="store_true", help="skip the per-phase table")
    ap.add_argument("--traffic", type=float, default=None,
                    help="HBM bytes per SpMV launch from a PMC pass (profiles/), if measured")
    ap.add_argument("--mode", choices=["sharded", "replicas"], default="sharded",
                    help="N > 1: shard one configs[4] mesh (default) or solve one problem per GPU")
    ap.add_argument("--shard-cells", type=int, default=3162,
                    help="cells per side of the sharded mesh (3162 -> 20M triangles, configs[4])")
    ap.add_argument("--force-sharded", action="store_true",
                    help="run the RCCL sharded path even at N = 1 (plumbing check)")
    ap.add_argument("--local-ranks", type=int, default=0,
                    help="with --force-sharded: R in-process ranks on one GPU (plumbing of the N > 1 line)")
    ap.add_argument("--no-same-mesh-1gpu", action="store_true",
                    help="skip rank 0's single-GPU solve of the sharded mesh")
    args = ap.parse_args()

    if args.force_sharded and args.local_ranks > 1:
        print(json.dumps(local_ranks_run(args)), flush=True)
        return
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus is not None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    if env_world is not None and args.gpus is not None and int(env_world) != args.gpus:
        print("bench.py: --gpus %d does not match the launcher's WORLD_SIZE=%s" % (args.gpus, env_world),
              file=sys.stderr, flush=True)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        print("[bench] rank %d/%d pid %d up (local rank %s)" % (rank, world, os.getpid(),
                                                               os.environ.get("LOCAL_RANK", "0")),
              file=sys.stderr, flush=True)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    cold_process = None
    if world == 1 and not args.no_fsolver and not args.force_sharded:
        cold_process = fsolver_cold_process(args)   # (before this process touches the GPU)
    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: F811
        with stdout_to_stderr():          # gloo's connection banner goes to stdout
            dist.init_process_group("gloo")
    sharded = (world > 1 and args.mode == "sharded") or args.force_sharded

    from xfemm_amd import kernels, synth
    comm = None
    if sharded:
        cells = args.shard_cells if world > 1 else args.cells
        kw = synth.magnetostatic(cells, nonlinear=args.nonlinear)
        uid = kernels.Comm.unique_id() if rank == 0 else None
        if dist is not None:
            box = [uid]
            dist.broadcast_object_list(box, src=0)
            uid = box[0]
        with stdout_to_stderr():
            comm = kernels.Comm.rccl(uid, rank, world, local)
        P = kernels.Static2DProblem(device=local, comm=comm, precond=args.precond, amg_sweeps=args.amg_sweeps,
                                    amg_omega=args.amg_omega, amg_dense=args.amg_dense, amg_theta=args.amg_theta,
                                    amg_replicate=args.amg_replicate, **kw)
        n_dof = P.n_nodes                       # global DoF of the sharded mesh
    else:
        cells = args.cells
        kw = synth.magnetostatic(cells, nonlinear=args.nonlinear)
        P = kernels.Static2DProblem(device=local, precond=args.precond, amg_sweeps=args.amg_sweeps,
                                    amg_omega=args.amg_omega, amg_dense=args.amg_dense, amg_theta=args.amg_theta, **kw)
        n_dof = P.n_nodes

    def barrier():
        _hip_sync()
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        P.solve(rebuild_symbolic=True)
    barrier()
    t0 = time.perf_counter()
    results = []
    for _ in range(args.steps):
        results.append(P.solve(rebuild_symbolic=True, time_spmv=True))
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # roofline of the dominant kernel (the CSR SpMV of the PCG), measured live
    spmv_ms = sum(r["spmv_ms_avg"] * r["spmv_samples"] for r in results) / max(
        1, sum(r["spmv_samples"] for r in results))
    nnz = results[-1]["nnz"]
    rows = P.n_rows
    amg = results[-1]["precond"] == kernels.XFK_PRECOND_AMG
    col_bytes = P.spmv_col_bytes()
    algo = spmv_bytes(rows, nnz, amg, col_bytes)
    achieved = algo / (spmv_ms * 1e-3) / 1e9 if spmv_ms > 0 else 0.0
    ms_step = 1e3 * elapsed / args.steps
    traffic, traffic_src = (args.traffic, "--traffic") if args.traffic is not None else pmc_traffic(algo)
    value = (1 if sharded else world) * n_dof * args.steps / elapsed
    pcg_iters = results[-1]["cg_iters"]

    # per-phase table (outside the timed region): the AMG setup steps and every
    # launch of one PCG iteration, HIP events on the solve stream
    phases = None
    phases_src = None
    if amg and not sharded and world == 1 and not args.no_phases:
        iters = max(1, pcg_iters)
        phases = []
        for ph in P.phase_profile(iters=iters, setup=True):
            setup = ph["name"].startswith("setup")
            row = {"phase": ph["name"], "launches_per_%s" % ("setup" if setup else "iteration"):
                   ph["calls"] if setup else ph["calls"] / iters, "us_per_launch": ph["us_per_call"]}
            if ph["bytes_per_call"] > 0:
                gbs = ph["bytes_per_call"] / (ph["us_per_call"] * 1e-6) / 1e9
                row.update({"bytes_per_launch": ph["bytes_per_call"], "achieved_GBps": gbs,
                            "frac": gbs / HBM_PEAK_GBS, "bound": "unmeasured"})
            phases.append(row)
        phases_src = annotate_phases(phases)

    diagnosis = sharded_diagnosis(P, comm, dist, rank, world) if sharded else None

    same_mesh = None
    if sharded and world > 1 and not args.no_same_mesh_1gpu:
        # strong-scaling reference: rank 0 alone on the same mesh (after the timed region)
        P.close()
        if rank == 0:
            Q = kernels.Static2DProblem(device=local, precond=args.precond, amg_sweeps=args.amg_sweeps,
                                        amg_omega=args.amg_omega, amg_dense=args.amg_dense, amg_theta=args.amg_theta, **kw)
            Q.solve(rebuild_symbolic=True)
            t1 = time.perf_counter()
            r1 = Q.solve(rebuild_symbolic=True)
            _hip_sync()
            dt1 = time.perf_counter() - t1
            Q.close()
            same_mesh = {"one_gpu_dof_s": n_dof / dt1, "one_gpu_ms_per_step": 1e3 * dt1,
                         "one_gpu_pcg_iters": r1["cg_iters"], "speedup": value / (n_dof / dt1)}
        dist.barrier()
    out = {
        "metric": "solved DoF/s (assembly+CG to tol) on 2M-tri magnetostatic",
        "value": value,
        "unit": "DoF/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "strong" if sharded else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {
            "workload": "%s: synthetic %d-tri square-domain magnetostatic, %s, tol %g%s" % (
                "configs[4]" if (sharded or cells == 3162) else (
                    ("configs[3]" if args.nonlinear else "configs[2]") if cells == 1000 else "custom size"),
                2 * cells ** 2,
                "nonlinear M-19 B-H (Newton)" if args.nonlinear else "linear mu",
                kw["precision"], (", row-block sharded over %d GPU(s), RCCL halo + all-reduce" % world)
                if sharded else (", one independent problem per GPU" if world > 1 else "")),
            "triangles": 2 * cells ** 2,
            "dof_total": n_dof * (1 if sharded else world),
            "dof_per_gpu": rows,
            "nnz": nnz,
            "pcg_iters": pcg_iters,
            "ms_per_pcg_iteration": (results[-1]["ms_solve"] - results[-1]["ms_amg_setup"]) / max(1, pcg_iters),
            "newton_iters": results[-1]["newton_iters"],
            "preconditioner": ("smoothed-aggregation AMG V(%d,%d), Jacobi weight %.2f/rho, %d levels, "
                               "operator complexity %.2f"
                               % (args.amg_sweeps, args.amg_sweeps, args.amg_omega, results[-1]["amg_levels"],
                                  results[-1]["amg_op_complexity"])) if amg
                              else "jacobi",
            "pcg": "Chronopoulos-Gear" + (" + AMG V-cycle" if amg else ", 2 launches/iteration"),
            "ms_amg_setup": results[-1]["ms_amg_setup"],
            "ms_symbolic": results[-1]["ms_symbolic"],
            "ms_assemble": results[-1]["ms_assemble"],
            "ms_solve": results[-1]["ms_solve"],
            "parallelism": ("row-block shards x%d (RCCL)" % world) if sharded else (
                "independent problem per GPU (%d)" % world if world > 1 else "single GPU"),
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "k_cg_spmv (CSR SpMV of the PCG, LDS row tiles, fused u.w and r.u partials)",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "algorithmic_bytes_per_launch": algo,
            "column_bytes_per_nonzero": col_bytes,
            "launch_us": spmv_ms * 1e3,
            "launches_sampled": sum(r["spmv_samples"] for r in results),
        },
    }
    if phases is not None:
        it_phases = [p for p in phases if "launches_per_iteration" in p]
        out["roofline"]["phases"] = phases
        out["roofline"]["phases_note"] = (
            "xfk_phase_profile after the timed region: AMG setup rebuilt once, then %d PCG iterations; "
            "us per launch from HIP events; algorithmic bytes per launch (matrix stream 12 B/nnz, 10 with 16-bit tile columns, + 4 B/row, each "
            "vector once); peak %g GB/s; one PCG iteration = %.1f us of phases. rocprof_us, traffic_bytes and "
            "bound: one iteration of the same workload from %s (tools/phase_pmc.py: kernel trace + FETCH_SIZE / "
            "WRITE_SIZE passes; bound 'cache' when traffic < 0.5 x algorithmic bytes, else 'hbm' at >= 30 %% of peak by rocprof duration, 'latency' below)" % (
                max(1, pcg_iters), HBM_PEAK_GBS,
                sum(p["us_per_launch"] * p["launches_per_iteration"] for p in it_phases), phases_src))
    if same_mesh is not None:
        out["config"]["same_mesh_1gpu"] = same_mesh
    if diagnosis is not None:
        out["sharded_diagnosis"] = diagnosis
    if rank == 0 and world == 1 and not sharded:
        out["cold_first_solve"] = cold_first_solve(local, args, kw)
        if not args.no_fsolver:
            out["fsolver_end_to_end"] = fsolver_end_to_end(local, args)
            out["fsolver_cold_process"] = cold_process
    if rank == 0 and world == 1 and not sharded and not args.nonlinear and not args.no_secondary:
        P.close()
        out["secondary"] = [nonlinear_secondary(local, args)]
        if not args.no_configs4:
            out["secondary"].append(configs4_secondary(local, args))
            out["secondary"].append(configs4_rank0_of_8(local, args))
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_cells, args.nonlinear)
    if rank == 0:
        print(json.dumps(out), flush=True)
    P.close()
    if comm is not None:
        comm.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
