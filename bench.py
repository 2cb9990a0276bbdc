"""Bench: solved DoF/s of the fsolver static-2D hot path on MI355X.

One step = FSolver::Static2D from a device-resident mesh: symbolic phase (CSR
pattern, element colouring, BC maps), element assembly, boundary conditions
and the PCG solve to the problem's Precision (1e-8), plus the Newton loop for
nonlinear problems.  Inputs (mesh + property tables) are uploaded before the
timed region.

N = 1 workload: BASELINE configs[2], synthetic 2M-triangle square-domain
magnetostatic problem with linear mu (1000 x 1000 cells -> 2,000,000
triangles, 1,002,001 nodes), synthetic data.

N > 1 (one process per GPU, torchrun): every rank solves its own instance of
the same problem (an independent-problem sweep, e.g. rotor positions): no
data-path collective, "scaling": "weak".  The host barrier / max-over-ranks
uses torch.distributed (gloo) on scalars only.

Output: one JSON line (rank 0) with roofline (SpMV kernel, HIP-event timing
inside the timed region) and cpu_baseline (reference spars.cpp via oracle/_ref,
single core, bounded sample).
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def _hip_sync():
    lib = ctypes.CDLL("libamdhip64.so")
    lib.hipDeviceSynchronize()


def spmv_bytes(n_rows, nnz):
    """Algorithmic HBM bytes of one CSR SpMV launch of the PCG (k_cg_spmv,
    xfemm_amd/csrc/xfk_pcg.hip): val 8 B + col 4 B per nonzero, rowptr 4 B per
    row (+1), u read once 8 B per row, w written 8 B per row (the fused u.w
    partial re-reads u from cache)."""
    return 12 * nnz + 4 * (n_rows + 1) + 16 * n_rows


def cpu_baseline(n_cells, nonlinear):
    """Reference CPU solver on a bounded sample of the same workload family:
    the reference's own CBigLinProb (spars.cpp: linked-list matrix, SSOR-PCG,
    SetValue) compiled into oracle/_ref, driven by the restated Static2D
    element loop (oracle/static2d_oracle.c).  Single thread."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle import oracle
    from util import synth_to_oracle
    from xfemm_amd import synth
    kind = "reference" if oracle.ref_available() else "port"
    kw = synth.magnetostatic(n_cells, nonlinear=nonlinear)
    pr, mesh, _ = synth_to_oracle(kw)
    # the reference's PCGSolve printf()s to stdout: keep stdout for the JSON line
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        t0 = time.perf_counter()
        _, st, _ = oracle.solve(pr, mesh, "reference" if kind == "reference" else "oracle")
        dt = time.perf_counter() - t0
    finally:
        os.dup2(saved, 1)
        os.close(saved)
    dof = len(mesh.x)
    return {
        "value": dof / dt,
        "unit": "DoF/s",
        "cores": 1,
        "kind": kind,
        "sample": "%dx%d-cell square (%d tri, %d DoF)%s: full Static2D (assembly + SSOR-PCG to 1e-8, %d PCG iters) "
                  "in %.1f s; smaller than the GPU workload, so fewer iterations per DoF (favours the CPU)"
                  % (n_cells, n_cells, 2 * n_cells * n_cells, dof, " M-19" if nonlinear else "",
                     st["cg_iters"] if st["cg_iters"] >= 0 else -1, dt),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cells", type=int, default=1000, help="cells per side (2*cells^2 triangles)")
    ap.add_argument("--nonlinear", action="store_true", help="M-19 B-H steel (configs[3])")
    ap.add_argument("--cpu-cells", type=int, default=500)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic", type=float, default=None,
                    help="HBM bytes per SpMV launch from a PMC pass (profiles/), if measured")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: F811
        dist.init_process_group("gloo")

    from xfemm_amd import kernels, synth
    kw = synth.magnetostatic(args.cells, nonlinear=args.nonlinear)
    P = kernels.Static2DProblem(device=local, **kw)
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
    algo = spmv_bytes(n_dof, nnz)
    achieved = algo / (spmv_ms * 1e-3) / 1e9 if spmv_ms > 0 else 0.0
    ms_step = 1e3 * elapsed / args.steps
    value = world * n_dof * args.steps / elapsed
    out = {
        "metric": "solved DoF/s (assembly+CG to tol) on 2M-tri magnetostatic",
        "value": value,
        "unit": "DoF/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {
            "workload": "configs[%d]: synthetic %d-tri square-domain magnetostatic, %s, tol %g%s" % (
                3 if args.nonlinear else 2, 2 * args.cells ** 2,
                "nonlinear M-19 B-H (Newton)" if args.nonlinear else "linear mu",
                kw["precision"], ", one independent problem per GPU" if world > 1 else ""),
            "triangles": 2 * args.cells ** 2,
            "dof_per_gpu": n_dof,
            "nnz": nnz,
            "pcg_iters": results[-1]["cg_iters"],
            "newton_iters": results[-1]["newton_iters"],
            "preconditioner": "jacobi", "pcg": "Chronopoulos-Gear, 2 launches/iteration",
            "ms_symbolic": results[-1]["ms_symbolic"],
            "ms_assemble": results[-1]["ms_assemble"],
            "ms_solve": results[-1]["ms_solve"],
            "parallelism": "independent problem per GPU (%d)" % world if world > 1 else "single GPU",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "k_cg_spmv (CSR SpMV of the PCG, LDS row tiles, fused u.w partial)",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": args.traffic,
            "algorithmic_bytes_per_launch": algo,
            "launch_us": spmv_ms * 1e3,
            "launches_sampled": sum(r["spmv_samples"] for r in results),
        },
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_cells, args.nonlinear)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
