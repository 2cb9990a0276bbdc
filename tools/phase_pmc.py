"""Per-launch rocprof duration and HBM traffic of one PCG iteration, in launch
order, from the passes of tools/profile.sh (kernel trace + FETCH_SIZE /
WRITE_SIZE PMC runs of bench.py).

An iteration is the run of dispatches from one k_cg_axpy to the next; the
modal kernel sequence is kept (iterations launched after convergence exit at
once and are dropped by their near-zero SpMV traffic).  For every position of
the sequence: the kernel, its grid, the median rocprof duration over the
iterations, and the median FETCH_SIZE / WRITE_SIZE converted to bytes with the
width-calibrated factors of tools/pmc_summary.py.  bench.py matches the
positions to its phase table (roofline.phases): rocprof durations next to the
HIP-event ones, per-level traffic, and the bound of each launch ("cache"
when the traffic is below half the algorithmic bytes, else "hbm" at >= 30 % of
the peak by rocprof duration and "latency" below).

usage: python tools/phase_pmc.py PROFDIR [CALIB.json]
"""
import csv
import glob
import json
import os
import sys
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import MIX, factor  # noqa: E402

ITER_KERNELS = ("k_cg_axpy", "k_amg_smooth", "k_csr_mv_tile", "k_csr_mv_g", "k_fold_pre", "k_dense_mv",
                "k_fold_post0", "k_cg_spmv")


def _rows(pattern):
    out = []
    for path in glob.glob(pattern, recursive=True):
        with open(path) as f:
            out.extend(csv.DictReader(f))
    return out


def iterations(seq):
    """Split a dispatch list (name, ...) at k_cg_axpy; keep the modal sequence."""
    its, cur = [], None
    for d in seq:
        if d[0].startswith("k_cg_axpy"):
            if cur:
                its.append(cur)
            cur = [d]
        elif cur is not None:
            if d[0].startswith(ITER_KERNELS):
                cur.append(d)
            else:        # something else between iterations (setup of a new solve): close
                its.append(cur)
                cur = None
    if cur:
        its.append(cur)
    names = Counter(tuple(x[0] for x in it) for it in its)
    if not names:
        return [], []
    modal = names.most_common(1)[0][0]
    return modal, [it for it in its if tuple(x[0] for x in it) == modal]


def median(v):
    v = sorted(v)
    return v[len(v) // 2] if v else None


def main(prof, calib_path=None):
    cal = None
    if calib_path and os.path.exists(calib_path):
        with open(calib_path) as f:
            cal = json.load(f)
    trace = _rows(os.path.join(prof, "trace", "**", "*kernel_trace.csv"))
    trace.sort(key=lambda r: int(r["Start_Timestamp"]))
    tseq = [(r["Kernel_Name"], int(r["Grid_Size_X"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
            for r in trace]
    modal, its = iterations(tseq)
    out = {"sequence": [], "iterations_traced": len(its)}
    if not its:
        print(json.dumps(out))
        return
    spmv_pos = [k for k, n in enumerate(modal) if n.startswith("k_cg_spmv")]
    # drop the post-convergence iterations (their SpMV exits at once)
    full = median([it[spmv_pos[0]][2] for it in its]) if spmv_pos else None
    if full:
        its = [it for it in its if it[spmv_pos[0]][2] > 0.5 * full]

    def pmc(sub, counter):
        rows = [r for r in _rows(os.path.join(prof, sub, "**", "*counter_collection.csv"))
                if r.get("Counter_Name") == counter]
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
        seq = [(r["Kernel_Name"], int(r["Grid_Size"]), float(r["Counter_Value"]) * 1024.0) for r in rows]
        m, pits = iterations(seq)
        if tuple(m) != tuple(modal):
            return None
        sp = [k for k, n in enumerate(m) if n.startswith("k_cg_spmv")]
        if sp:
            top = median([it[sp[0]][2] for it in pits])
            pits = [it for it in pits if it[sp[0]][2] > 0.5 * top]
        return [median([it[k][2] for it in pits]) for k in range(len(m))]

    fetch = pmc("pmc_fetch", "FETCH_SIZE")
    write = pmc("pmc_write", "WRITE_SIZE")
    for k, name in enumerate(modal):
        base = name.split("<")[0]
        mix = MIX.get(base, {"read": {8: 1.0}, "write": {8: 1.0}})
        ff, fw = factor(cal, "read", mix["read"]), factor(cal, "write", mix["write"])
        if ff is None or fw is None:
            ff, fw = 2.0, 1.0
        e = {"kernel": base, "grid": its[0][k][1], "rocprof_us": median([it[k][2] for it in its])}
        if fetch is not None and write is not None:
            e["traffic_bytes"] = ff * fetch[k] + fw * write[k]
        out["sequence"].append(e)
    out["iterations_traced"] = len(its)
    out["correction"] = ("calibrated per access width (%s)" % os.path.relpath(calib_path)) if cal else \
        "uncalibrated: MI355X_MICROARCH.md 16-B rule (reads x2)"
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
