"""Per-kernel HBM traffic from the rocprofv3 PMC passes of tools/profile.sh.

FETCH_SIZE and WRITE_SIZE are KiB per dispatch.  MI355X_MICROARCH.md
calibrates only wide (16 B / lane) coalesced reads on gfx950 (FETCH_SIZE = half
their bytes); the fsolver kernels read 4-B ints and 8-B doubles.  So the
conversion to bytes is CALIBRATED per access width on known-byte kernels
(tools/pmc_calib.hip, run by tools/pmc_calib.sh):

    factor_w = bytes streamed / (counter * 1024)        w = 4, 8, 16 B / lane

and a kernel whose algorithmic bytes split by width as phi_w converts as
    bytes = counter * 1024 / sum_w (phi_w / factor_w).
The width mixes of the measured kernels are stated in MIX below (from their
code); kernels without a mix use the 8-B factor.  Without a calibration file
the guide's 16-B rule (x2 reads, x1 writes) is applied and flagged.

Usage:
    python tools/pmc_summary.py --calib DIR           -> calibration JSON (factors)
    python tools/pmc_summary.py PROFDIR [CALIB.json]  -> kernel -> bytes / launch
(median over launches: the PCG's post-convergence launches exit early and
read nothing).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

# read / write byte fractions by access width (B / lane) of each kernel
MIX = {
    # k_cg_spmv: col 4 B + val 8 B per nonzero, rowptr 4 B per row, u (+ r) 8 B; w 8 B written
    "k_cg_spmv": {"read": {4: 0.30, 8: 0.70}, "write": {8: 1.0}},
    # k_cg_axpy (AMG mode): double2 loads / stores of w, z, p, x, r, u
    "k_cg_axpy": {"read": {16: 1.0}, "write": {16: 1.0}},
    # smoother / CSR tile kernels: as the SpMV
    "k_amg_smooth": {"read": {4: 0.30, 8: 0.70}, "write": {8: 1.0}},
    "k_csr_mv_tile": {"read": {4: 0.30, 8: 0.70}, "write": {8: 1.0}},
    # dense coarsest apply: 16-B loads of the f32 inverse rows (and of b)
    "k_dense_mv": {"read": {16: 1.0}, "write": {8: 1.0}},
}

CALIB_KERNELS = {  # name fragment -> (direction, width)
    "k_calib_read<int>": ("read", 4), "k_calib_read<double>": ("read", 8),
    "k_calib_read<HIP_vector_type<double, 2u> >": ("read", 16),
    "k_calib_write<int>": ("write", 4), "k_calib_write<double>": ("write", 8),
    "k_calib_write<HIP_vector_type<double, 2u> >": ("write", 16),
}


def counter_values(root, counter):
    acc = defaultdict(list)
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") == counter:
                    acc[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return acc


def median(v):
    return sorted(v)[len(v) // 2]


def calibrate(root):
    """Factors bytes / (counter KiB * 1024) per (direction, width)."""
    with open(os.path.join(root, "fetch.log")) as f:
        txt = f.read()
    i = txt.index('{"bytes_per_launch"')
    known = json.loads(txt[i:txt.index("}", i) + 1])["bytes_per_launch"]
    out = {"bytes_per_launch": known, "read": {}, "write": {}, "kernels": {}}
    for sub, counter in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        for name, vals in counter_values(os.path.join(root, sub), counter).items():
            for frag, (direction, w) in CALIB_KERNELS.items():
                want = "read" if counter == "FETCH_SIZE" else "write"
                if frag in name and direction == want:
                    m = median(vals) * 1024.0
                    out[direction][str(w)] = known / m if m > 0 else None
                    out["kernels"][frag] = {"counter_bytes": m, "launches": len(vals)}
    return out


def factor(cal, direction, mix):
    inv = 0.0
    for w, phi in mix.items():
        f = cal[direction].get(str(w)) if cal else None
        if f is None:
            return None
        inv += phi / f
    return 1.0 / inv


def main(prof, calib_path=None):
    cal = None
    if calib_path and os.path.exists(calib_path):
        with open(calib_path) as f:
            cal = json.load(f)
    fetch = counter_values(os.path.join(prof, "pmc_fetch"), "FETCH_SIZE")
    write = counter_values(os.path.join(prof, "pmc_write"), "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        mix = MIX.get(k, {"read": {8: 1.0}, "write": {8: 1.0}})
        fr = median(fetch[k]) * 1024.0 if k in fetch else 0.0
        wr = median(write[k]) * 1024.0 if k in write else 0.0
        ff, fw = factor(cal, "read", mix["read"]), factor(cal, "write", mix["write"])
        if ff is None or fw is None:
            ff, fw, how = 2.0, 1.0, "uncalibrated: MI355X_MICROARCH.md 16-B rule (reads x2)"
        else:
            how = "calibrated per access width (%s)" % os.path.relpath(calib_path)
        res[k] = {"fetch_counter_bytes": fr, "write_counter_bytes": wr, "fetch_bytes_corrected": ff * fr,
                  "write_bytes": fw * wr, "traffic_bytes": ff * fr + fw * wr, "correction": how,
                  "read_factor": ff, "write_factor": fw,
                  "launches_fetch": len(fetch.get(k, ())), "launches_write": len(write.get(k, ()))}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "--calib":
        print(json.dumps(calibrate(sys.argv[2]), indent=1))
    else:
        main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
