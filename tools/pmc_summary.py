"""Per-kernel HBM traffic from the rocprofv3 PMC passes of tools/profile.sh.

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch; on gfx950 FETCH_SIZE counts
wide coalesced reads at half their bytes (MI355X_MICROARCH.md, HBM section),
so it is doubled here.  Prints one JSON object: kernel -> median bytes/launch
(median: the PCG's post-convergence launches exit early and read nothing).
"""
import csv, glob, json, os, sys
from collections import defaultdict


def counter_means(root, counter):
    acc = defaultdict(list)
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                acc[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    med = {k: sorted(v)[len(v) // 2] for k, v in acc.items()}
    return med, {k: len(v) for k, v in acc.items()}


def main(out):
    fetch, nf = counter_means(os.path.join(out, "pmc_fetch"), "FETCH_SIZE")
    write, nw = counter_means(os.path.join(out, "pmc_write"), "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        f = 2.0 * fetch.get(k, 0.0) * 1024.0
        w = write.get(k, 0.0) * 1024.0
        res[k] = {"fetch_bytes_corrected": f, "write_bytes": w, "traffic_bytes": f + w,
                  "launches_fetch": nf.get(k, 0), "launches_write": nw.get(k, 0)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
