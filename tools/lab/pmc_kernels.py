"""Mean PMC counter value per kernel name from rocprofv3 --pmc CSV output dirs.
usage: python tools/lab/pmc_kernels.py DIR [DIR ...]"""
import csv, glob, sys
from collections import defaultdict
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        acc = defaultdict(list)
        for r in csv.DictReader(open(f)):
            acc[(r['Kernel_Name'][:40], r['Counter_Name'])].append(float(r['Counter_Value']))
        for (k, c), v in sorted(acc.items()):
            print("%-40s %-14s n=%4d mean=%.4g" % (k, c, len(v), sum(v) / len(v)))
