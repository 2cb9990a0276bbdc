"""Lab: bench.fsolver_end_to_end (configs[1] TorqueBenchmark refined, configs[2]
square) with the creation / load traces on (run with XFK_TRACE_CREATE=1
XFEMM_TRACE_LOAD=1).  Usage: python tools/lab/fs_probe.py [cells]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

cells = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
for rec in bench.fsolver_end_to_end(0, argparse.Namespace(cells=cells)):
    print(json.dumps(rec), flush=True)
