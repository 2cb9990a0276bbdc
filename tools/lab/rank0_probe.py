"""Lab: configs[4] rank r of R, compute only (bench.configs4_rank0_of_8 with
knobs), under environment variants given as NAME=VALUE[,NAME=VALUE] args.
Each variant runs in a child process (the library reads its switches once).
Usage: python tools/lab/rank0_probe.py [--cells 3162] [--ranks 8] '' XFK_NO_OVERLAP=1 ..."""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def child(cells, ranks, steps):
    sys.path.insert(0, ROOT)
    import bench
    ns = argparse.Namespace(shard_cells=cells, precond="amg", amg_sweeps=1, amg_omega=1.75, amg_dense=None,
                            amg_theta=None, secondary_steps=steps,
                            amg_replicate=int(os.environ["REP"]) if os.environ.get("REP") else None)
    bench.R_OVERRIDE = ranks
    r = bench.configs4_rank0_of_8(0, ns)
    r.pop("workload", None)
    print(json.dumps(r), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=3162)
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("variants", nargs="*")
    a = ap.parse_args()
    if a.child:
        return child(a.cells, a.ranks, a.steps)
    for v in a.variants or [""]:
        env = dict(os.environ)
        for kv in filter(None, v.split(",")):
            k, val = kv.split("=", 1)
            env[k] = val
        p = subprocess.run([sys.executable, __file__, "--child", "--cells", str(a.cells), "--ranks", str(a.ranks),
                            "--steps", str(a.steps)], env=env, capture_output=True, text=True, timeout=600)
        line = p.stdout.strip().splitlines()[-1] if p.stdout.strip() else p.stderr[-2000:]
        print("[%s] %s" % (v or "default", line), flush=True)


if __name__ == "__main__":
    main()
