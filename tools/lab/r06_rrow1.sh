# Lab (round 6): the level-0 restriction with one lane per row (XFK_R0_ROW1=1)
# against the tile kernel: bench phases and the solution's bits.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for m in 0 1 0 1; do
  XFK_R0_ROW1=$m timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --no-fsolver --steps 20 \
    > gpurun_out/r06_rrow1_$m.json 2> gpurun_out/r06_rrow1_$m.err || exit $?
  XFK_R0_ROW1=$m timeout -k 10 200 python tools/lab/solve_dump.py gpurun_out/r06_rrow1_A_$m.npy || exit $?
  python - $m <<'PY'
import json, sys, numpy as np
m = sys.argv[1]
d = json.loads(open("gpurun_out/r06_rrow1_%s.json" % m).read().strip().splitlines()[-1])
ph = {p["phase"]: p for p in d["roofline"]["phases"]}
same = bool(np.array_equal(np.load("gpurun_out/r06_rrow1_A_0.npy"), np.load("gpurun_out/r06_rrow1_A_%s.npy" % m)))
print("XFK_R0_ROW1=%s  %.1f M DoF/s  %.3f ms  pcg %d  restriction %.2f us  bits equal %s" % (
    m, d["value"] / 1e6, d["ms_per_step"], d["config"]["pcg_iters"], ph["L0 restriction R r"]["us_per_launch"], same))
PY
done
