# Lab (round 6): the level-0 restriction with the LDS window of r' (XFK_R0_WIN
# 0 = tile kernel, 1/2/3 = window variants): bench phases per variant and the
# solution's bits against the tile kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for m in 0 1 2 3; do
  XFK_R0_WIN=$m timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --no-fsolver --steps 10 \
    > gpurun_out/r06_rwin_$m.json 2> gpurun_out/r06_rwin_$m.err || exit $?
  XFK_R0_WIN=$m timeout -k 10 200 python tools/lab/solve_dump.py gpurun_out/r06_rwin_A_$m.npy || exit $?
done
python - <<'PY'
import json, numpy as np
a0 = np.load("gpurun_out/r06_rwin_A_0.npy")
for m in range(4):
    d = json.loads(open("gpurun_out/r06_rwin_%d.json" % m).read().strip().splitlines()[-1])
    ph = {p["phase"]: p for p in d["roofline"]["phases"]}
    r = ph.get("L0 restriction R r", {})
    a = np.load("gpurun_out/r06_rwin_A_%d.npy" % m)
    print("XFK_R0_WIN=%d  %.1f M DoF/s  %.3f ms/step  pcg %d  restriction %.2f us  bit-identical %s" % (
        m, d["value"] / 1e6, d["ms_per_step"], d["config"]["pcg_iters"], r.get("us_per_launch", -1),
        bool(np.array_equal(a, a0))))
PY
