# Lab (round 6): strength threshold of the coarse levels (XFK_AMG_THETA_COARSE;
# level 0 keeps 0.08): bench value, PCG iterations, setup and the dense
# coarsest's Gauss-Jordan per variant, two runs each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for rep in 1 2; do
for t in none 0.06 0.04 0.03 0.02; do
  if [ $t = none ]; then unset XFK_AMG_THETA_COARSE; else export XFK_AMG_THETA_COARSE=$t; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --no-fsolver --steps 20 \
    > gpurun_out/r06_theta_${t}_$rep.json 2> gpurun_out/r06_theta_${t}_$rep.err || exit $?
done
done
unset XFK_AMG_THETA_COARSE
python - <<'PY'
import json
for rep in (1, 2):
    for t in ("none", "0.06", "0.04", "0.03", "0.02"):
        d = json.loads(open("gpurun_out/r06_theta_%s_%d.json" % (t, rep)).read().strip().splitlines()[-1])
        ph = {p["phase"]: p for p in d["roofline"]["phases"]}
        gj = [p for p in d["roofline"]["phases"] if "dense inverse (blocked" in p["phase"]]
        c = d["config"]
        print("theta_coarse %-5s run %d: %.1f M DoF/s %.3f ms  pcg %d  setup %.3f ms  levels %d  GJ %s  cold %.1f M" % (
            t, rep, d["value"] / 1e6, d["ms_per_step"], c["pcg_iters"], c["ms_amg_setup"], d["config"]["preconditioner"].count("levels") and int(c["preconditioner"].split(" levels")[0].split()[-1]),
            ["%.0f us" % p["us_per_launch"] for p in gj], d["cold_first_solve"]["value"] / 1e6))
PY
