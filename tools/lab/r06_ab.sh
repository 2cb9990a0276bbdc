# Lab (round 6): A/B of env switches on the N = 1 bench (configs[2]); each
# argument is one variant: "base" or space-separated VAR=value settings.
# Two passes over the variants; a summary table at the end.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab
STEPS=${AB_STEPS:-20}
EXTRA=${AB_EXTRA:---no-cpu-baseline --no-secondary --no-fsolver}
i=0
for rep in 1 2; do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    if [ "$v" = base ]; then envs=""; else envs="$v"; fi
    env $envs timeout -k 10 300 python bench.py $EXTRA --steps $STEPS > gpurun_out/ab/v${i}_$rep.json 2> gpurun_out/ab/v${i}_$rep.err || exit $?
    echo "$v" > gpurun_out/ab/v${i}.name
  done
done
python - "$#" <<'PY'
import json, sys
n = int(sys.argv[1])
for i in range(1, n + 1):
    name = open("gpurun_out/ab/v%d.name" % i).read().strip()
    for rep in (1, 2):
        d = json.loads(open("gpurun_out/ab/v%d_%d.json" % (i, rep)).read().strip().splitlines()[-1])
        c = d["config"]
        gj = [p["us_per_launch"] for p in d["roofline"].get("phases", []) if "dense inverse (blocked" in p["phase"]]
        mis = sum(p["us_per_launch"] for p in d["roofline"].get("phases", []) if "MIS-2" in p["phase"])
        sec = d.get("secondary", [])
        s3 = (" | c3 %.1f M (%d pcg)" % (sec[0]["value"] / 1e6, sec[0]["pcg_iters"])) if sec else ""
        print("%-40s run %d: %.1f M DoF/s %.3f ms pcg %d setup %.3f ms %s GJ %s MIS %.0f us cold %.1f M%s" % (
            name[:40], rep, d["value"] / 1e6, d["ms_per_step"], c["pcg_iters"], c["ms_amg_setup"],
            c["preconditioner"].split(",")[2].strip() if "," in c["preconditioner"] else "",
            ["%.0f" % g for g in gj], mis, d["cold_first_solve"]["value"] / 1e6, s3))
PY
