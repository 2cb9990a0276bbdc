# Lab (round 6): configs[2] A/B of one environment switch, alternating,
# 3 x 2 runs of 20 steps.  Usage: bash tools/lab/r06_env_ab.sh VAR A B TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
V=$1; A=$2; B=$3; T=$4
for k in 1 2 3; do
  for m in $A $B; do
    env $V=$m timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --no-fsolver \
      --no-phases --steps 20 > gpurun_out/${T}_${m}_$k.json 2> gpurun_out/${T}_${m}_$k.err || exit $?
  done
done
