# V-cycle kernel-shape experiment: bench phases for several env settings.
# Usage: bash tools/lab/shape_exp.sh "ENV=.. ENV2=.." "..." ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
k=0
for cfg in "$@"; do
  k=$((k+1))
  env $cfg timeout -k 10 120 python bench.py --no-cpu-baseline --no-secondary --steps 3 > gpurun_out/shape_$k.json 2> gpurun_out/shape_$k.err || exit $?
  echo "$k $cfg" >> gpurun_out/shape_index.txt
done
