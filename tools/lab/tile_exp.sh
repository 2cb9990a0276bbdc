# V-cycle kernel-shape experiment: the bench under rocprofv3 --stats for
# several XFK_TILE_MIN_ROWS thresholds.  Usage: bash tools/lab/tile_exp.sh T1 T2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
for T in "$@"; do
  export XFK_TILE_MIN_ROWS=$T
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/tile_$T -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary > gpurun_out/tile_$T.json 2> gpurun_out/tile_$T.err || exit $?
done
