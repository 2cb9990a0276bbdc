# rocprofv3 kernel trace of a short bench run (no PMC), for setup timelines.
# usage: bash tools/lab/trace_only.sh TAG [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT/trace -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-configs4 --no-phases "$@" > $OUT/bench_trace.json 2> $OUT/trace.err
