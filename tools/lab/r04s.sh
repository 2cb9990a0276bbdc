# the default bench (CPU baseline, FSolver end-to-end, secondaries)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_r04s.json 2> gpurun_out/bench_r04s.err
echo "bench rc=$?"
