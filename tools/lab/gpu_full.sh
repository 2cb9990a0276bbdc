# Full GPU pass: gpu tests, default bench (with CPU baseline), rocprof trace + PMC passes.
# Usage: bash tools/lab/gpu_full.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
bash tools/profile.sh $TAG
