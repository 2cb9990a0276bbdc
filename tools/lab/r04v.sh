set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) exit $1;; esac; }
XFK_TRACE_CREATE=1 timeout -k 10 300 python tools/lab/cold_probe.py 1000 > gpurun_out/cold_r04v.txt 2>&1
rc=$?; echo "cold rc=$rc"; fatal $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_r04v.log 2>&1
rc=$?; echo "tests rc=$rc"; fatal $rc
timeout -k 10 400 python bench.py --no-cpu-baseline --no-secondary > gpurun_out/bench_r04v.json 2> gpurun_out/bench_r04v.err
echo "bench rc=$?"
