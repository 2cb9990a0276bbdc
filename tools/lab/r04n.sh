# the determinism tests and the AMG / full-size suites, then the bench (no secondaries)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_amg.py tests/test_gpu_fullsize.py tests/test_gpu_static2d.py tests/test_gpu_harmonic.py -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_r04n.log 2>&1
rc=$?; echo "tests rc=$rc"; fatal $rc
timeout -k 10 400 python bench.py --no-cpu-baseline --no-fsolver --no-secondary > gpurun_out/bench_r04n.json 2> gpurun_out/bench_r04n.err
echo "bench rc=$?"
