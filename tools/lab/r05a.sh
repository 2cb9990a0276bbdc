# round 5: arena reuse + advice fixes -- targeted GPU tests, then a quick bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_memory.py tests/test_gpu_amg.py tests/test_gpu_sharded.py tests/test_gpu_newton_ac.py tests/test_gpu_harmonic_sharded.py tests/test_gpu_comm_order.py -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_r05a.log 2>&1
rc=$?; echo "tests rc=$rc"; fatal $rc
timeout -k 10 400 python bench.py --no-cpu-baseline --no-fsolver > gpurun_out/bench_r05a.json 2> gpurun_out/bench_r05a.err
rc=$?; echo "bench rc=$rc"; fatal $rc
