# round 5: AMG hints across problems -- AMG tests, the foreign-hint tests, cold-solve bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_amg_foreign.py tests/test_gpu_amg.py tests/test_gpu_memory.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_r05m.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline --no-fsolver > gpurun_out/bench_r05m.json 2> gpurun_out/bench_r05m.err
rc=$?; echo "bench rc=$rc"; fatal $rc
exit $rc
