# bench (no CPU baseline), full -m gpu suite, antiperiodic trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) exit $1;; esac; }
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_r04m.json 2> gpurun_out/bench_r04m.err
rc=$?; echo "bench rc=$rc"; fatal $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_r04m.log 2>&1
rc=$?; echo "tests rc=$rc"; fatal $rc
XFK_TRACE_NEWTON=1 XFK_AMG_HINTS_PRINT=1 timeout -k 10 200 python -u tools/lab/anti_probe.py anti > gpurun_out/anti_r04m.txt 2>&1
echo "anti rc=$?"
XFK_TRACE_CREATE=1 XFEMM_TRACE_LOAD=1 timeout -k 10 300 python -u tools/lab/fs_probe.py > gpurun_out/fs_probe_r04m.txt 2>&1
echo "fs probe rc=$?"
