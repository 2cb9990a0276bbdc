# determinism / AMG / full-size tests, then the A/B against the pre-round-4 build, then the cold probe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_amg.py tests/test_gpu_fullsize.py tests/test_gpu_static2d.py -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_r04q.log 2>&1
rc=$?; echo "tests rc=$rc"; fatal $rc
bash tools/lab/r04o.sh || exit $?
XFK_TRACE_CREATE=1 XFK_AMG_HINTS_PRINT=1 timeout -k 10 300 python tools/lab/cold_probe.py 1000 > gpurun_out/cold_r04q.txt 2>&1
echo "cold rc=$?"
