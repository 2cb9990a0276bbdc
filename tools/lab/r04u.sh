set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) exit $1;; esac; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_r04u.log 2>&1
rc=$?; echo "tests rc=$rc"; fatal $rc
XFK_TRACE_CREATE=1 XFEMM_TRACE_LOAD=1 timeout -k 10 300 python -u tools/lab/fs_probe.py > gpurun_out/fs_probe_r04u.txt 2>&1
echo "fs probe rc=$?"
