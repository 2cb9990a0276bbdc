# round 5: local smoothing on sharded levels -- rank 0 of 8 A/B, sharded tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) exit $1;; esac; }
timeout -k 10 500 python tools/lab/rank0_probe.py '' XFK_AMG_HALO_SMOOTH=1 > gpurun_out/rank0_r05l.txt 2>&1
rc=$?; echo "probe rc=$rc"; fatal $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_comm_order.py tests/test_gpu_harmonic_sharded.py tests/test_gpu_configs4.py tests/test_gpu_fsolver_sharded.py tests/test_gpu_memory.py -v --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_r05l.log 2>&1
rc=$?; echo "tests rc=$rc"; fatal $rc
