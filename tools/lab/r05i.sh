# round 5: inexact Newton A/B + nonlinear / sharded FSolver tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) exit $1;; esac; }
timeout -k 10 300 python tools/lab/newton_ab.py 1000 > gpurun_out/newton_ab_r05i.txt 2>&1
rc=$?; echo "ab rc=$rc"; fatal $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_fsolver_sharded.py tests/test_gpu_static2d.py tests/test_gpu_fullsize.py tests/test_gpu_amg.py tests/test_gpu_sharded.py tests/test_gpu_antiperiodic_flux.py tests/test_gpu_axisymmetric.py tests/test_gpu_age.py -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_r05i.log 2>&1
rc=$?; echo "tests rc=$rc"; fatal $rc
