# round 5: sharded Newton AC and Case-2 circuits
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_harmonic_sharded.py tests/test_gpu_newton_ac.py tests/test_gpu_harmonic.py tests/test_gpu_fsolver_sharded.py tests/test_gpu_memory.py -v -s --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_r05n.log 2>&1
rc=$?; echo "tests rc=$rc"; exit $rc
