# the round-4 fixes (prev-solution loader, harmonic surrogate strength), then the antiperiodic AMG traces
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_prev_solution.py tests/test_gpu_harmonic.py tests/test_gpu_harmonic_sharded.py -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_r04j.log 2>&1
rc=$?; echo "tests rc=$rc"
case $rc in 124|137|134|139) exit $rc;; esac
XFK_TRACE_NEWTON=1 XFK_AMG_DEBUG=1 timeout -k 10 200 python -u tools/lab/anti_probe.py anti torque > gpurun_out/anti_signed_r04j.txt 2>&1
rc=$?; echo "anti signed rc=$rc"
case $rc in 124|137|134|139) exit $rc;; esac
XFK_AMG_ABS_STRENGTH=1 XFK_TRACE_NEWTON=1 XFK_AMG_DEBUG=1 timeout -k 10 200 python -u tools/lab/anti_probe.py anti torque > gpurun_out/anti_abs_r04j.txt 2>&1
echo "anti abs rc=$?"
