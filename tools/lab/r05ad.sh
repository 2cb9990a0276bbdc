# round 5: periodic-map composition on a term pool -- the periodic / air-gap GPU tests and the configs[1] host path
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r05ad /tmp/hp1
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_torque.py tests/test_gpu_age.py tests/test_gpu_antiperiodic_flux.py tests/test_gpu_harmonic.py tests/test_gpu_newton_ac.py tests/test_gpu_static2d.py tests/test_gpu_prev_solution.py tests/test_gpu_fsolver_sharded.py tests/test_gpu_harmonic_sharded.py tests/test_gpu_sharded.py > gpurun_out/r05ad/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
XFK_TRACE_CREATE=1 XFEMM_TRACE_LOAD=1 timeout -k 10 200 python3 tools/lab/host_path.py /tmp/hp1 0 > gpurun_out/r05ad/c1.txt 2>&1
rc=$?; echo "c1 rc=$rc"; exit $rc
