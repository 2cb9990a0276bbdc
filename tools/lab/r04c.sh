# first setups through the deferred slots: determinism / sharded / full-size tests, bench cold lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_amg.py tests/test_gpu_fullsize.py tests/test_gpu_sharded.py tests/test_gpu_static2d.py tests/test_gpu_torque.py > gpurun_out/tests_r04c.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
for k in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-fsolver --no-secondary > gpurun_out/c_$k.json 2> gpurun_out/c_$k.err
  rc=$?; echo "bench $k rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
