# refold threshold sweep on configs[3] (XFK_REFOLD_MIN), AMG tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_amg.py > gpurun_out/tests_r04z4.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
for v in 0 12 16 20 100000; do
  XFK_TRACE_NEWTON=1 XFK_REFOLD_MIN=$v timeout -k 10 300 python bench.py --nonlinear --steps 3 --warmup 1 --no-cpu-baseline --no-fsolver --no-secondary > gpurun_out/nl_rm${v}_$k.json 2> gpurun_out/nl_rm${v}_$k.err
  rc=$?; echo "min $v $k rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
done
