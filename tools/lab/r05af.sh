# round 5: row-gather assembly with the element pipeline -- tests, then bench A/B (configs[2] + configs[3])
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r05af
export TMPDIR=/tmp
O=gpurun_out/r05af
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_static2d.py tests/test_gpu_fullsize.py tests/test_gpu_axisymmetric.py tests/test_gpu_magdir.py tests/test_gpu_torque.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
for v in 1 0 1 0; do
  XFK_ASM_PIPE=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-fsolver --no-configs4 > $O/bench_pipe$v.json 2> $O/bench_pipe$v.err
  rc=$?; echo "bench pipe$v rc=$rc"; [ $rc -ne 0 ] && exit $rc
  cat $O/bench_pipe$v.json >> $O/bench_all.jsonl
done
exit 0
