# round 5: P = S P_tent row by row (k_ptent_rows) -- AMG tests, then bench A/B against the sort SpGEMM
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r05ag
export TMPDIR=/tmp
O=gpurun_out/r05ag
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_amg.py tests/test_gpu_amg_foreign.py tests/test_gpu_static2d.py tests/test_gpu_fullsize.py tests/test_gpu_memory.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
for v in 1 0 1 0; do
  XFK_PTENT_ROWS=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-fsolver --no-configs4 > $O/bench_pr$v.json 2> $O/bench_pr$v.err
  rc=$?; echo "bench pr$v rc=$rc"; [ $rc -ne 0 ] && exit $rc
  cat $O/bench_pr$v.json >> $O/bench_all.jsonl
done
exit 0
