# recorded refold products, capacity 8 + byte offsets: refold/state tests, configs[3] bench, Newton trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_amg.py > gpurun_out/tests_r04z2.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  timeout -k 10 300 python bench.py --nonlinear --steps 3 --warmup 1 --no-cpu-baseline --no-fsolver --no-secondary > gpurun_out/nl_z2_$k.json 2> gpurun_out/nl_z2_$k.err
  rc=$?; echo "nl $k rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
OUT=gpurun_out/prof_r04z2
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT/trace -o run -- python3 bench.py --nonlinear --steps 1 --warmup 2 --no-cpu-baseline --no-fsolver --no-secondary --no-phases > $OUT/bench_trace.json 2> $OUT/trace.err
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
T=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python3 tools/lab/newton_tl.py "$T" 6 3 > gpurun_out/newton_tl_r04z2.txt 2>&1
echo "tl rc=$?"
rm -f "$T"
