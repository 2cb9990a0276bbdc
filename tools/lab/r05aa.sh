# round 5: high-priority setup side stream A/B (bench, configs[2]) and the configs[3] Newton trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r05aa
export TMPDIR=/tmp
O=gpurun_out/r05aa
for v in 1 0 1 0; do
  XFK_SIDE_PRIO=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-fsolver --no-configs4 > $O/bench_prio$v.json 2> $O/bench_prio$v.err
  rc=$?; echo "bench prio$v rc=$rc"; [ $rc -ne 0 ] && exit $rc
  cat $O/bench_prio$v.json >> $O/bench_all.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace -T -f csv -d $O/trace -o run -- python3 tools/lab/cold_trace.py > $O/cold_out.txt 2> $O/cold_err.log
rc=$?; echo "cold trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
T=$(ls $O/trace/*/run_kernel_trace.csv $O/trace/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/lab/trace_window.py $T $O/cold_err.log warm > $O/window_warm.txt 2>&1
gzip -f $T
XFK_TRACE_NEWTON=1 timeout -k 10 300 rocprofv3 --kernel-trace -T -f csv -d $O/ntrace -o run -- python3 tools/lab/newton_trace.py > $O/newton_out.txt 2> $O/newton_err.log
rc=$?; echo "newton trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
T=$(ls $O/ntrace/*/run_kernel_trace.csv $O/ntrace/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/lab/trace_window.py $T $O/newton_err.log newton > $O/window_newton.txt 2>&1
gzip -f $T
exit 0
