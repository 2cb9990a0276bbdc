# round 5: kernel trace of the configs[2] cold first solve vs the repeated solve
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r05w
export TMPDIR=/tmp
O=gpurun_out/r05w
timeout -k 10 300 rocprofv3 --kernel-trace -T -f csv -d $O/trace -o run -- python3 tools/lab/cold_trace.py > $O/out.txt 2> $O/err.log
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
T=$(ls $O/trace/*/run_kernel_trace.csv $O/trace/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/lab/trace_window.py $T $O/err.log cold > $O/window_cold.txt 2>&1
python3 tools/lab/trace_window.py $T $O/err.log warm > $O/window_warm.txt 2>&1
gzip -f $T
exit 0
