# round 5: kernel trace of a configs[3] solve (Newton passes, host gaps)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r05y
export TMPDIR=/tmp XFK_TRACE_NEWTON=1
O=gpurun_out/r05y
timeout -k 10 300 rocprofv3 --kernel-trace -T -f csv -d $O/trace -o run -- python3 tools/lab/newton_trace.py > $O/out.txt 2> $O/err.log
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
T=$(ls $O/trace/*/run_kernel_trace.csv $O/trace/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/lab/trace_window.py $T $O/err.log newton > $O/window.txt 2>&1
gzip -f $T
exit 0
