# round 5: kernel trace of configs[4] rank 0 of 8 (replay), folded vs unfolded sharded post-step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp XFK_LAB_WINDOW=1
for v in fold nofold; do
  if [ $v = nofold ]; then export XFK_AMG_FOLD_DIST=0; fi
  O=gpurun_out/r05r_$v
  mkdir -p $O
  timeout -k 10 400 rocprofv3 --kernel-trace -T -f csv -d $O/trace -o run -- python3 tools/lab/rank0_probe.py --child --cells 3162 --ranks 8 --steps 3 > $O/out.json 2> $O/err.log
  rc=$?; echo "$v rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  python3 tools/lab/trace_window.py $(ls $O/trace/*/run_kernel_trace.csv $O/trace/run_kernel_trace.csv 2>/dev/null | head -1) $O/err.log > $O/window.txt 2>&1
  gzip -f $(ls $O/trace/*/run_kernel_trace.csv $O/trace/run_kernel_trace.csv 2>/dev/null | head -1)
done
exit 0
