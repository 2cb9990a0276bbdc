# Lab (round 6): kernel trace of configs[4] rank 0 of 8 replayed alone
# (bench.configs4_rank0_of_8), then one PCG iteration and the setup of the
# last timed solve from the trace (tools/lab/rank0_iter.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06_rank0
mkdir -p $O
XFK_LAB_WINDOW=1 timeout -k 10 500 rocprofv3 --kernel-trace -T -f csv -d $O/trace -o run -- \
  python3 tools/lab/rank0_probe.py --child --steps 2 > $O/out.json 2> $O/err.log || exit $?
python3 tools/lab/rank0_iter.py $O/trace/run_kernel_trace.csv $O/err.log > gpurun_out/r06_rank0_iter.txt 2>&1
