# Lab (round 6): kernel trace of the configs[3] step (bench.py --nonlinear):
# the last timed step's kernels by name (busy, gaps) and its Newton passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06_nl
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace -T -f csv -d $O/trace -o run -- \
  python3 bench.py --nonlinear --no-secondary --no-cpu-baseline --no-fsolver --no-phases --steps 3 --warmup 1 \
  > $O/bench.json 2> $O/err.log || exit $?
python3 tools/lab/step_timeline.py $O/trace/run_kernel_trace.csv 2 > gpurun_out/r06_nl_step.txt 2>&1
