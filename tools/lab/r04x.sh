# configs[3] (nonlinear M-19): Newton pass trace and a kernel timeline per pass
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
XFK_TRACE_NEWTON=1 timeout -k 10 300 python bench.py --nonlinear --steps 2 --warmup 1 --no-cpu-baseline --no-fsolver --no-secondary > gpurun_out/nl_r04x.json 2> gpurun_out/nl_r04x.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/prof_r04x
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT/trace -o run -- python3 bench.py --nonlinear --steps 1 --warmup 1 --no-cpu-baseline --no-fsolver --no-secondary --no-phases > $OUT/bench_trace.json 2> $OUT/trace.err
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
T=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python3 tools/lab/newton_tl.py "$T" 6 > gpurun_out/newton_tl_r04x.txt 2>&1
echo "tl rc=$?"
rm -f "$T"
