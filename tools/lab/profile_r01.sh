# rocprofv3 kernel trace + separate PMC passes (FETCH_SIZE, WRITE_SIZE) of the bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_r01
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT/trace -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_trace.json 2> $OUT/trace.err && \
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -T -f csv --kernel-include-regex k_pcg_spmv -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/bench_fetch.json 2> $OUT/fetch.err && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -T -f csv --kernel-include-regex k_pcg_spmv -d $OUT/pmc_write -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/bench_write.json 2> $OUT/write.err
echo "profile rc=$?" >> $OUT/trace.err
find $OUT -name "*.csv" | head -20 > $OUT/files.txt
