# rocprofv3 kernel trace (+ --stats) of the bench, then separate PMC passes
# (FETCH_SIZE, WRITE_SIZE; never combined with tracing domains) over the PCG
# kernels.  Usage: bash tools/profile.sh TAG [extra bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-r01}
shift || true
OUT=gpurun_out/prof_$TAG
REGEX='k_cg_spmv|k_cg_axpy|k_amg_smooth|k_fold_post0|k_fold_pre|k_csr_mv_tile|k_csr_mv_g|k_dense_mv|k_spgemm_sort|k_assemble_rows|k_bgj_multi'
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT/trace -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-fsolver "$@" > $OUT/bench_trace.json 2> $OUT/trace.err && \
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -T -f csv --kernel-include-regex "$REGEX" -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary --no-fsolver "$@" > $OUT/bench_fetch.json 2> $OUT/fetch.err && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -T -f csv --kernel-include-regex "$REGEX" -d $OUT/pmc_write -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary --no-fsolver "$@" > $OUT/bench_write.json 2> $OUT/write.err && \
python3 tools/pmc_summary.py $OUT $(ls -t gpurun_out/calib_*/calib.json profiles/*_pmc_calib.json 2>/dev/null | head -1) > $OUT/pmc_summary.json && \
python3 tools/phase_pmc.py $OUT $(ls -t gpurun_out/calib_*/calib.json profiles/*_pmc_calib.json 2>/dev/null | head -1) > $OUT/phase_pmc.json
