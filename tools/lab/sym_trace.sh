set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/symtrace
mkdir -p $OUT
timeout -k 10 300 python3 tools/lab/sym_probe.py > $OUT/plain.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace -T -f csv -d $OUT/trace -o run -- python3 tools/lab/sym_probe.py > $OUT/traced.log 2>&1 && \
python3 tools/lab/timeline.py $OUT/trace/run_kernel_trace.csv k_count_incidence k_assemble_color 2 > $OUT/timeline.txt
