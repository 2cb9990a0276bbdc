# cold setup timeline after the deferred first-setup lengths (gaps > 3 us, per-kernel totals)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/lab/trace_only.sh r04ct --no-fsolver
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
T=$(find gpurun_out/prof_r04ct/trace -name "*kernel_trace.csv" | head -1)
python3 tools/lab/setup_tl.py "$T" -2 --gaps > gpurun_out/setup_tl_cold_r04ct.txt 2>&1
python3 tools/lab/setup_tl.py "$T" -1 --gaps > gpurun_out/setup_tl_next_r04ct.txt 2>&1
python3 tools/lab/setup_tl.py "$T" --gaps > gpurun_out/setup_tl_warm_r04ct.txt 2>&1
echo "tl rc=$?"
rm -f "$T"
