# A/B: level-0 restriction tile rows (configs[2] bench phases); rank 0 of 8 with / without
# the sharded f32 transfers; rank-0 kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/lab/variant_exp.sh r04h XFK_R0_TILE "256 128 64" --no-fsolver --steps 10 --warmup 3 || exit 1
timeout -k 10 500 python tools/lab/rank0_probe.py '' XFK_AMG_F32=0 > gpurun_out/rank0_f32_r04h.txt 2>&1
rc=$?; echo "rank0 f32 A/B rc=$rc"
case $rc in 124|137|134|139) exit $rc;; esac
XFK_AMG_DEBUG=1 timeout -k 10 120 python tools/lab/amg_probe.py 1000 --no-jacobi > gpurun_out/amgdebug_r04h.txt 2>&1
echo "amg debug rc=$?"
# rank 0 of 8 (configs[4]) replayed alone: kernel time per solve inside the timed window
XFK_LAB_WINDOW=1 timeout -k 10 500 rocprofv3 --kernel-trace -T -f csv -d gpurun_out/prof_rank0_r04h -o run -- python3 tools/lab/rank0_probe.py --child --steps 3 > gpurun_out/rank0_trace_r04h.log 2>&1
echo "rank0 trace rc=$?"
T=$(find gpurun_out/prof_rank0_r04h -name "*kernel_trace.csv" | head -1)
python3 tools/lab/trace_window.py "$T" gpurun_out/rank0_trace_r04h.log rank0 > gpurun_out/rank0_window_r04h.txt 2>&1
rm -f "$T"
# warm setup timeline (kernel trace of a short bench run): gaps between kernels
bash tools/lab/trace_only.sh r04h --no-fsolver
echo "trace rc=$?"
T=$(find gpurun_out/prof_r04h/trace -name "*kernel_trace.csv" | head -1)
python3 tools/lab/setup_tl.py "$T" --gaps > gpurun_out/setup_tl_r04h.txt 2>&1
python3 tools/lab/setup_tl.py "$T" > gpurun_out/setup_tl_full_r04h.txt 2>&1
echo "tl rc=$?"
