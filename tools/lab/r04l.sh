# bench (no CPU baseline) + cold probe, then the r04h experiments
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_r04l.json 2> gpurun_out/bench_r04l.err
rc=$?; echo "bench rc=$rc"
case $rc in 124|137|134|139) exit $rc;; esac
XFK_TRACE_CREATE=1 timeout -k 10 300 python tools/lab/cold_probe.py 1000 > gpurun_out/cold_r04l.txt 2>&1
rc=$?; echo "cold rc=$rc"
case $rc in 124|137|134|139) exit $rc;; esac
bash tools/lab/r04h.sh
