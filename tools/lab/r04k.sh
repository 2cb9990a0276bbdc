# full -m gpu suite (no -x), the antiperiodic trace, then the quick bench (fsolver end-to-end, rank-0-of-8)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_r04k.log 2>&1
rc=$?; echo "tests rc=$rc"
case $rc in 124|137|134|139) exit $rc;; esac
XFK_TRACE_NEWTON=1 timeout -k 10 200 python -u tools/lab/anti_probe.py anti > gpurun_out/anti_r04k.txt 2>&1
rc=$?; echo "anti rc=$rc"
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_r04k.json 2> gpurun_out/bench_r04k.err
echo "bench rc=$?"
XFK_TRACE_CREATE=1 timeout -k 10 300 python tools/lab/cold_probe.py 1000 > gpurun_out/cold_r04k.txt 2>&1
echo "cold rc=$?"
