# round 5: full -m gpu suite, smoke, default bench, rocprof trace + PMC passes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) exit $1;; esac; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_r05j.log 2>&1
rc=$?; echo "tests rc=$rc"; fatal $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r05j.log 2>&1
rc=$?; echo "smoke rc=$rc"; fatal $rc
timeout -k 10 500 python bench.py > gpurun_out/bench_r05j.json 2> gpurun_out/bench_r05j.err
rc=$?; echo "bench rc=$rc"; fatal $rc
bash tools/profile.sh r05j --no-fsolver
echo "prof rc=$?"
