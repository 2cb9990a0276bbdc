# GPU pass for one tag: tests, bench, rocprof trace + PMC passes.
# Each step has its own time limit; a step that times out or crashes (124,
# 137, 134, 139) ends the script -- nothing more runs on the GPU after it.
# An ordinary test failure (rc 1) is recorded and the measurement steps still run.
# Usage: bash tools/gpu_steps.sh TAG [tests|bench|prof]...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-r02}
shift || true
STEPS=${*:-tests bench prof}
mkdir -p gpurun_out
fatal() { case $1 in 124|137|134|139) return 0;; *) return 1;; esac; }
for st in $STEPS; do
  case $st in
    tests) timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread \
             > gpurun_out/gpu_tests_$TAG.log 2>&1; rc=$? ;;
    bench) timeout -k 10 500 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; rc=$? ;;
    benchq) timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; rc=$? ;;
    prof) bash tools/profile.sh $TAG; rc=$? ;;
    sharded) timeout -k 10 300 python bench.py --force-sharded --steps 3 --warmup 1 --no-cpu-baseline \
               > gpurun_out/bench_force_sharded_$TAG.json 2> gpurun_out/bench_force_sharded_$TAG.err && \
             timeout -k 10 400 python bench.py --force-sharded --local-ranks 8 --shard-cells 3162 --steps 2 --warmup 1 \
               > gpurun_out/bench_local8_$TAG.json 2> gpurun_out/bench_local8_$TAG.err; rc=$? ;;
    smoke) timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1; rc=$? ;;
    *) echo "unknown step $st"; rc=2 ;;
  esac
  echo "step $st rc=$rc"
  if fatal $rc; then echo "fatal rc $rc in step $st: stopping"; exit $rc; fi
done
