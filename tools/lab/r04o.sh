# A/B: the pre-round-4-perf build (64b0b3a, in ab_old/) against HEAD, alternating, configs[2] bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) exit $1;; esac; }
for k in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-fsolver --no-secondary > gpurun_out/ab_new_$k.json 2> gpurun_out/ab_new_$k.err
  rc=$?; echo "new $k rc=$rc"; fatal $rc
  (cd ab_old && timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary > ../gpurun_out/ab_old_$k.json 2> ../gpurun_out/ab_old_$k.err)
  rc=$?; echo "old $k rc=$rc"; fatal $rc
done
