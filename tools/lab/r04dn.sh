# dense coarsest size A/B (--amg-dense) with today's W-cycle: bench lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for k in 1 2; do
for v in 2048 1024 512 256; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-fsolver --no-secondary --amg-dense $v > gpurun_out/dn_${v}_$k.json 2> gpurun_out/dn_${v}_$k.err
  rc=$?; echo "dense $v $k rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
done
