# Lab (round 6): the CG SpMV's matrix stream with nontemporal loads
# (XFK_SPMV_NT=1) against plain loads (=0), alternating, configs[2].
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for k in 1 2 3; do
  for m in 0 1; do
    XFK_SPMV_NT=$m timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-fsolver --no-phases \
      --no-configs4 --steps 20 > gpurun_out/nt_ab_${m}_$k.json 2> gpurun_out/nt_ab_${m}_$k.err || exit $?
  done
done
