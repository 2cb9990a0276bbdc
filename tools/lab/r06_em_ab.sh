# Lab (round 6): planar Newton passes with the element matrices evaluated once
# per element (XFK_ASM_EM=1, k_planar_elem + k_assemble_rows_em) against the
# rows' own evaluation (=0, k_planar_state + k_assemble_rows_pre): the answers
# (bitwise), then configs[3] bench lines alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for m in 0 1; do
  XFK_ASM_EM=$m timeout -k 10 120 python tools/lab/em_dump.py gpurun_out/em_A_$m.npy 300 || exit $?
done
python -c "import numpy as np; a=np.load('gpurun_out/em_A_0.npy'); b=np.load('gpurun_out/em_A_1.npy'); print('bitwise equal:', np.array_equal(a.view(np.int64), b.view(np.int64)), 'max rel diff', float(np.abs(a-b).max()/np.abs(a).max()))"
for k in 1 2 3; do
  for m in 0 1; do
    XFK_ASM_EM=$m timeout -k 10 300 python bench.py --nonlinear --no-cpu-baseline --no-secondary --no-fsolver \
      --no-phases --steps 10 > gpurun_out/em_ab_${m}_$k.json 2> gpurun_out/em_ab_${m}_$k.err || exit $?
  done
done
