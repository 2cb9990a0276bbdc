# Lab (round 6): configs[3] A/B of the Newton residual read at the PCG's
# final poll (XFK_NWS_AT_POLL=1, default) against its own launch + host
# round trip after the solve (=0), alternating, 10 steps each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for k in 1 2 3; do
  for m in 1 0; do
    XFK_NWS_AT_POLL=$m timeout -k 10 300 python bench.py --nonlinear --no-cpu-baseline --no-secondary --no-fsolver \
      --no-phases --steps 10 > gpurun_out/nws_ab_${m}_$k.json 2> gpurun_out/nws_ab_${m}_$k.err || exit $?
  done
done
