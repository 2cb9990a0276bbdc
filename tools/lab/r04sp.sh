# A/B: host waits spin (hipDeviceScheduleSpin via XFK_SPIN_WAIT) -- warm and cold lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for k in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-fsolver --no-secondary > gpurun_out/sp_0_$k.json 2> gpurun_out/sp_0_$k.err
  rc=$?; echo "default $k rc=$rc"; [ $rc -eq 0 ] || exit $rc
  XFK_SPIN_WAIT=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-fsolver --no-secondary > gpurun_out/sp_1_$k.json 2> gpurun_out/sp_1_$k.err
  rc=$?; echo "spin $k rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
