# A/B: kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1), configs[2] bench, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
fatal() { case $1 in 124|137|134|139) exit $1;; esac; }
for k in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-fsolver --no-secondary > gpurun_out/kern_0_$k.json 2> gpurun_out/kern_0_$k.err
  rc=$?; echo "default $k rc=$rc"; fatal $rc
  HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-fsolver --no-secondary > gpurun_out/kern_1_$k.json 2> gpurun_out/kern_1_$k.err
  rc=$?; echo "devkernarg $k rc=$rc"; fatal $rc
done
