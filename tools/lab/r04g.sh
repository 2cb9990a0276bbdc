set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
XFK_AMG_ABS_STRENGTH=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_antiperiodic_flux.py tests/test_gpu_torque.py -v -s --timeout 150 --timeout-method thread > gpurun_out/iters_abs_r04g.log 2>&1
echo "abs rc=$?"
timeout -k 10 300 python -u -m pytest tests/test_gpu_antiperiodic_flux.py tests/test_gpu_torque.py -v -s --timeout 150 --timeout-method thread > gpurun_out/iters_signed_r04g.log 2>&1
echo "signed rc=$?"
bash tools/gpu_steps.sh r04g tests || exit 1
XFK_TRACE_CREATE=1 XFK_AMG_HINTS_PRINT=1 timeout -k 10 300 python tools/lab/cold_probe.py 1000 300 > gpurun_out/cold_r04g.txt 2>&1 || exit 1
bash tools/gpu_steps.sh r04g benchq
