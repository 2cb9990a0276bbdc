# GPU tests + parity/timing probe; stops at the first failing step.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python tools/lab/gpu_probe.py > gpurun_out/probe.log 2>&1
