# GPU tests, the RCCL sharded bench path at N = 1, and the 1-GPU configs[4] mesh.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --force-sharded --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_forcesharded.json 2> gpurun_out/bench_forcesharded.err && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err && \
timeout -k 10 600 python bench.py --cells 3162 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_20M_1gpu.json 2> gpurun_out/bench_20M_1gpu.err
