cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/exp2
timeout -k 10 120 python tools/lab/spmv_lab.py > gpurun_out/exp2/spmv_lab.txt 2>&1
