cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/exp1
for d in 2048 1024 512 256; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-secondary --steps 5 --amg-dense $d > gpurun_out/exp1/dense_$d.json 2>gpurun_out/exp1/dense_$d.err || exit $?
done
XFK_SPIN_WAIT=1 timeout -k 10 120 python bench.py --no-cpu-baseline --no-secondary --steps 5 > gpurun_out/exp1/spin.json 2>gpurun_out/exp1/spin.err || exit $?
bash tools/pmc_calib.sh r02e
timeout -k 10 120 python tools/lab/spmv_lab.py > gpurun_out/exp1/spmv_lab.txt 2>&1
