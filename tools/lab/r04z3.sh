# PMC: HBM traffic of the Newton-refresh kernels (configs[3])
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/pmc_r04z3
mkdir -p $OUT
REGEX='k_refold|k_planar_state|k_assemble_rows|k_fold_p|k_amg_rho'
for C in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  tag=$(echo $C | cut -d' ' -f1)
  timeout -s KILL 200 rocprofv3 --pmc $C -T -f csv --kernel-include-regex "$REGEX" -d $OUT/$tag -o run -- python3 bench.py --nonlinear --steps 1 --warmup 0 --no-cpu-baseline --no-fsolver --no-secondary --no-phases > $OUT/$tag.json 2> $OUT/$tag.err
  rc=$?; echo "$tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 tools/lab/pmc_kernels.py $OUT/FETCH_SIZE $OUT/WRITE_SIZE $OUT/SQ_WAVES > gpurun_out/pmc_r04z3.txt 2>&1
echo "sum rc=$?"
