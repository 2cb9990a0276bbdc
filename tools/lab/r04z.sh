# recorded refold products (k_refold_rec) + planar Newton state pass: targeted GPU tests, configs[3] bench, Newton trace; L0 restriction slots 2/3/4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_amg.py tests/test_gpu_static2d.py tests/test_gpu_antiperiodic_flux.py > gpurun_out/tests_r04z.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  timeout -k 10 300 python bench.py --nonlinear --steps 3 --warmup 1 --no-cpu-baseline --no-fsolver --no-secondary > gpurun_out/nl_z_$k.json 2> gpurun_out/nl_z_$k.err
  rc=$?; echo "nl $k rc=$rc"; [ $rc -eq 0 ] || exit $rc
  XFK_ASM_STATE=0 timeout -k 10 300 python bench.py --nonlinear --steps 3 --warmup 1 --no-cpu-baseline --no-fsolver --no-secondary > gpurun_out/nl_zs_$k.json 2> gpurun_out/nl_zs_$k.err
  rc=$?; echo "nl per-row state $k rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
bash tools/lab/variant_exp.sh r04z XFK_R0_SLOTS "6 4 3 2 6" --no-fsolver --steps 10 --warmup 3 || exit $?
OUT=gpurun_out/prof_r04z
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT/trace -o run -- python3 bench.py --nonlinear --steps 1 --warmup 2 --no-cpu-baseline --no-fsolver --no-secondary --no-phases > $OUT/bench_trace.json 2> $OUT/trace.err
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
T=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python3 tools/lab/newton_tl.py "$T" 6 3 > gpurun_out/newton_tl_r04z.txt 2>&1
echo "tl rc=$?"
rm -f "$T"
