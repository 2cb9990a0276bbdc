# round 5: one-wavefront pivot-block inverse -- lab timing, dense-coarsest tests, bench A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 tools/lab/gj_lab > gpurun_out/r05z_gj_lab.txt 2>&1
rc=$?; echo "lab rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_amg.py > gpurun_out/r05z_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-fsolver --no-configs4 > gpurun_out/bench_r05z_wave.json 2> gpurun_out/bench_r05z_wave.err
rc=$?; echo "bench wave rc=$rc"; [ $rc -ne 0 ] && exit $rc
XFK_BGJ_INV=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-fsolver --no-configs4 > gpurun_out/bench_r05z_mfma4.json 2> gpurun_out/bench_r05z_mfma4.err
rc=$?; echo "bench mfma4 rc=$rc"; exit $rc
