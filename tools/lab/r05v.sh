# round 5: the fused W tail -- bit identity, AMG tests, then the bench with and without it
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_amg.py -k "fused_w_tail or deterministic or w_cycle or folded" > gpurun_out/r05v_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-fsolver --no-configs4 > gpurun_out/bench_r05v_fused.json 2> gpurun_out/bench_r05v_fused.err
rc=$?; echo "bench fused rc=$rc"; [ $rc -ne 0 ] && exit $rc
XFK_AMG_FUSED_TAIL=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-fsolver --no-configs4 > gpurun_out/bench_r05v_sep.json 2> gpurun_out/bench_r05v_sep.err
rc=$?; echo "bench separate rc=$rc"; exit $rc
