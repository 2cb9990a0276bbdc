# round 5: folded post-step on sharded levels -- sharded tests, then rank 0 of 8 A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_sharded.py tests/test_gpu_comm_order.py tests/test_gpu_harmonic_sharded.py tests/test_gpu_fsolver_sharded.py > gpurun_out/r05q_tests.log 2>&1
rc=$?; echo "tests rc=$rc"
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 660 python -u tools/lab/rank0_probe.py --cells 3162 --ranks 8 '' XFK_AMG_FOLD_DIST=0 XFK_AMG_HB=0 XFK_AMG_FOLD_DIST=0,XFK_AMG_HB=0 > gpurun_out/r05q_rank0.txt 2>&1
rc2=$?; echo "probe rc=$rc2"; exit $(( rc ? rc : rc2 ))
