# round 5: the configs[2] FSolver host path stage by stage, and the box's /tmp
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r05ae /tmp/hp2
export TMPDIR=/tmp
(df -T /tmp; grep -E " /tmp | / " /proc/mounts; nproc; grep -c processor /proc/cpuinfo; cat /sys/kernel/mm/transparent_hugepage/enabled) > gpurun_out/r05ae/host.txt 2>&1
XFK_TRACE_CREATE=1 XFEMM_TRACE_LOAD=1 timeout -k 10 300 python3 tools/lab/host_path.py /tmp/hp2 1000 > gpurun_out/r05ae/c2.txt 2>&1
rc=$?; echo "c2 rc=$rc"; [ $rc -ne 0 ] && exit $rc
XFK_TRACE_CREATE=1 XFEMM_TRACE_LOAD=1 timeout -k 10 200 python3 tools/lab/host_path.py /tmp/hp1 0 > gpurun_out/r05ae/c1.txt 2>&1
rc=$?; echo "c1 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_static2d.py tests/test_gpu_torque.py tests/test_gpu_fsolver_sharded.py tests/test_gpu_prev_solution.py > gpurun_out/r05ae/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; exit $rc
