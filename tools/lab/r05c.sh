# round 5: host path -- .ans byte identity through the mapped writer, torque .fem -> .ans, host stage probe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) exit $1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_static2d.py tests/test_gpu_torque.py tests/test_gpu_prev_solution.py tests/test_gpu_harmonic.py tests/test_gpu_magdir.py -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_r05c.log 2>&1
rc=$?; echo "tests rc=$rc"; fatal $rc
timeout -k 10 240 python tools/lab/host_probe.py 1000 3 > gpurun_out/host_probe_r05c.txt 2>&1
rc=$?; echo "probe rc=$rc"; fatal $rc
df -h /tmp | tail -1; mount | grep -E " /tmp | / " | head -3
