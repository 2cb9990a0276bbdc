set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_newton_ac.py -v -s --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/newton_ac_r04t.log 2>&1
echo "nac rc=$?"
