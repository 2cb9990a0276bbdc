# the full -m gpu suite without -x (every failure listed), then the smoke
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_r04i.log 2>&1
rc=$?
echo "tests rc=$rc"
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r04i.log 2>&1
echo "smoke rc=$?"
