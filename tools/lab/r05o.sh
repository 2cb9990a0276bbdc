# round 5: sharded Newton AC periodic-16: aux matrices single vs row blocks
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/lab/aux_dump_cmp.py periodic 16 2 > gpurun_out/aux_cmp.txt 2> gpurun_out/aux_cmp.err
rc=$?; echo "probe rc=$rc"; exit $rc
