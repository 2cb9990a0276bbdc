# rocprofv3 PMC calibration on known-byte kernels (tools/pmc_calib.hip):
# FETCH_SIZE and WRITE_SIZE in separate passes, each under its own time limit.
# Usage: bash tools/pmc_calib.sh TAG   -> gpurun_out/calib_TAG/{fetch,write}/...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-r02}
OUT=gpurun_out/calib_$TAG
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/fetch -o run -- xfemm_amd/bin/pmc_calib > $OUT/fetch.log 2>&1 && \
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/write -o run -- xfemm_amd/bin/pmc_calib > $OUT/write.log 2>&1 && \
python3 tools/pmc_summary.py --calib $OUT > $OUT/calib.json
