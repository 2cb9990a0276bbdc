# round 5: the FSolver host path stage by stage on the box (configs[2], configs[1])
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r05ab /tmp/hp2 /tmp/hp1
export TMPDIR=/tmp XFEMM_TRACE_LOAD=1 XFK_TRACE_CREATE=1
echo "nproc $(nproc)" > gpurun_out/r05ab/host.txt
timeout -k 10 300 python3 tools/lab/host_path.py /tmp/hp2 1000 > gpurun_out/r05ab/c2.txt 2>&1
rc=$?; echo "c2 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/lab/host_path.py /tmp/hp1 0 > gpurun_out/r05ab/c1.txt 2>&1
rc=$?; echo "c1 rc=$rc"; exit $rc
