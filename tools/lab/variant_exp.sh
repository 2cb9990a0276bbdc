# A/B of an env-selected kernel variant through bench.py's phase table.
# usage: bash tools/lab/variant_exp.sh TAG VAR "v1 v2 ..." [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=$1; VAR=$2; VALS=$3; shift 3
mkdir -p gpurun_out
for v in $VALS; do
  env $VAR=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-configs4 "$@" \
      > gpurun_out/${TAG}_${VAR}_$v.json 2> gpurun_out/${TAG}_${VAR}_$v.err
  rc=$?
  echo "$VAR=$v rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
