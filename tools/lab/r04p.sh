set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/lab/r04n.sh || exit $?
bash tools/lab/r04o.sh
