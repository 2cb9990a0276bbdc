# W-cycle depth / dense-coarsest size experiments on configs[2].
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=$1
mkdir -p gpurun_out
run() { name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-configs4 $BARGS \
      > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err
  rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
BARGS= run base XFK_X=0
BARGS="--amg-dense 256" run d256 XFK_X=0
BARGS="--amg-dense 256" run d256_wlo1 XFK_AMG_W_LO=1
BARGS="--amg-dense 256" run d256_w1 XFK_AMG_W=1
BARGS="--amg-dense 512" run d512_wlo1 XFK_AMG_W_LO=1
BARGS= run base2 XFK_X=0
