# Lab (round 6): HIP bring-up cost of a fresh process, three link variants.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
O=gpurun_out/init_probe
mkdir -p $O
R=/opt/rocm
hipcc -O2 -o $O/plain tools/lab/init_probe.cpp
hipcc -O2 -o $O/rccl tools/lab/init_probe.cpp -Wl,--no-as-needed -L$R/lib -lrccl -Wl,-rpath,$R/lib
hipcc -O2 -DWITH_XFK -o $O/xfk tools/lab/init_probe.cpp -Lxfemm_amd/lib -lxfemm_kernels -Wl,-rpath,$PWD/xfemm_amd/lib
for v in plain rccl xfk plain rccl xfk; do
  echo "== $v"; t0=$(date +%s%N); timeout -k 5 60 $O/$v; t1=$(date +%s%N); echo "wall $(( (t1 - t0) / 1000000 )) ms"
done > gpurun_out/r06_init_probe.txt 2>&1
cat gpurun_out/r06_init_probe.txt
