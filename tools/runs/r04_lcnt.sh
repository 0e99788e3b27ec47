# int8 GEMM with LDS-counter hand-offs in place of the per-slab barrier (tools/microbench/igemm_lcnt.hpp)
# vs the product kernel, random-residue triangle, interleaved
set -o pipefail
R=gpurun_out/r04_lcnt
mkdir -p $R
cd "$GRAFT_REPO_ROOT/tools/microbench"
for i in 1 2; do
  timeout -k 10 60 ./igemm_FULL >> ../../$R/micro.txt 2>&1 || exit 1
  timeout -k 10 60 ./igemm_LCNT >> ../../$R/micro.txt 2>&1 || exit 1
done
IGEMM_ZERO=1 timeout -k 10 60 ./igemm_FULL >> ../../$R/micro.txt 2>&1 || exit 1
IGEMM_ZERO=1 timeout -k 10 60 ./igemm_LCNT >> ../../$R/micro.txt 2>&1 || exit 1
