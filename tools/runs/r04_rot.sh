# the late wave group's slab step rotated by half a step (tools/microbench/igemm_rot.hpp):
# triangular launch + sampled check, and dense K = 8192 / 2048, against the product kernel
set -o pipefail
R=gpurun_out/r04_rot
mkdir -p $R
cd "$GRAFT_REPO_ROOT/tools/microbench"
for i in 1 2; do
  timeout -k 10 120 ./igemm_FULL >> ../../$R/micro.txt 2>&1 || exit 1
  timeout -k 10 120 ./igemm_ROT >> ../../$R/micro.txt 2>&1 || exit 1
  timeout -k 10 120 ./igemm_ROT2 >> ../../$R/micro.txt 2>&1 || exit 1
done
for k in 8192 2048; do
  IGEMM_K=$k timeout -k 10 120 ./igemm_FULL >> ../../$R/micro.txt 2>&1 || exit 1
  IGEMM_K=$k timeout -k 10 120 ./igemm_ROT >> ../../$R/micro.txt 2>&1 || exit 1
  IGEMM_K=$k timeout -k 10 120 ./igemm_ROT2 >> ../../$R/micro.txt 2>&1 || exit 1
  timeout -k 10 120 ./igemm_ROT2 >> ../../$R/micro.txt 2>&1 || exit 1   # (an extra triangular run)
done
