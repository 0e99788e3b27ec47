# int8 GEMM epilogue timing: the product kernel, its dev copy (LDS-transposed epilogue) and the
# dev copy storing residues straight from the MFMA registers (tools/microbench/igemm_epi.hpp)
set -o pipefail
R=gpurun_out/r04_epi
mkdir -p $R
cd "$GRAFT_REPO_ROOT/tools/microbench"
for i in 1 2; do
  for v in FULL EPI_LDS EPI_DIRECT; do
    timeout -k 10 120 ./igemm_$v >> ../../$R/epi.txt 2>&1 || exit 1
  done
done
for k in 2048 8192; do
  for v in FULL EPI_LDS EPI_DIRECT; do
    IGEMM_K=$k timeout -k 10 120 ./igemm_$v >> ../../$R/epi.txt 2>&1 || exit 1
  done
done
