# int8 GEMM cycle shares by in-kernel stamps (tools/microbench/igemm_stamps.hpp), beside the product kernel
set -o pipefail
R=gpurun_out/r04_stamps
mkdir -p $R
cd "$GRAFT_REPO_ROOT/tools/microbench"
timeout -k 10 120 ./igemm_FULL > ../../$R/full.txt 2>&1 || exit 1
timeout -k 10 120 ./igemm_STAMPS > ../../$R/stamps.txt 2>&1 || exit 1
IGEMM_ZERO=1 timeout -k 10 120 ./igemm_STAMPS > ../../$R/stamps_zero.txt 2>&1 || exit 1
