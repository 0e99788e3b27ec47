# the twelve per-modulus int8 GEMM launches of a predict chunk vs one launch with the moduli on
# blockIdx.z (tools/microbench/igemm_zbatch.hip), n = 2048 (config B) and 8192 (headline)
set -o pipefail
R=gpurun_out/r04_zbatch
mkdir -p $R
cd "$GRAFT_REPO_ROOT/tools/microbench"
timeout -k 10 300 ./igemm_zbatch > ../../$R/zbatch.txt 2>&1
