# round 3, call f: int8 GEMM — 128x128 per wave, one wave per SIMD (igemm_W128) vs the product kernel
set -o pipefail
R=gpurun_out/r03f; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/microbench/pmc_clock.sh FULL W128 W128S > $R/w128.txt 2>&1; echo "rc $?"; cat $R/w128.txt
