# POTRF critical-path kernels in isolation: the skinny panel GEMM per row count and the launch
# floor (tools/microbench/panel_bench.hip), the diagonal kernel (diag_bench)
set -o pipefail
R=gpurun_out/r04_chain
mkdir -p $R
cd "$GRAFT_REPO_ROOT/tools/microbench"
timeout -k 10 60 ./panel_bench > ../../$R/panel.txt 2>&1 || exit 1
timeout -k 10 60 ./diag_bench > ../../$R/diag.txt 2>&1 || exit 1
