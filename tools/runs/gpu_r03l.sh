# round 3, call l: SYRK (POTRF trailing update, lower tiles, beta = 1) rate vs K at the D sizes
set -o pipefail
R=gpurun_out/r03l; mkdir -p $R
cd "$GRAFT_REPO_ROOT/tools/microbench"
for K in 256 512 1024; do timeout -k 10 120 ./syrk_K$K >> ../../$R/syrk.txt 2>&1 || exit 1; done
cat ../../$R/syrk.txt
