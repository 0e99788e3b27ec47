# round 3: SYRK tile rate at K = 512 vs K = 256 (microbench), the gain a four-panel update would see
set -o pipefail
R=gpurun_out/r03sk; mkdir -p $R
cd tools/microbench
for v in epi1 k512 epi1 k512; do timeout -k 10 240 ./syrk_$v >> ../../$R/syrk.txt 2>&1 || exit 1; done
cat ../../$R/syrk.txt
