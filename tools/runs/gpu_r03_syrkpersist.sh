# round 3: persistent SYRK (2 workgroups per CU walk the tiles; the next tile's first slab is
# loaded under the C epilogue) vs the product SYRK launch, K = 256 microbench
set -o pipefail
R=gpurun_out/r03sp; mkdir -p $R
cd tools/microbench
for v in epi1 persist epi1 persist; do timeout -k 10 240 ./syrk_$v >> ../../$R/syrk.txt 2>&1 || exit 1; done
cat ../../$R/syrk.txt
