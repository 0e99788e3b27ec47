# round 3: SYRK phase offset — the first round's second workgroup per CU sleeps S × 8128 cycles so
# the two co-resident workgroups do not reach the C read-modify-write together (K = 256 microbench)
set -o pipefail
R=gpurun_out/r03sg; mkdir -p $R
cd tools/microbench
for v in 0 4 8 12 0 4 8 12; do timeout -k 10 240 ./syrk_stg$v >> ../../$R/syrk.txt 2>&1 || exit 1; done
cat ../../$R/syrk.txt
