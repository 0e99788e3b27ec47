# round 3: SYRK phase offset — the first round's second workgroup per CU sleeps S × 8128 cycles so
# the two co-resident workgroups do not reach the C read-modify-write together (K = 256 microbench)
set -o pipefail
R=gpurun_out/r03sg; mkdir -p $R
cd tools/microbench
for v in 0 4 8 12 0 4 8 12; do timeout -k 10 240 ./syrk_stg$v >> ../../$R/syrk.txt 2>&1 || exit 1; done
cat ../../$R/syrk.txt
cd ../..
for v in 0 6 10 0 6 10; do
  echo "== stagger $v" >> $R/fit.txt
  GP2D_LIB=$PWD/tools/microbench/libgp2d_stg$v.so timeout -k 10 240 python -u tools/probe_fit.py 4096 16384 >> $R/fit.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $R/fit.txt
