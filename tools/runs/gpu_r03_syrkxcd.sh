# round 3: SYRK tile order A/B — tri_tile order (XCD=0: consecutive tiles of a row on different
# XCDs) vs XCD-grouped 8×8 super-tiles (1): microbench at K = 256, then whole fits (N = 4096, 16384)
set -o pipefail
R=gpurun_out/r03sx; mkdir -p $R
cd tools/microbench
for v in 0 1 0 1; do timeout -k 10 240 ./syrk_xcd$v >> ../../$R/syrk.txt 2>&1 || exit 1; done
cd ../..
cat $R/syrk.txt
for v in 0 1 0 1; do
  echo "== xcd$v" >> $R/fit.txt
  GP2D_LIB=$PWD/tools/microbench/libgp2d_xcd$v.so timeout -k 10 240 python -u tools/probe_fit.py 4096 16384 >> $R/fit.txt 2>&1 || exit 1
done
cat $R/fit.txt
