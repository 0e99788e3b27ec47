# round 3: SYRK C epilogue A/B — four exposed C round trips per tile (EPI_PIPE=0) vs group mi+1's
# loads issued before group mi's stores (1): microbench at K = 256, then whole fits (N = 4096, 16384)
set -o pipefail
R=gpurun_out/r03se; mkdir -p $R
cd tools/microbench
for v in 0 1 0 1; do timeout -k 10 240 ./syrk_epi$v >> ../../$R/syrk.txt 2>&1 || exit 1; done
cd ../..
cat $R/syrk.txt
for v in 0 1 0 1; do
  echo "== epi$v" >> $R/fit.txt
  GP2D_LIB=$PWD/tools/microbench/libgp2d_epi$v.so timeout -k 10 240 python -u tools/probe_fit.py 4096 16384 >> $R/fit.txt 2>&1 || exit 1
done
cat $R/fit.txt
