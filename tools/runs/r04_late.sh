# staggered LDS-DMA issue in the int8 GEMM (GP2D_IG_LATE): microbench A/B on random residues with
# stamp shares, int8 parity tests, then the bench with the product (LATE=1) vs build/libgp2d_late0.so
set -o pipefail
R=gpurun_out/r04_late
mkdir -p $R
cd "$GRAFT_REPO_ROOT/tools/microbench"
for i in 1 2; do
  timeout -k 10 120 ./igemm_FULL >> ../../$R/micro.txt 2>&1 || exit 1
  timeout -k 10 120 ./igemm_LATE0 >> ../../$R/micro.txt 2>&1 || exit 1
done
timeout -k 10 120 ./igemm_STAMPS > ../../$R/stamps_late1.txt 2>&1 || exit 1
timeout -k 10 120 ./igemm_STAMPS0 > ../../$R/stamps_late0.txt 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_ozaki.py tests/test_gpu_configs.py tests/test_gpu_jobs.py -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 3 --cpu-baseline 0 > $R/bench_$i.json 2> $R/bench_$i.err || exit 1
  GP2D_LIB=$PWD/build/libgp2d_late0.so timeout -k 10 200 python -u bench.py --steps 100 --warmup 3 --cpu-baseline 0 > $R/late0_$i.json 2> $R/late0_$i.err || exit 1
done
