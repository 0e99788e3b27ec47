# K* residues without the int conversion (magic-number low bytes, v_perm packing), buffer stores with
# 32-bit plane offsets, unrolled finalize sums: parity, bench, kernel trace; then the CRT with 8 rows
# per lane (68 VGPRs, 7 waves per SIMD; build/libgp2d_crt8.so via GP2D_LIB) against the default 16
set -o pipefail
R=gpurun_out/r04_kstar
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || exit 1
timeout -k 10 120 python -u __graft_entry__.py smoke > $R/smoke.txt 2>&1 || exit 1
GP2D_LIB=$PWD/build/libgp2d_crt8.so timeout -k 10 400 python -u -m pytest tests/test_gpu_ozaki.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $R/tests_crt8.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 3 --cpu-baseline 0 > $R/bench_$i.json 2> $R/bench_$i.err || exit 1
  GP2D_LIB=$PWD/build/libgp2d_crt8.so timeout -k 10 200 python -u bench.py --steps 100 --warmup 3 --cpu-baseline 0 > $R/crt8_$i.json 2> $R/crt8_$i.err || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/prof -o trace -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline 0 --unpipelined-steps 0 > $R/prof_bench.json 2> $R/prof.err || exit 1
GP2D_LIB=$PWD/build/libgp2d_crt8.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/prof8 -o trace -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline 0 --unpipelined-steps 0 > $R/prof8_bench.json 2> $R/prof8.err
