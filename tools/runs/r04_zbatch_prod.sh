# moduli batched on grid.z in the product predict (n ≤ 4096): int8 / predict / batch GPU tests,
# then config B (n = 2048) and the headline (n = 8192, unchanged path) against the previous
# library (build/libgp2d_zb0.so), alternating
set -o pipefail
R=gpurun_out/r04_zbatch_prod
mkdir -p $R
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ozaki.py tests/test_gpu_jobs.py tests/test_gpu_batched.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --config B --cpu-baseline 0 > $R/B_new_$i.json 2> $R/B_new_$i.err || exit 1
  GP2D_LIB=$PWD/build/libgp2d_zb0.so timeout -k 10 300 python -u bench.py --config B --cpu-baseline 0 > $R/B_old_$i.json 2> $R/B_old_$i.err || exit 1
done
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --cpu-baseline 0 > $R/head_new.json 2> $R/head_new.err || exit 1
GP2D_LIB=$PWD/build/libgp2d_zb0.so timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --cpu-baseline 0 > $R/head_old.json 2> $R/head_old.err || exit 1
