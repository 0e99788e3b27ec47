# distributed factor with 512-column super-blocks: parity, then timing (P = 1, one rank's P = 8 share)
set -o pipefail
R=gpurun_out/r04_dfit512
mkdir -p $R
cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_configs.py -x -v -k "distributed or dfit" --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe_dfit.py --sizes 4096,16384 --reps 3 --emulate 8 > $R/probe.log 2>&1 || exit 1
timeout -k 10 200 python -u -m pytest tests/test_gpu_jobs.py -x -q --timeout 150 --timeout-method thread > $R/jobs.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 40 --warmup 3 --unpipelined-steps 10 --cpu-baseline 0 > $R/bench.json 2> $R/bench.err || exit 1
GP2D_IG_TBN=128 timeout -k 10 200 python -u -m pytest tests/test_gpu_ozaki.py -x -q --timeout 150 --timeout-method thread > $R/tbn128_ozaki.log 2>&1 || exit 1
GP2D_IG_TBN=128 timeout -k 10 200 python -u bench.py --steps 40 --warmup 3 --unpipelined-steps 10 --cpu-baseline 0 > $R/bench_tbn128.json 2> $R/bench_tbn128.err || exit 1
