# POTRF chain panel GEMM shapes: microbench, factorisation tests, fit latency per size, bench
set -o pipefail
R=gpurun_out/r04_panel
mkdir -p $R
cd "$GRAFT_REPO_ROOT/tools/microbench"
timeout -k 10 60 ./panel_bench > ../../$R/panel.txt 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batched.py tests/test_gpu_distributed.py tests/test_gpu_configs.py tests/test_gpu_jobs.py tests/test_gpu_lml.py -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe_potrf_sched.py --sizes 1024,2048,4096,8192,16384 > $R/fit.jsonl 2> $R/fit.err || exit 1
timeout -k 10 300 python -u tools/probe_fit_batch.py --sizes 1024,4096 --batches 1,8 > $R/fit_batch.jsonl 2> $R/fit_batch.err || exit 1
timeout -k 10 300 python -u bench.py --steps 40 --warmup 2 --cpu-baseline 0 --unpipelined-steps 10 > $R/bench.json 2> $R/bench.err || exit 1
for c in B E; do
  timeout -k 10 300 python -u bench.py --config $c --cpu-baseline 0 > $R/config_$c.json 2> $R/config_$c.err || exit 1
done
