# round-4 end-of-session check at HEAD: full GPU suite, smoke, the driver's exact bench command
# under a kernel trace (timed-region frac), configs B / C / E with the library defaults
set -o pipefail
R=gpurun_out/r04_final
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $R/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $R/smoke.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $R/exact_bench.json 2> $R/exact_bench.err || exit 1
python3 tools/rocprof_timed.py $R/prof/run_kernel_trace.csv $R/exact_bench.json $R/exact_timed_region.json > /dev/null || exit 1
for c in B C E; do
  timeout -k 10 300 python -u bench.py --config $c --cpu-baseline 0 > $R/config_$c.json 2> $R/config_$c.err || exit 1
done
timeout -k 10 400 python -u bench.py > $R/bench_default.json 2> $R/bench_default.err || exit 1
