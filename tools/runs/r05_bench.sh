#!/bin/bash
# r05: the driver's exact bench command, then the same command under a rocprofv3 kernel trace with
# the timed region marked (GP2D_TRACE_MARKS=1) → which kernels run in the timed region
set -o pipefail
mkdir -p gpurun_out/r05_bench
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05_bench/default.json 2> gpurun_out/r05_bench/default.err || exit 1
GP2D_TRACE_MARKS=1 timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r05_bench/trace -o run -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05_bench/traced.json 2> gpurun_out/r05_bench/traced.err || exit 1
f=$(find gpurun_out/r05_bench/trace -name "*kernel_trace.csv" | head -n 1)
python3 tools/timed_kernels.py "$f" gpurun_out/r05_bench/timed_kernels.json > /dev/null
s=$(find gpurun_out/r05_bench/trace -name "*kernel_stats.csv" | head -n 1)
cp "$s" gpurun_out/r05_bench/kernel_stats.csv
python3 tools/rocprof_timed.py "$f" gpurun_out/r05_bench/traced.json gpurun_out/r05_bench/timed_region.json > /dev/null || true
rm -f "$f"
