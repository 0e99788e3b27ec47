#!/bin/bash
# r06 profile set at HEAD: the three PMC passes of the dominant kernel (tools/profile_round.sh's first
# part: clock + MFMA busy, FETCH_SIZE, WRITE_SIZE), then the driver's exact bench command, then the same
# command under a rocprofv3 kernel trace with the timed region marked (GP2D_TRACE_MARKS=1)
set -o pipefail
R=gpurun_out/r06_profile
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="bench.py --steps 1 --warmup 1 --cpu-baseline 0 --pipeline 0 --f64-steps 0 --dropin-steps 0 --unpipelined-steps 0"
csv() { find "$1" -name "*counter_collection.csv" | head -n 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -f csv -d $R/pmc_clock -o run -- \
  python3 $B > $R/pmc_clock.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $R/pmc_fetch -o run -- python3 $B > $R/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $R/pmc_write -o run -- python3 $B > $R/pmc_write.log 2>&1 || exit 1
python3 tools/pmc_igemm.py "$(csv $R/pmc_clock)" "$(csv $R/pmc_fetch)" "$(csv $R/pmc_write)" $R/pmc_traffic_ozaki.json > $R/pmc.txt || exit 1
rm -rf $R/pmc_clock $R/pmc_fetch $R/pmc_write
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --pmc-json $R/pmc_traffic_ozaki.json > $R/default.json 2> $R/default.err || exit 1
GP2D_TRACE_MARKS=1 timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d $R/trace -o run -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 --pmc-json $R/pmc_traffic_ozaki.json > $R/traced.json 2> $R/traced.err || exit 1
f=$(find $R/trace -name "*kernel_trace.csv" | head -n 1)
python3 tools/timed_kernels.py "$f" $R/timed_kernels.json > /dev/null
s=$(find $R/trace -name "*kernel_stats.csv" | head -n 1)
cp "$s" $R/kernel_stats.csv
python3 tools/rocprof_timed.py "$f" $R/traced.json $R/timed_region.json > /dev/null || true
rm -rf $R/trace
