#!/bin/bash
# Round profile set for the bench workload (run on the GPU box from the repo root):
#   1. three PMC passes on the unpipelined bench (GRBM_GUI_ACTIVE + SQ_VALU_MFMA_BUSY_CYCLES +
#      SQ_BUSY_CYCLES; FETCH_SIZE; WRITE_SIZE) → clock, MFMA-busy fraction and HBM bytes per
#      launch of the dominant kernel (tools/pmc_igemm.py, or tools/pmc_traffic.py for f64)
#   2. rocprofv3 --kernel-trace --stats of the default (pipelined) bench → per-kernel summary
#   3. the bench line itself, reading the PMC result for roofline.traffic
# Everything lands in gpurun_out/<round>/; copy the summaries into profiles/.
# usage: bash tools/profile_round.sh r02 [ozaki|f64]
set -euo pipefail
R=$1; V=${2:-ozaki}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$R
mkdir -p "$OUT"
export TMPDIR=/tmp
B="bench.py --steps 1 --warmup 1 --cpu-baseline 0 --pipeline 0 --variance $V"
csv() { find "$1" -name "*counter_collection.csv" | head -n 1; }
if [ "$V" = ozaki ]; then
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -f csv -d "$OUT/pmc_clock_$V" -o run -- \
    python3 $B > "$OUT/pmc_clock_$V.log" 2>&1
fi
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/pmc_fetch_$V" -o run -- python3 $B > "$OUT/pmc_fetch_$V.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT/pmc_write_$V" -o run -- python3 $B > "$OUT/pmc_write_$V.log" 2>&1
if [ "$V" = ozaki ]; then
  python3 tools/pmc_igemm.py "$(csv "$OUT/pmc_clock_$V")" "$(csv "$OUT/pmc_fetch_$V")" "$(csv "$OUT/pmc_write_$V")" \
    "$OUT/pmc_traffic_$V.json" > /dev/null
else
  python3 tools/pmc_traffic.py "$(csv "$OUT/pmc_fetch_$V")" "$(csv "$OUT/pmc_write_$V")" "$OUT/pmc_traffic_$V.json" \
    "gemm_f64_kernel<false, 1>" > /dev/null
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_$V" -o run -- \
  python3 bench.py --steps 5 --warmup 2 --cpu-baseline 0 --variance "$V" --pmc-json "$OUT/pmc_traffic_$V.json" \
  > "$OUT/prof_$V.log" 2>&1
timeout -k 10 400 python3 bench.py --variance "$V" --pmc-json "$OUT/pmc_traffic_$V.json" > "$OUT/bench_$V.json" 2> "$OUT/bench_$V.err"
cat "$OUT/bench_$V.json"
