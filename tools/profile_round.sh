#!/bin/bash
# Round profile set for the bench workload (run on the GPU box from the repo root):
#   1. two PMC passes (FETCH_SIZE, WRITE_SIZE) → HBM bytes per launch of the dominant kernel
#   2. rocprofv3 --kernel-trace --stats → per-kernel summary
#   3. the bench line itself, reading the PMC result for roofline.traffic
# Everything lands in gpurun_out/<round>/; copy the summaries into profiles/.
# usage: bash tools/profile_round.sh r01 [ozaki|f64]
set -euo pipefail
R=$1; V=${2:-ozaki}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$R
mkdir -p "$OUT"
if [ "$V" = ozaki ]; then PAT=igemm_nt_mod_kernel; else PAT="gemm_f64_kernel<false, 1>"; fi
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/pmc_fetch_$V" -o run -- \
  python3 bench.py --steps 1 --warmup 1 --cpu-baseline 0 --variance "$V" > "$OUT/pmc_fetch_$V.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT/pmc_write_$V" -o run -- \
  python3 bench.py --steps 1 --warmup 1 --cpu-baseline 0 --variance "$V" > "$OUT/pmc_write_$V.log" 2>&1
F=$(find "$OUT/pmc_fetch_$V" -name "*counter_collection.csv" | head -n 1)
W=$(find "$OUT/pmc_write_$V" -name "*counter_collection.csv" | head -n 1)
python3 tools/pmc_traffic.py "$F" "$W" "$OUT/pmc_traffic_$V.json" "$PAT" > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_$V" -o run -- \
  python3 bench.py --steps 5 --warmup 2 --cpu-baseline 0 --variance "$V" --pmc-json "$OUT/pmc_traffic_$V.json" \
  > "$OUT/prof_$V.log" 2>&1
timeout -k 10 400 python3 bench.py --variance "$V" --pmc-json "$OUT/pmc_traffic_$V.json" > "$OUT/bench_$V.json" 2> "$OUT/bench_$V.err"
cat "$OUT/bench_$V.json"
