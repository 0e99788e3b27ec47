#!/bin/bash
# r06: the unpipelined job with the K* planes generated on a side stream during the fit
# (bench.py --kstar-ahead 1: its `unpipelined` reading) against inline K* (0), alternating
set -o pipefail
R=gpurun_out/r06_kstar_ahead
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
X="--steps 10 --warmup 2 --cpu-baseline 0 --f64-steps 0 --dropin-steps 0 --unpipelined-steps 20"
for v in "a0:0" "a1:1" "b0:0" "b1:1"; do
  timeout -k 10 300 python -u bench.py $X --kstar-ahead ${v#*:} > $R/${v%%:*}.json 2> $R/${v%%:*}.err || exit 1
done
