#!/bin/bash
# r06: bisect the bench-state effect — how many unpipelined jobs bring the pipelined stream to its
# fast state, and does it survive into a second timed stream in the same process
set -o pipefail
R=gpurun_out/r06_benchstate2
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python -u bench.py --f64-steps 0 --dropin-steps 0 --cpu-baseline 0 --steps 48"
for u in 0 1 3 20; do
  timeout -k 10 300 $B --unpipelined-steps $u > $R/u$u.json 2> $R/u$u.err || exit 1
done
