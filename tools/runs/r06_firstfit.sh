#!/bin/bash
# r06: which first action of a process gives the job stream its fast state (tools/probe_first_fit.py),
# with the engine's stream warm-up (engine.warm_streams); the bench without its reference phase;
# the rank-share emulation with the warm-up before RCCL's init
set -o pipefail
R=gpurun_out/r06_firstfit3
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for a in none fit_side pool_then_potrf potrf_tiny none; do
  timeout -k 10 200 python -u tools/probe_first_fit.py $a 40 >> $R/first.jsonl 2>> $R/first.err || exit 1
done
timeout -k 10 300 python -u bench.py --f64-steps 0 --dropin-steps 0 --cpu-baseline 0 --steps 48 --unpipelined-steps 0 > $R/u0.json 2> $R/u0.err && \
timeout -k 10 600 python -u tools/probe_rank_share.py --jobs 96 --warm 24 --P 1,8 --ranks 0,4,last --transport rccl > $R/share.jsonl 2> $R/share.err
