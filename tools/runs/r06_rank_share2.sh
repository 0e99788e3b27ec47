#!/bin/bash
# r06: the rank-share emulation with 24 warm jobs before each timed stream (allocator / clock state as
# in bench.py's timed region), P = 1 / 2 / 4 / 8, and the bench on the same box
set -o pipefail
R=gpurun_out/r06_rank_share2
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u tools/probe_rank_share.py --jobs 96 --warm 24 --P 1,2,4,8 --ranks 0,4,last --transport rccl > $R/share.jsonl 2> $R/share.err && \
timeout -k 10 400 python -u bench.py --f64-steps 0 --dropin-steps 0 --cpu-baseline 0 > $R/bench.json 2> $R/bench.err
