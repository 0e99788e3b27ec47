#!/bin/bash
# r06: the rank-share emulation after the stream-binding fix at P = 1 / 2 / 4 (ranks 0 and last; P = 8
# is r06_rank_share_warm.jsonl), 96 timed jobs after 24 warm ones, RCCL self send/recv receives
set -o pipefail
R=gpurun_out/r06_rank_share3
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u tools/probe_rank_share.py --jobs 96 --warm 24 --P 1,2,4 --ranks 0,last --transport rccl > $R/share.jsonl 2> $R/share.err
