#!/bin/bash
# r06: kernel statistics of the rank-share emulation at P = 1 and P = 2 (rank 0): where a P = 2
# rank's extra ~3 ms per job goes
set -o pipefail
R=gpurun_out/r06_share_trace
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for p in 1 2; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/p$p -o run -- python3 -u tools/probe_rank_share.py --jobs 48 --warm 12 --P $p --ranks 0 --transport rccl > $R/p$p.jsonl 2> $R/p$p.err || exit 1
done
