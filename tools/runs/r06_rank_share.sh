#!/bin/bash
# r06: one rank's share of the P-GPU round-robin job stream emulated on one GPU (tools/probe_rank_share.py)
set -o pipefail
R=gpurun_out/r06_rank_share
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u tools/probe_rank_share.py --jobs 48 > $R/share.jsonl 2> $R/share.err
