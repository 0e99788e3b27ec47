#!/bin/bash
# r06: does a long RCCL copy on the comm stream (an xGMI-length transfer: the payload copied 10
# times per received job) hold up the predict stream (tools/probe_rank_share.py --copy-repeat)?
set -o pipefail
R=gpurun_out/r06_commq
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u tools/probe_rank_share.py --jobs 48 --warm 16 --P 8 --ranks 0 --transport rccl --copy-repeat 1 > $R/rep1.jsonl 2> $R/rep1.err && \
timeout -k 10 600 python -u tools/probe_rank_share.py --jobs 48 --warm 16 --P 8 --ranks 0 --transport rccl --copy-repeat 10 > $R/rep10.jsonl 2> $R/rep10.err
