#!/bin/bash
# r06: one rank's share of the P-GPU round-robin job stream emulated on one GPU (tools/probe_rank_share.py):
# P = 1, 2, 4, 8, first/last rank, RCCL copy vs plain copy; then every rank of P = 8 (96 jobs)
set -o pipefail
R=gpurun_out/r06_rank_share
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u tools/probe_rank_share.py --jobs 96 --P 1,8 --ranks all --transport rccl > $R/share_p8_all.jsonl 2> $R/share_p8_all.err && \
timeout -k 10 400 python -u bench.py --f64-steps 0 --dropin-steps 0 --cpu-baseline 0 > $R/bench.json 2> $R/bench.err
