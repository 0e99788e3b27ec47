#!/bin/bash
# r06: the job stream at GPU_MAX_HW_QUEUES 4 (the box default) / 6 / 8 with the stream warm-up
set -o pipefail
R=gpurun_out/r06_hwq
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python -u bench.py --f64-steps 0 --dropin-steps 0 --cpu-baseline 0 --steps 48"
timeout -k 10 300 $B > $R/q4.json 2> $R/q4.err && \
GPU_MAX_HW_QUEUES=6 timeout -k 10 300 $B > $R/q6.json 2> $R/q6.err && \
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 $B > $R/q8.json 2> $R/q8.err && \
timeout -k 10 300 $B > $R/q4b.json 2> $R/q4b.err
