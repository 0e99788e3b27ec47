#!/bin/bash
# r06: why a bare krige_jobs stream (tools/probe_*) runs ~4 ms per job slower than bench.py's timed
# region: the bench with and without its unpipelined phase, and with 24 warmup jobs
set -o pipefail
R=gpurun_out/r06_benchstate
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python -u bench.py --f64-steps 0 --dropin-steps 0 --cpu-baseline 0"
timeout -k 10 300 $B > $R/default.json 2> $R/default.err && \
timeout -k 10 300 $B --unpipelined-steps 0 > $R/nounpiped.json 2> $R/nounpiped.err && \
timeout -k 10 300 $B --unpipelined-steps 0 --warmup 24 > $R/nounpiped_w24.json 2> $R/nounpiped_w24.err && \
timeout -k 10 300 $B --steps 48 > $R/steps48.json 2> $R/steps48.err
