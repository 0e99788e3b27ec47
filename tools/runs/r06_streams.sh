#!/bin/bash
# r06: the fit side stream's pool index vs the headline job stream (tools/probe_stream_pick.py),
# the recv-cost proxy on fixed streams (tools/probe_recv_cost.py), and the bench on the same box
set -o pipefail
R=gpurun_out/r06_streams
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/probe_stream_pick.py 20 > $R/pick.jsonl 2> $R/pick.err && \
timeout -k 10 400 python -u tools/probe_recv_cost.py --jobs 40 > $R/recv.jsonl 2> $R/recv.err && \
timeout -k 10 400 python -u bench.py --f64-steps 0 --dropin-steps 0 --cpu-baseline 0 > $R/bench.json 2> $R/bench.err
