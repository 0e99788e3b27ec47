#!/bin/bash
# r06: the job stream's rate after different preambles (tools/probe_alloc_state.py)
set -o pipefail
R=gpurun_out/r06_alloc
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u tools/probe_alloc_state.py 40 > $R/alloc.jsonl 2> $R/alloc.err
