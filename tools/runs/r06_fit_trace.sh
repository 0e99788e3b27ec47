#!/bin/bash
# r06: kernel trace of lone N_train = 4096 fits (tools/probe_fit.py: fused, two-call, fused) for the
# POTRF chain's composition at HEAD (tools/fit_trace.py on the database)
set -o pipefail
R=gpurun_out/r06_fit_trace
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/db -o run -- python3 -u tools/probe_fit.py 4096 > $R/fit.txt 2> $R/fit.err
