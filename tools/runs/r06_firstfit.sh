#!/bin/bash
# r06: which first action of a process gives the job stream its fast state (tools/probe_first_fit.py)
set -o pipefail
R=gpurun_out/r06_firstfit
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for a in none fit_nocheck fit_check fit_side job potrf_tiny none; do
  timeout -k 10 200 python -u tools/probe_first_fit.py $a 40 >> $R/first.jsonl 2>> $R/first.err || exit 1
done
