#!/bin/bash
# r06: the factor chain on reserved CUs with and without the fused inverse
# (tools/probe_fit_reserve.py R FUSED STREAM)
set -o pipefail
R=gpurun_out/r06_reserve2
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for a in "0 0 0" "0 1 0" "64 0 0" "64 1 0" "96 1 0" "128 1 0" "32 1 0" "0 0 0"; do
  timeout -k 10 200 python -u tools/probe_fit_reserve.py $a >> $R/reserve.jsonl 2>> $R/reserve.err || exit 1
done
