#!/bin/bash
# r06: the factor chain on reserved CUs (tools/probe_fit_reserve.py), R = 0 / 16 / 32 / 64 / 0
set -o pipefail
R=gpurun_out/r06_reserve
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 0 16 32 64 0; do
  timeout -k 10 200 python -u tools/probe_fit_reserve.py $r >> $R/reserve.jsonl 2>> $R/reserve.err || exit 1
done
