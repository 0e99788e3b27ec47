#!/bin/bash
# r06: a single fit's parts timed alone (tools/probe_fit_parts.py)
set -o pipefail
R=gpurun_out/r06_fitparts
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/probe_fit_parts.py 4096 > $R/parts.txt 2> $R/parts.err && \
timeout -k 10 300 python -u tools/probe_fit_parts.py 1024 >> $R/parts.txt 2>> $R/parts.err
