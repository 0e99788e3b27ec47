#!/bin/bash
# r05: per-launch durations and grids of one N_train = 4096 fit's kernels (kernel trace, csv)
set -o pipefail
mkdir -p gpurun_out/r05_trtri
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/r05_trtri/prof -o run -- \
  python3 tools/probe_diag.py 4096 > gpurun_out/r05_trtri/probe.txt 2>&1
