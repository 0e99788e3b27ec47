#!/bin/bash
# r05: TRTRI k-split limit (GP2D_TRTRI_SPLIT_TILES: 64 = level 2048 unsplit, 256 = product,
# 1024 = the top level split too): fit medians; then one fit's kernel trace per setting
set -o pipefail
mkdir -p gpurun_out/r05_trtri
export TMPDIR=/tmp
for t in 256 64 1024 256; do
  GP2D_TRTRI_SPLIT_TILES=$t timeout -k 10 300 python3 tools/probe_diag.py 4096 2048 > gpurun_out/r05_trtri/fit_$t.txt 2>&1 || exit 1
done
for t in 256 1024; do
  GP2D_TRTRI_SPLIT_TILES=$t timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/r05_trtri/prof_$t -o run -- \
    python3 tools/probe_diag.py 4096 > gpurun_out/r05_trtri/probe_$t.txt 2>&1 || exit 1
done
