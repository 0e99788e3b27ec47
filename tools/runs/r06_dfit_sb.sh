#!/bin/bash
# r06: the distributed factor with 512- vs 1024-column super-blocks (DF_SB; the 1024 build is
# tools/dev/libgp2d_sb1024.so, made on the CPU side from the same sources with DF_SB = 1024)
set -o pipefail
R=gpurun_out/r06_dfit_sb
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/probe_dfit.py --sizes 16384 --emulate 8 > $R/sb512.jsonl 2> $R/sb512.err || exit 1
GP2D_LIB=$GRAFT_REPO_ROOT/tools/dev/libgp2d_sb1024.so timeout -k 10 300 python -u tools/probe_dfit.py --sizes 16384 --emulate 8 > $R/sb1024.jsonl 2> $R/sb1024.err || exit 1
