#!/bin/bash
# r05: the diagonal-block kernel's panel pivots with the lagged update (GP2D_PANEL_LAG; factor.hpp at git 9434024)
# vs panel_step (dev build tools/_p/libgp2d_lag0.so): per-call time, fit medians, factor bits;
# then phase stamps (tools/microbench/diag_stamps.h) of dev builds: lag1, lag0, lag1 without the
# second row set of panels 0-1 (NOX1: timing only).
set -o pipefail
mkdir -p gpurun_out/r05_diag
for v in prod lag0; do
  lib=2d-gp_amd/gp2d/libgp2d.so; [ "$v" = lag0 ] && lib=tools/_p/libgp2d_lag0.so
  GP2D_LIB=$lib timeout -k 10 300 python -u tools/probe_diag.py 4096 1024 16384 \
    > gpurun_out/r05_diag/$v.txt 2>&1 || exit 1
done
for v in st_lag1 st_lag0 st_nox1; do
  GP2D_LIB=tools/_p/libgp2d_$v.so timeout -k 10 300 python -u tools/probe_diag.py 1024 > gpurun_out/r05_diag/$v.txt 2>&1 || exit 1
done
