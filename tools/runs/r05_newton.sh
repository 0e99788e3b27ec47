#!/bin/bash
# r05: diagonal-kernel phase stamps of dev builds (tools/runs/r05_diag.sh builds), product probe
set -o pipefail
mkdir -p gpurun_out/r05_diag
for v in ${DIAG_VARIANTS:-st_lag1 st_lag0}; do
  GP2D_LIB=tools/_p/libgp2d_$v.so timeout -k 10 300 python -u tools/probe_diag.py 1024 > gpurun_out/r05_diag/$v.txt 2>&1 || exit 1
done
timeout -k 10 300 python -u tools/probe_diag.py 4096 1024 > gpurun_out/r05_diag/prod.txt 2>&1
