#!/bin/bash
# r05: the diagonal kernel's 32×32 block products on the f64 matrix core (GP2D_DIAG_MFMA=1, product)
# vs the FMA tiles (dev build tools/_p/libgp2d_mf0.so): phase stamps (diag_stamps.h builds), fit
# medians, kernel stats; alternated
set -o pipefail
mkdir -p gpurun_out/r05_diagmf
export TMPDIR=/tmp
for v in st_mf1 st_mf0; do
  GP2D_LIB=tools/_p/libgp2d_$v.so timeout -k 10 300 python3 tools/probe_diag.py 1024 > gpurun_out/r05_diagmf/$v.txt 2>&1 || exit 1
done
for v in prod mf0 prod2 mf0b; do
  lib=2d-gp_amd/gp2d/libgp2d.so; case $v in mf0*) lib=tools/_p/libgp2d_mf0.so;; esac
  GP2D_LIB=$lib timeout -k 10 300 python3 tools/probe_diag.py 4096 1024 16384 > gpurun_out/r05_diagmf/$v.txt 2>&1 || exit 1
done
for v in prod mf0; do
  lib=2d-gp_amd/gp2d/libgp2d.so; [ "$v" = mf0 ] && lib=tools/_p/libgp2d_mf0.so
  GP2D_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r05_diagmf/prof_$v -o run -- \
    python3 tools/probe_diag.py 4096 > gpurun_out/r05_diagmf/prof_$v.txt 2>&1 || exit 1
  find gpurun_out/r05_diagmf/prof_$v -name "*kernel_trace.csv" -delete
done
