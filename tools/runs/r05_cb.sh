#!/bin/bash
# r05: the panel's column broadcast stored by all 64 lanes (product candidate) vs lanes < 32 under an
# EXEC mask (tools/_p/libgp2d_cb0.so): stamps and fit medians alternated
set -o pipefail
mkdir -p gpurun_out/r05_cb
for r in 1 2; do
  for v in st_cb1 st_cb0; do
    GP2D_LIB=tools/_p/libgp2d_$v.so timeout -k 10 200 python3 tools/probe_diag.py 1024 > gpurun_out/r05_cb/${v}_$r.txt 2>&1 || exit 1
  done
  for v in cb1 cb0; do
    lib=2d-gp_amd/gp2d/libgp2d.so; [ "$v" = cb0 ] && lib=tools/_p/libgp2d_cb0.so
    GP2D_LIB=$lib timeout -k 10 200 python3 tools/probe_diag.py 4096 1024 > gpurun_out/r05_cb/${v}_$r.txt 2>&1 || exit 1
  done
done
