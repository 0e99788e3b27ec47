#!/bin/bash
# r05: the pivot column scaled by one select (lane ≥ K; the pivot lane gets d·(1/√d) = rd) vs two
# (dev builds tools/_p/libgp2d_sc1.so / sc0.so): stamps and fit medians alternated
set -o pipefail
mkdir -p gpurun_out/r05_sc
for r in 1 2; do
  for v in st_sc1 st_sc0; do
    GP2D_LIB=tools/_p/libgp2d_$v.so timeout -k 10 200 python3 tools/probe_diag.py 1024 > gpurun_out/r05_sc/${v}_$r.txt 2>&1 || exit 1
  done
  for v in sc1 sc0; do
    lib=tools/_p/libgp2d_$v.so
    GP2D_LIB=$lib timeout -k 10 200 python3 tools/probe_diag.py 4096 1024 > gpurun_out/r05_sc/${v}_$r.txt 2>&1 || exit 1
  done
done
