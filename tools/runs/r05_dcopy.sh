#!/bin/bash
# r05: the diagonal kernel's final inv(L_kk) copy loop unrolled by 8 (product) vs not unrolled
# (tools/_p/libgp2d_u1.so): phase stamps and engine.fit medians, alternated in one call
set -o pipefail
mkdir -p gpurun_out/r05_dcopy
for r in 1 2; do
  for v in st_u8 st_u1; do
    GP2D_LIB=tools/_p/libgp2d_$v.so timeout -k 10 200 python3 tools/probe_diag.py 1024 > gpurun_out/r05_dcopy/${v}_$r.txt 2>&1 || exit 1
  done
  for v in u8 u1; do
    lib=2d-gp_amd/gp2d/libgp2d.so; [ "$v" = u1 ] && lib=tools/_p/libgp2d_u1.so
    GP2D_LIB=$lib timeout -k 10 200 python3 tools/probe_diag.py 4096 1024 > gpurun_out/r05_dcopy/${v}_$r.txt 2>&1 || exit 1
  done
done
