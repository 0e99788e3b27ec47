#!/bin/bash
# r05: the panel broadcast's LDS base opaque (one base VGPR + offsets; product candidate) vs the
# compiler's per-read absolute addresses (tools/_p/libgp2d_ba0.so): tests, stamps and fit medians
set -o pipefail
mkdir -p gpurun_out/r05_ba
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_batched.py > gpurun_out/r05_ba/tests.log 2>&1 || exit 1
for r in 1 2; do
  for v in st_ba1 st_ba0; do
    GP2D_LIB=tools/_p/libgp2d_$v.so timeout -k 10 200 python3 tools/probe_diag.py 1024 > gpurun_out/r05_ba/${v}_$r.txt 2>&1 || exit 1
  done
  for v in ba1 ba0; do
    lib=2d-gp_amd/gp2d/libgp2d.so; [ "$v" = ba0 ] && lib=tools/_p/libgp2d_ba0.so
    GP2D_LIB=$lib timeout -k 10 200 python3 tools/probe_diag.py 4096 1024 > gpurun_out/r05_ba/${v}_$r.txt 2>&1 || exit 1
  done
done
