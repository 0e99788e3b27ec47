#!/bin/bash
# r05: the diagonal kernel's block load overlapped with panel 0 (product) vs load-then-barrier
# (tools/_p/libgp2d_ld0.so, the previous commit): tests, phase stamps and fit medians alternated,
# then the round-end sequence
set -o pipefail
mkdir -p gpurun_out/r05_load
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_batched.py > gpurun_out/r05_load/tests.log 2>&1 || exit 1
for r in 1 2; do
  for v in st_ld1 st_ld0; do
    GP2D_LIB=tools/_p/libgp2d_$v.so timeout -k 10 200 python3 tools/probe_diag.py 1024 > gpurun_out/r05_load/${v}_$r.txt 2>&1 || exit 1
  done
  for v in ld1 ld0; do
    lib=2d-gp_amd/gp2d/libgp2d.so; [ "$v" = ld0 ] && lib=tools/_p/libgp2d_ld0.so
    GP2D_LIB=$lib timeout -k 10 200 python3 tools/probe_diag.py 4096 1024 > gpurun_out/r05_load/${v}_$r.txt 2>&1 || exit 1
  done
done
bash tools/gpu_round_end.sh r05_load_round_end
