#!/bin/bash
# r05: the CRT kernel's residue-plane loads non-temporal (dev build tools/_p/libgp2d_crtnt.so,
# -DGP2D_CRT_NTLOAD=1) vs the product, alternated, same bench command
set -o pipefail
mkdir -p gpurun_out/r05_crtnt
for r in 1 2; do
  for v in prod crtnt; do
    lib=2d-gp_amd/gp2d/libgp2d.so; [ "$v" = prod ] || lib=tools/_p/libgp2d_$v.so
    GP2D_LIB=$lib timeout -k 10 300 python3 bench.py --steps 30 --warmup 3 --unpipelined-steps 10 --cpu-baseline 0 \
      --f64-steps 0 --dropin-steps 0 > gpurun_out/r05_crtnt/${v}_$r.json 2> gpurun_out/r05_crtnt/${v}_$r.err || exit 1
  done
done
