#!/bin/bash
# r05: what a pipelined headline job pays for its fit — the product build vs
# dev builds whose fit skips its FP64 GEMM arithmetic (GP2D_DEV_SKIP: 1 = POTRF SYRKs, 2 = TRTRI
# products, 3 = both) while its chain and launch pattern stay.  Same bench command each time.
set -o pipefail
mkdir -p gpurun_out/r05_attrib
for v in prod 1 2 3; do
  lib=2d-gp_amd/gp2d/libgp2d.so; [ "$v" = prod ] || lib=tools/_p/libgp2d_skip$v.so
  GP2D_LIB=$lib GP2D_GUARD=0 timeout -k 10 300 python -u bench.py --steps 40 --warmup 3 --unpipelined-steps 10 \
    --cpu-baseline 0 --f64-steps 0 --dropin-steps 0 > gpurun_out/r05_attrib/$v.json || exit 1
done
