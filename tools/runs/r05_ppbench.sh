#!/bin/bash
# r05: the headline bench with the int8 GEMM in lockstep (product) vs ping-pong (GP2D_IGEMM=pp),
# alternated twice on one box (A B A B)
set -o pipefail
mkdir -p gpurun_out/r05_ppbench
for r in 1 2; do
  for v in lockstep pp; do
    GP2D_IGEMM=$v timeout -k 10 300 python3 bench.py --steps 30 --warmup 3 --unpipelined-steps 10 --cpu-baseline 0 \
      --f64-steps 0 --dropin-steps 0 > gpurun_out/r05_ppbench/${v}_$r.json 2> gpurun_out/r05_ppbench/${v}_$r.err || exit 1
  done
done
