#!/bin/bash
# r05: the int8 GEMM's residue-plane stores non-temporal (GP2D_IG_NTSTORE=1: microbench igemm_NT,
# dev build tools/_p/libgp2d_nt.so) vs the product, alternated: microbench launches, then the bench
set -o pipefail
mkdir -p gpurun_out/r05_nt
cd tools/microbench
for b in igemm_FULL igemm_NT igemm_FULL igemm_NT; do
  timeout -k 10 90 ./$b >> ../../gpurun_out/r05_nt/micro.txt 2>&1 || exit 1
done
cd ../..
for r in 1 2; do
  for v in prod nt; do
    lib=2d-gp_amd/gp2d/libgp2d.so; [ "$v" = prod ] || lib=tools/_p/libgp2d_$v.so
    GP2D_LIB=$lib timeout -k 10 300 python3 bench.py --steps 30 --warmup 3 --unpipelined-steps 10 --cpu-baseline 0 \
      --f64-steps 0 --dropin-steps 0 > gpurun_out/r05_nt/${v}_$r.json 2> gpurun_out/r05_nt/${v}_$r.err || exit 1
  done
done
