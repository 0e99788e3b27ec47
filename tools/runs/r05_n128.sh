#!/bin/bash
# r05: the int8 GEMM as two 256x128 workgroups per CU (independent barriers, one's epilogue under
# the other's MFMAs) re-measured on the round-5 issue path: microbench (random residues), then the
# headline bench with a dev build of libgp2d.so (-DGP2D_IG_TBN=128, tools/_p/libgp2d_n128.so) vs
# the product build, alternated
set -o pipefail
mkdir -p gpurun_out/r05_n128
cd tools/microbench
for b in igemm_FULL igemm_N128 igemm_FULL igemm_N128; do
  timeout -k 10 90 ./$b >> ../../gpurun_out/r05_n128/micro.txt 2>&1 || exit 1
  IGEMM_K=4096 timeout -k 10 90 ./$b >> ../../gpurun_out/r05_n128/micro.txt 2>&1 || exit 1
done
cd ../..
for r in 1 2; do
  for v in prod n128; do
    lib=2d-gp_amd/gp2d/libgp2d.so; [ "$v" = prod ] || lib=tools/_p/libgp2d_$v.so
    GP2D_LIB=$lib timeout -k 10 300 python3 bench.py --steps 30 --warmup 3 --unpipelined-steps 10 --cpu-baseline 0 \
      --f64-steps 0 --dropin-steps 0 > gpurun_out/r05_n128/${v}_$r.json 2> gpurun_out/r05_n128/${v}_$r.err || exit 1
  done
done
