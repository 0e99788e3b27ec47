#!/bin/bash
# r05: the int8 GEMM's LDS-DMA through buffer descriptors (BUF) and the wave-uniform wave index +
# offset-field fragment reads (V2): microbench variants (random residues, triangle + dense K = 4096),
# then the headline bench with dev builds of libgp2d.so (tools/_p/libgp2d_buf.so: BUF;
# libgp2d_buf2.so: BUF + V2) vs the product build, alternated
set -o pipefail
mkdir -p gpurun_out/r05_bufbench
cd tools/microbench
for b in igemm_FULL igemm_BUF igemm_V2 igemm_BUF2 igemm_FULL igemm_BUF2; do
  timeout -k 10 90 ./$b >> ../../gpurun_out/r05_bufbench/micro.txt 2>&1 || exit 1
  IGEMM_K=4096 timeout -k 10 90 ./$b >> ../../gpurun_out/r05_bufbench/micro.txt 2>&1 || exit 1
done
cd ../..
for r in 1 2; do
  for v in prod buf2 buf; do
    lib=2d-gp_amd/gp2d/libgp2d.so; [ "$v" = prod ] || lib=tools/_p/libgp2d_$v.so
    GP2D_LIB=$lib timeout -k 10 300 python3 bench.py --steps 30 --warmup 3 --unpipelined-steps 10 --cpu-baseline 0 \
      --f64-steps 0 --dropin-steps 0 > gpurun_out/r05_bufbench/${v}_$r.json 2> gpurun_out/r05_bufbench/${v}_$r.err || exit 1
  done
done
