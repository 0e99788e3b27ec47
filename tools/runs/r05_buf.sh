#!/bin/bash
# r05: the int8 GEMM's LDS-DMA through buffer descriptors (igemm_BUF) vs global_load_lds (igemm_FULL),
# microbench on random residues (triangle, 4096 sampled outputs checked; dense K = 4096), A B A B
set -o pipefail
mkdir -p gpurun_out/r05_buf
cd tools/microbench
for r in 1 2; do
  for b in igemm_FULL igemm_BUF; do
    timeout -k 10 90 ./$b >> ../../gpurun_out/r05_buf/$b.txt 2>&1 || exit 1
    IGEMM_K=4096 timeout -k 10 90 ./$b >> ../../gpurun_out/r05_buf/$b.txt 2>&1 || exit 1
  done
done
