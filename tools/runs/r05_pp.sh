#!/bin/bash
# (the ping-pong binaries were built from igemm_pp.hpp, at commit fb5a59c)
# r05: the int8 GEMM with its wave groups in ping-pong (csrc/igemm_pp.hpp; schedule variants
# IGPP_DMA / IGPP_PRIO) vs the product kernel, microbench on random residues (triangle + 4096
# sampled outputs checked), then dense K = 4096
set -o pipefail
mkdir -p gpurun_out/r05_pp
cd tools/microbench
for b in ${PP_BINS:-igemm_FULL}; do
  timeout -k 10 90 ./$b > ../../gpurun_out/r05_pp/$b.txt 2>&1 || exit 1
  IGEMM_K=4096 timeout -k 10 90 ./$b >> ../../gpurun_out/r05_pp/$b.txt 2>&1 || exit 1
done
