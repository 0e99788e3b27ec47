#!/bin/bash
# r05: the int8 GEMM's ring depth on the round-5 issue path: 3 / 4 (product) / 5 stages, microbench
set -o pipefail
mkdir -p gpurun_out/r05_nst
cd tools/microbench
for b in igemm_FULL igemm_FULL5 igemm_FULL3 igemm_FULL igemm_FULL5 igemm_FULL3; do
  timeout -k 10 90 ./$b >> ../../gpurun_out/r05_nst/micro.txt 2>&1 || exit 1
  IGEMM_K=4096 timeout -k 10 90 ./$b >> ../../gpurun_out/r05_nst/micro.txt 2>&1 || exit 1
done
