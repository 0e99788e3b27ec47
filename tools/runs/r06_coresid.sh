#!/bin/bash
# The CRT beside the int8 GEMM (tools/microbench/coresid.hip, built on the CPU side): each alone
# and side by side on two streams.
set -o pipefail
mkdir -p gpurun_out/r06_coresid
cd tools/microbench
timeout -k 10 180 ./coresid 5 > ../../gpurun_out/r06_coresid/coresid.json 2> ../../gpurun_out/r06_coresid/coresid.err
