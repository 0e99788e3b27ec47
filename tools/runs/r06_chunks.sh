#!/bin/bash
# r06: the headline's predict chunk (grid points per K* / GEMM / CRT pass): 8192 (the default),
# 16384, 32768, 65536 (the whole grid), then 8192 again; bench.py extras off
set -o pipefail
R=gpurun_out/r06_chunks
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
X="--steps 40 --warmup 2 --cpu-baseline 0 --f64-steps 0 --dropin-steps 0 --unpipelined-steps 5"
i=0
for c in ${CHUNKS:-8192 16384 32768 65536 8192}; do
  i=$((i + 1))
  timeout -k 10 300 python -u bench.py $X --chunk $c > $R/r${i}_c$c.json 2> $R/r${i}_c$c.err || exit 1
done
