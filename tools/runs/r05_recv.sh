#!/bin/bash
# r05: the receive path's time, two gloo ranks on one card at the headline
# workload — receivers prepare the int8 planes from the packed payload (default) vs the round-4
# path (GP2D_RECV_UNPACK=1: full n×n W rebuilt, then prepared); the comm block carries both
set -o pipefail
mkdir -p gpurun_out/r05_recv
for v in 0 1; do
  GP2D_DIST_BACKEND=gloo GP2D_RECV_UNPACK=$v timeout -k 10 400 python3 bench.py --gpus 2 --steps 10 --warmup 3 \
    > gpurun_out/r05_recv/unpack$v.json 2> gpurun_out/r05_recv/unpack$v.err || exit 1
done
