#!/bin/bash
# r05: Ozaki accuracy at (l, noise) settings away from the bench's
set -eo pipefail
mkdir -p gpurun_out
for lib in 2d-gp_amd/gp2d/libgp2d.so tools/_p/libgp2d_50_50.so tools/_p/libgp2d_46_45.so; do
  GP2D_LIB=$lib timeout -k 10 300 python -u tools/probe_guard.py "$@" >> gpurun_out/r05_guard.jsonl
done
