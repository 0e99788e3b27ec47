#!/bin/bash
# r05: the guard's calibration on the other vector kernels (mixed, curl-free), then the BASELINE
# configs B / C / D / E at HEAD with the library defaults
set -o pipefail
mkdir -p gpurun_out/r05_configs
timeout -k 10 400 python -u tools/probe_guard.py mixed:5:0.0025 mixed:5:1e-4 mixed:12:1e-3 cf:5:0.0025 cf:5:1e-4 \
  > gpurun_out/r05_configs/guard_calib_kinds.jsonl || exit 1
for c in B C E D; do
  timeout -k 10 400 python3 bench.py --config $c --cpu-baseline 0 > gpurun_out/r05_configs/config_$c.json \
    2> gpurun_out/r05_configs/config_$c.err || exit 1
done
