#!/bin/bash
# r05 first GPU call: Ozaki accuracy probe across (l, noise), then the device-ordering tests
set -o pipefail
mkdir -p gpurun_out
bash tools/runs/r05_guard.sh 5:0.0025 12:0.001 2:0.05 5:0.0001 5:0.0005 8:0.0025 12:0.0025 || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_order.py \
  tests/test_gpu_ozaki.py tests/test_gpu_jobs.py tests/test_gpu_distributed.py > gpurun_out/r05_first_tests.log 2>&1
