#!/bin/bash
# r05: calibration data of the ozaki accuracy guard (tools/probe_guard.py), then its GPU tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/probe_guard.py "$@" > gpurun_out/r05_guard_calib.jsonl || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_guard.py \
  tests/test_gpu_order.py tests/test_gpu_ozaki.py > gpurun_out/r05_guard_tests.log 2>&1
