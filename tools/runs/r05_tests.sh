#!/bin/bash
# r05: the GPU suite (optionally a subset: pass pytest args), log under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
out=${OUT:-gpurun_out/r05_gpu_tests.log}
timeout -k 10 1000 python -u -m pytest ${PYTEST_X--x} -v --timeout 300 --timeout-method thread -m gpu "${@:-tests}" > "$out" 2>&1
