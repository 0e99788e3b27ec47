#!/bin/bash
# r06: the guard's decisions on the mixed / curl-free settings and the headline (printed), config D
# at every rank's shard
set -o pipefail
R=gpurun_out/r06_guard
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_guard.py tests/test_gpu_configs.py -k "mixed_and_curl or decision_at or every_rank_shard or every_grid" \
  > $R/tests.log 2>&1
