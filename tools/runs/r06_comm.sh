#!/bin/bash
# r06: the library's own RCCL communicator under test, then the one-GPU proxy
# of a received factor's cost to the running predict (tools/probe_recv_cost.py)
set -o pipefail
R=gpurun_out/r06_comm
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_distributed.py tests/test_gpu_bench.py > $R/tests.log 2>&1 && \
timeout -k 10 400 python -u tools/probe_recv_cost.py --jobs 40 > $R/probe.jsonl 2> $R/probe.err
