#!/bin/bash
# r06: the new parity tests (every grid point of the headline / C, the guard on mixed and curl-free,
# SURVEY's config E share, the lower-block assembly) and the changed suites, then the default bench
# and config E / C lines
set -o pipefail
R=gpurun_out/r06_parity
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_guard.py tests/test_gpu_configs.py tests/test_gpu_jobs.py \
  tests/test_gpu_batched.py tests/test_gpu_dropin.py -k "not every_rank_shard" > $R/tests.log 2>&1
rc=$?
timeout -k 10 400 python -u bench.py > $R/bench.json 2> $R/bench.err && \
timeout -k 10 300 python -u bench.py --config E > $R/config_E.json 2> $R/config_E.err && \
timeout -k 10 300 python -u bench.py --config C --f64-steps 0 --dropin-steps 0 > $R/config_C.json 2> $R/config_C.err
exit $rc
