#!/bin/bash
# r06: chunk c's CRT beside chunk c+1's int8 GEMMs (gp2d_ozaki_set_crt_side): the new test, the
# ozaki / jobs GPU tests, then bench.py with the side stream on / off, alternating, on one box
set -o pipefail
R=gpurun_out/r06_crtside
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ozaki.py tests/test_gpu_jobs.py > $R/tests.log 2>&1 || exit 1
for r in 1 2; do
  for c in 1 0; do
    timeout -k 10 300 python -u bench.py --steps 40 --warmup 2 --cpu-baseline 0 --f64-steps 0 --dropin-steps 0 --crt-side $c > $R/bench_c${c}_$r.json 2> $R/bench_c${c}_$r.err || exit 1
  done
done
