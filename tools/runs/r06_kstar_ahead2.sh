#!/bin/bash
# r06: bench.py --kstar-ahead 1 after the single_job fix (its step() reps no longer overlap)
set -o pipefail
R=gpurun_out/r06_kstar_ahead2
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-baseline 0 --f64-steps 0 --dropin-steps 0 --unpipelined-steps 10 --kstar-ahead 1 > $R/a1.json 2> $R/a1.err
