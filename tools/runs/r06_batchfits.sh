#!/bin/bash
# r06: the headline job stream with batched fits (krige_jobs batch_fits / batch_ahead): b = 1 (the
# default), 2, 4 with the next batch's fit under the current batch's predicts
set -o pipefail
R=gpurun_out/r06_batchfits
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
X="--steps 40 --warmup 4 --cpu-baseline 0 --f64-steps 0 --dropin-steps 0 --unpipelined-steps 2"
for v in "b1:" "b2:--fits-ahead 0 --batch-fits 2 --batch-ahead 1" "b4:--fits-ahead 0 --batch-fits 4 --batch-ahead 1" "b8:--fits-ahead 0 --batch-fits 8 --batch-ahead 1" "b1r:"; do
  name=${v%%:*}; flags=${v#*:}
  timeout -k 10 300 python -u bench.py $X $flags > $R/$name.json 2> $R/$name.err || exit 1
done
