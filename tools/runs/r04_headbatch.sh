# headline job stream: one fit ahead (default) vs batches of 4 / 8 fits with the next batch's
# fit under this batch's predicts
set -o pipefail
R=gpurun_out/r04_headbatch
mkdir -p $R
cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 3 --cpu-baseline 0 > $R/h_default_$i.json 2> $R/h_default_$i.err || exit 1
  for b in 4 8; do
    timeout -k 10 300 python -u bench.py --steps 40 --warmup 3 --cpu-baseline 0 --fits-ahead 0 --batch-fits $b --batch-ahead 1 > $R/h_b${b}_$i.json 2> $R/h_b${b}_$i.err || exit 1
  done
done
