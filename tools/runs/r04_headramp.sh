# headline job stream at the driver's shape (20 jobs, 5 warmup) and 40 jobs: one fit ahead (the
# default) vs batches of 8 ahead with ramped batch sizes 1, 2, 4, 8; config B with / without ramp
set -o pipefail
R=gpurun_out/r04_headramp
mkdir -p $R
cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  for st in 20 40; do
    timeout -k 10 300 python -u bench.py --steps $st --warmup 5 --cpu-baseline 0 > $R/h_default_s${st}_$i.json 2> $R/h_default_s${st}_$i.err || exit 1
    timeout -k 10 300 python -u bench.py --steps $st --warmup 5 --cpu-baseline 0 --fits-ahead 0 --batch-fits 8 --batch-ahead 1 --batch-ramp 1 > $R/h_b8r_s${st}_$i.json 2> $R/h_b8r_s${st}_$i.err || exit 1
  done
  timeout -k 10 300 python -u bench.py --config B --cpu-baseline 0 --batch-ramp 0 > $R/B_r0_$i.json 2> $R/B_r0_$i.err || exit 1
  timeout -k 10 300 python -u bench.py --config B --cpu-baseline 0 --batch-ramp 1 > $R/B_r1_$i.json 2> $R/B_r1_$i.err || exit 1
done
