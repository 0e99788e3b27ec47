# config B with 8 / 16 / 32 fits per batched factorisation (engine.auto_fit_batch caps at 8)
set -o pipefail
R=gpurun_out/r04_bfit16
mkdir -p $R
cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  for b in 8 16 32; do
    timeout -k 10 300 python -u bench.py --config B --cpu-baseline 0 --batch-fits $b > $R/B_b${b}_$i.json 2> $R/B_b${b}_$i.err || exit 1
  done
done
