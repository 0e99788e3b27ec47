# config E with 8 / 12 / 16 settings per batched factorisation; config B with the new default (16)
set -o pipefail
R=gpurun_out/r04_ebatch2
mkdir -p $R
cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  for b in 16 32 64; do
    timeout -k 10 300 python -u bench.py --config E --cpu-baseline 0 --sweep-batch $b > $R/E_b${b}_$i.json 2> $R/E_b${b}_$i.err || exit 1
  done
done

