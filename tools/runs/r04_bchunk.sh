# config B (library defaults) with predict chunks of 4096 / 8192 / 16384 grid points
set -o pipefail
R=gpurun_out/r04_bchunk
mkdir -p $R
cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  for c in 4096 8192 16384; do
    timeout -k 10 300 python -u bench.py --config B --cpu-baseline 0 --chunk $c > $R/B_c${c}_$i.json 2> $R/B_c${c}_$i.err || exit 1
  done
done
