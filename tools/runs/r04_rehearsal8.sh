# N = 8 rehearsal on the one card: bench.py --gpus 8 starts 8 rank processes itself (gloo: RCCL
# refuses two ranks per device), then the headline size; correctness of the N = 8 code paths
# (round-robin fits, panel broadcasts of the distributed single job, ranks that own no
# super-column), not a speed measurement
set -o pipefail
R=gpurun_out/r04_rehearsal8
mkdir -p $R
cd "$GRAFT_REPO_ROOT"
GP2D_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 8 --ntrain 1024 --grid 128 --steps 8 --warmup 1 > $R/n8_small.json 2> $R/n8_small.err || exit 1
GP2D_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 8 --steps 8 --warmup 1 > $R/n8_headline.json 2> $R/n8_headline.err || exit 1
GP2D_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 4 --steps 8 --warmup 1 > $R/n4_headline.json 2> $R/n4_headline.err || exit 1
