set -o pipefail
R=${1:-persist2}
mkdir -p gpurun_out/$R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="bench.py --steps 20 --cpu-baseline 0"
for P in 2 4 0; do
  GP2D_IGEMM_TILES_PER_WG=$P timeout -k 10 300 python -u $B > gpurun_out/$R/b_p$P.json 2> gpurun_out/$R/b_p$P.err || exit 1
done
GP2D_IGEMM_PERSIST=0 timeout -k 10 300 python -u $B > gpurun_out/$R/b_tile.json 2> gpurun_out/$R/b_tile.err
