set -o pipefail
R=${1:-rr_full}
mkdir -p gpurun_out/$R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export GP2D_DIST_BACKEND=gloo
T="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
timeout -k 10 400 $T --nproc-per-node 4 --master-port 29581 bench.py --gpus 4 > gpurun_out/$R/n4.json 2> gpurun_out/$R/n4.err && \
timeout -k 10 400 $T --nproc-per-node 2 --master-port 29582 bench.py --gpus 2 > gpurun_out/$R/n2.json 2> gpurun_out/$R/n2.err
