set -o pipefail
R=${1:-rr_default}
mkdir -p gpurun_out/$R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export GP2D_DIST_BACKEND=gloo
T="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
timeout -k 10 300 $T --nproc-per-node 2 --master-port 29571 bench.py --gpus 2 --steps 8 --warmup 2 > gpurun_out/$R/n2_default.json 2> gpurun_out/$R/n2_default.err && \
timeout -k 10 300 $T --nproc-per-node 4 --master-port 29572 bench.py --gpus 4 --steps 8 --warmup 2 > gpurun_out/$R/n4_default.json 2> gpurun_out/$R/n4_default.err && \
timeout -k 10 300 $T --nproc-per-node 2 --master-port 29573 bench.py --gpus 2 --steps 4 --warmup 1 --scaling weak > gpurun_out/$R/n2_weak.json 2> gpurun_out/$R/n2_weak.err && \
timeout -k 10 300 python bench.py --steps 4 --warmup 1 --cpu-baseline 0 --unpipelined-steps 2 > gpurun_out/$R/n1.json 2> gpurun_out/$R/n1.err
