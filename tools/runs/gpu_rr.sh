set -o pipefail
R=${1:-rr_rehearsal}
mkdir -p gpurun_out/$R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export GP2D_DIST_BACKEND=gloo
T="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
timeout -k 10 300 $T --master-port 29561 bench.py --gpus 2 --steps 8 --warmup 2 > gpurun_out/$R/n2_replicate.json 2> gpurun_out/$R/n2_replicate.err && \
timeout -k 10 300 $T --master-port 29562 bench.py --gpus 2 --steps 8 --warmup 2 --fit-mode rr > gpurun_out/$R/n2_rr.json 2> gpurun_out/$R/n2_rr.err && \
timeout -k 10 300 $T --master-port 29563 bench.py --gpus 2 --steps 8 --warmup 2 --fit-mode rr --grid-global 256 > gpurun_out/$R/n2_rr_strong.json 2> gpurun_out/$R/n2_rr_strong.err && \
timeout -k 10 300 python bench.py --steps 8 --warmup 2 --grid-global 256 --fit-mode rr --cpu-baseline 0 --unpipelined-steps 0 > gpurun_out/$R/n1_rr_strong.json 2> gpurun_out/$R/n1_rr_strong.err
