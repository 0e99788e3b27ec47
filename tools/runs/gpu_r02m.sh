set -o pipefail
mkdir -p gpurun_out/r02m
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export GP2D_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 > gpurun_out/r02m/n2.json 2> gpurun_out/r02m/n2.err && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 2 --fit-mode bcast > gpurun_out/r02m/n2_bcast.json 2> gpurun_out/r02m/n2_bcast.err && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29543 bench.py --gpus 2 --config D --steps 2 --warmup 1 > gpurun_out/r02m/n2_D.json 2> gpurun_out/r02m/n2_D.err
