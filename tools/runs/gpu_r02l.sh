set -o pipefail
mkdir -p gpurun_out/r02l
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export GP2D_DIST_BACKEND=gloo GP2D_BENCH_TRACE=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 4 --warmup 1 --fit-mode auto > gpurun_out/r02l/auto.json 2> gpurun_out/r02l/auto.err && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 4 --warmup 1 --fit-mode auto --kstar-ahead 0 > gpurun_out/r02l/auto_noahead.json 2> gpurun_out/r02l/auto_noahead.err
