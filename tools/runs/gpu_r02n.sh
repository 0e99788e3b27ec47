set -o pipefail
mkdir -p gpurun_out/r02n
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export GP2D_DIST_BACKEND=gloo GP2D_BENCH_TRACE=1
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
timeout -k 10 200 $R --master-port 29551 bench.py --gpus 2 --pipeline 0 --steps 4 --cpu-baseline 0 > gpurun_out/r02n/p0.json 2> gpurun_out/r02n/p0.err && \
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 $R --master-port 29552 bench.py --gpus 2 --pipeline 0 --steps 4 > gpurun_out/r02n/p0_q8.json 2> gpurun_out/r02n/p0_q8.err && \
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 $R --master-port 29553 bench.py --gpus 2 --steps 4 > gpurun_out/r02n/p1_q8.json 2> gpurun_out/r02n/p1_q8.err
