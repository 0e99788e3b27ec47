# round 3, call g: the multi-rank code paths under the REAL RCCL backend on one GPU
# (GP2D_FORCE_COLLECTIVES=1, torchrun --nproc-per-node 1): round-robin stream, broadcasts,
# the distributed single job (panel broadcasts, all_gather_into_tensor, all_reduce)
set -o pipefail
R=gpurun_out/r03g; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export GP2D_FORCE_COLLECTIVES=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 1 --steps 4 --warmup 2 > $R/rccl1.json 2> $R/rccl1.err
echo "headline rc $?"; tail -c 1500 $R/rccl1.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29572 bench.py --gpus 1 --config D --steps 2 --warmup 1 > $R/rccl1_D.json 2> $R/rccl1_D.err
echo "D rc $?"; tail -c 1500 $R/rccl1_D.json
