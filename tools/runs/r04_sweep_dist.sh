# two-rank (gloo, one card) hyper.sweep with batched factorisations vs one process
set -o pipefail
R=gpurun_out/r04_sweep_dist
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || exit 1
