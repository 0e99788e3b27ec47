set -o pipefail
R=${1:-persist}
mkdir -p gpurun_out/$R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_ozaki.py tests/test_gpu_configs.py tests/test_gpu_jobs.py tests/test_gpu_bench.py -x -q --timeout 200 --timeout-method thread > gpurun_out/$R/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --cpu-baseline 0 > gpurun_out/$R/b.json 2> gpurun_out/$R/b.err && \
GP2D_IGEMM_PERSIST=0 timeout -k 10 300 python -u bench.py --steps 20 --cpu-baseline 0 > gpurun_out/$R/b_tile.json 2> gpurun_out/$R/b_tile.err
