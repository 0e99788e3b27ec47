set -o pipefail
R=${1:-epi}
mkdir -p gpurun_out/$R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 bash tools/microbench/pmc_clock.sh OLDEPI FULL OLDEPI FULL > gpurun_out/$R/clock.txt 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_ozaki.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/$R/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --cpu-baseline 0 > gpurun_out/$R/b.json 2> gpurun_out/$R/b.err
