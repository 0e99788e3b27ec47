set -o pipefail
R=${1:-round_end}
mkdir -p gpurun_out/$R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$R/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$R/smoke.txt 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/$R/bench.json 2> gpurun_out/$R/bench.err
