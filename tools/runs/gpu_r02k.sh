set -o pipefail
mkdir -p gpurun_out/r02k
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02k/gpu_tests.log 2>&1
