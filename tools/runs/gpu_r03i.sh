set -o pipefail
R=gpurun_out/r03i; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 800 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_bench.py -x -v --timeout 300 --timeout-method thread > $R/tests.log 2>&1
rc=$?; echo "rc $rc"; tail -4 $R/tests.log
