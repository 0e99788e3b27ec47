set -o pipefail
R=gpurun_out/r03h; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench.py -x -v --timeout 300 --timeout-method thread > $R/bench_tests.log 2>&1
rc=$?; echo "rc $rc"; tail -6 $R/bench_tests.log
