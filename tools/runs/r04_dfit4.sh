# distributed factor: owned-column assembly, alpha and zeroing — parity, timing
set -o pipefail
R=gpurun_out/r04_dfit4
mkdir -p $R
cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_configs.py tests/test_gpu_bench.py -x -v -k "distributed or dfit or two_ranks or self_launch or rccl" --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe_dfit.py --sizes 4096,16384 --reps 3 --emulate 8 > $R/probe.log 2>&1 || exit 1
