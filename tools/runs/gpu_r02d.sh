set -o pipefail
mkdir -p gpurun_out/r02d
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "potrf" --timeout 120 --timeout-method thread > gpurun_out/r02d/potrf.log 2>&1 && \
timeout -k 10 300 python -u tools/probe_fit.py 4096 16384 > gpurun_out/r02d/probe_fit.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/r02d/bench.json 2> gpurun_out/r02d/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02d/prof -o run -- python -u bench.py --steps 3 --warmup 1 --cpu-baseline 0 > gpurun_out/r02d/prof.log 2>&1
