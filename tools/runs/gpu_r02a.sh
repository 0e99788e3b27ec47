set -o pipefail
mkdir -p gpurun_out/r02a
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02a/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r02a/bench.json 2> gpurun_out/r02a/bench.err
