set -o pipefail
mkdir -p gpurun_out/r02b
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r02b/configs.log 2>&1
