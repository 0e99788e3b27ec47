set -o pipefail
mkdir -p gpurun_out/r02c
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r02c/dist.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config D --steps 2 --warmup 1 > gpurun_out/r02c/bench_D.json 2> gpurun_out/r02c/bench_D.err && \
timeout -k 10 300 python -u bench.py --grid-global 256 --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/r02c/bench_strong256.json 2> gpurun_out/r02c/bench_strong256.err
