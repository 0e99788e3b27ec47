set -o pipefail
mkdir -p gpurun_out/r02i
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 bash tools/microbench/pmc_clock.sh FULL EPI_ONLY > gpurun_out/r02i/ablate.txt 2>&1 && \
(cd tools/microbench && timeout -k 10 60 ./igemm_FULL) >> gpurun_out/r02i/ablate.txt 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_ozaki.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r02i/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-baseline 0 > gpurun_out/r02i/bench.json 2> gpurun_out/r02i/bench.err
