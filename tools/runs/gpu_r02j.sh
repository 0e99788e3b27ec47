set -o pipefail
mkdir -p gpurun_out/r02j
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
(cd tools/microbench && timeout -k 10 60 ./igemm_N128 && timeout -k 10 60 ./igemm_FULL) > gpurun_out/r02j/ab.txt 2>&1 && \
timeout -k 10 300 bash tools/microbench/pmc_clock.sh FULL N128 >> gpurun_out/r02j/ab.txt 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_ozaki.py tests/test_gpu_configs.py tests/test_gpu_st.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r02j/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-baseline 0 > gpurun_out/r02j/bench128.json 2> gpurun_out/r02j/bench128.err && \
GP2D_IGEMM_TBN=256 timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-baseline 0 > gpurun_out/r02j/bench256.json 2> gpurun_out/r02j/bench256.err
