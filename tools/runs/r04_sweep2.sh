# config E: batches of 8 settings on two streams (batch g+1's chain beside batch g's gradients)
set -o pipefail
R=gpurun_out/r04_sweep2
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_batched.py tests/test_gpu_lml.py -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --config E --cpu-baseline 0 > $R/configE_$i.json 2> $R/configE_$i.err || exit 1
done
timeout -k 10 300 python -u bench.py --config E --cpu-baseline 0 --sweep-batch 16 > $R/configE_b16.json 2> $R/configE_b16.err || exit 1
