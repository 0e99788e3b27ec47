# batched fits in the back-to-back job stream (engine.krige_jobs batch_fits): job-stream and
# batched tests, config B with the library default (8 fits per batch) vs batch_fits 1, headline
set -o pipefail
R=gpurun_out/r04_batched_b
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_jobs.py tests/test_gpu_batched.py -x -v --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --config B --cpu-baseline 0 > $R/configB_batch_$i.json 2> $R/configB_batch_$i.err || exit 1
  timeout -k 10 200 python -u bench.py --config B --cpu-baseline 0 --batch-fits 1 > $R/configB_b1_$i.json 2> $R/configB_b1_$i.err || exit 1
done
timeout -k 10 200 python -u bench.py --steps 40 --warmup 2 --cpu-baseline 0 --unpipelined-steps 5 > $R/headline.json 2> $R/headline.err || exit 1
