# config B: batched fits with batch g+1's fit under batch g's predicts (krige_jobs batch_ahead) vs back to back
set -o pipefail
R=gpurun_out/r04_batch_ahead
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_jobs.py -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --config B --cpu-baseline 0 --batch-ahead 1 > $R/ahead_$i.json 2> $R/ahead_$i.err || exit 1
  timeout -k 10 200 python -u bench.py --config B --cpu-baseline 0 --batch-ahead 0 > $R/serial_$i.json 2> $R/serial_$i.err || exit 1
  timeout -k 10 200 python -u bench.py --config B --cpu-baseline 0 --batch-ahead 1 --batch-fits 4 > $R/ahead4_$i.json 2> $R/ahead4_$i.err || exit 1
done
