# batched factorisations (gp2d_potrf_batched / gp2d_trtri_batched, engine.fit_batch,
# hyper.sweep batch): bit-identity tests, the fit/LML suites, batched fit latency, config E A/B
set -o pipefail
R=gpurun_out/r04_batched
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_batched.py tests/test_gpu_lml.py tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe_fit_batch.py --sizes 1024,4096 --batches 1,2,4,8 > $R/fit_batch.jsonl 2> $R/fit_batch.err || exit 1
timeout -k 10 300 python -u bench.py --config E --cpu-baseline 0 > $R/configE_batch.json 2> $R/configE_batch.err || exit 1
timeout -k 10 300 python -u bench.py --config E --cpu-baseline 0 --sweep-concurrent 2 > $R/configE_conc2.json 2> $R/configE_conc2.err || exit 1
