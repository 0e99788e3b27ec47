# round 3, call m: concurrent fits (factor stream-set pool) — tests, then config B fits_ahead 1/2/3
# and config E sweep concurrency 1/2/3
set -o pipefail
R=gpurun_out/r03m; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_jobs.py tests/test_gpu_lml.py -x -v --timeout 200 --timeout-method thread > $R/tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -3 $R/tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
for a in 1 2 3; do
  timeout -k 10 200 python -u bench.py --config B --fits-ahead $a --steps 100 --warmup 5 --unpipelined-steps 0 --cpu-baseline 0 > $R/B_$a.json 2>> $R/B.err || exit 1
  python3 -c "import json;d=json.load(open('$R/B_$a.json'));print('B ahead $a', d['value'], d['ms_per_step'])"
done
for c in 1 2 3; do
  timeout -k 10 200 python -u bench.py --config E --sweep-concurrent $c --steps 2 --warmup 1 > $R/E_$c.json 2>> $R/E.err || exit 1
  python3 -c "import json;d=json.load(open('$R/E_$c.json'));print('E conc $c', d['value'], d['ms_per_step'])"
done
