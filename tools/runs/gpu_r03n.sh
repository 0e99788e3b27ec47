# round 3, call n: factor stream set chosen by the caller stream — config B fits_ahead 1/2/3 (x2),
# headline default bench
set -o pipefail
R=gpurun_out/r03n; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_jobs.py -x -q --timeout 200 --timeout-method thread > $R/tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -1 $R/tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do for a in 1 2 3; do
  timeout -k 10 200 python -u bench.py --config B --fits-ahead $a --steps 100 --warmup 5 --unpipelined-steps 0 --cpu-baseline 0 > $R/B_$a.json 2>> $R/B.err || exit 1
  python3 -c "import json;d=json.load(open('$R/B_$a.json'));print('B ahead $a', d['value'], d['ms_per_step'])"
done; done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $R/head.json 2> $R/head.err || exit 1
python3 -c "import json;d=json.load(open('$R/head.json'));print('headline', d['value'], d['ms_per_step'], d['unpipelined']['ms_per_step'])"
