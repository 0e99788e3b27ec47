# round 3, call o: opt-in factor stream sets — config B fits_ahead 1/2/3 at GPU_MAX_HW_QUEUES 4 and 16
set -o pipefail
R=gpurun_out/r03o; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_jobs.py tests/test_gpu_lml.py -x -q --timeout 200 --timeout-method thread > $R/tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -1 $R/tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
for q in 4 16; do for a in 1 2 3; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u bench.py --config B --fits-ahead $a --steps 100 --warmup 5 --unpipelined-steps 0 --cpu-baseline 0 > $R/B_$q_$a.json 2>> $R/B.err || exit 1
  python3 -c "import json;d=json.load(open('$R/B_$q_$a.json'));print('B hwq $q ahead $a', d['value'], d['ms_per_step'])"
done; done
