# round 3: job stream with the next fit queued after this job's predict and joined on the host
# (GP2D_JOBS_JOIN=1) vs queued before it with the caller's wait pending (0); headline config
# (the GP2D_JOBS_JOIN=1 variant was measured no faster and removed from engine.krige_jobs; kept as the record)
set -o pipefail
R=gpurun_out/r03jj; mkdir -p $R
export GP2D_JOBS_JOIN=1
timeout -k 10 200 python -u -m pytest tests/test_gpu_jobs.py -x -q --timeout 120 --timeout-method thread > $R/tests.log 2>&1 || { tail -20 $R/tests.log; exit 1; }
tail -1 $R/tests.log
for i in 1 2; do
  for j in 0 1; do
    GP2D_JOBS_JOIN=$j timeout -k 10 300 python -u bench.py --cpu-baseline 0 > $R/b_${j}_$i.json 2> $R/b_${j}_$i.err || exit 1
    python3 -c "import json;d=json.load(open('$R/b_${j}_$i.json'));print('join $j run $i: %.4e pts/s %.2f ms/job frac %.3f single %.1f ms' % (d['value'], d['ms_per_step'], d['roofline']['frac'], d['single_job']['ms']))"
  done
done
