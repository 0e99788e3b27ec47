# round 3: hardware queues for concurrent factorisations — config E settings in flight 1/2 and
# config B fits ahead 2/3 at GPU_MAX_HW_QUEUES 16 (the box default is 4 per priority level)
set -o pipefail
R=gpurun_out/r03hwq; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in 1 2; do
  GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python -u bench.py --config E --sweep-concurrent $c --cpu-baseline 0 > $R/E16_$c.json 2> $R/E16_$c.err || exit 1
  python3 -c "import json;d=json.load(open('$R/E16_$c.json'));print('E hwq16 conc $c', round(d['value'],1))"
done
for a in 2 3; do
  GPU_MAX_HW_QUEUES=16 timeout -k 10 200 python -u bench.py --config B --fits-ahead $a --steps 100 --warmup 5 --unpipelined-steps 0 --cpu-baseline 0 > $R/B16_$a.json 2> $R/B16_$a.err || exit 1
  python3 -c "import json;d=json.load(open('$R/B16_$a.json'));print('B hwq16 ahead $a', round(d['value']), round(d['ms_per_step'],3))"
  timeout -k 10 200 python -u bench.py --config B --fits-ahead $a --steps 100 --warmup 5 --unpipelined-steps 0 --cpu-baseline 0 > $R/B4_$a.json 2> $R/B4_$a.err || exit 1
  python3 -c "import json;d=json.load(open('$R/B4_$a.json'));print('B hwq4 ahead $a', round(d['value']), round(d['ms_per_step'],3))"
done
