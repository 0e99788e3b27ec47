# round 3: the other BASELINE configurations and the FP64 engine on the final code (one GPU)
set -o pipefail
R=gpurun_out/r03cfg; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u bench.py --config C --steps 20 --warmup 3 --cpu-baseline 0 > $R/C.json 2> $R/C.err || exit 1
timeout -k 10 300 python -u bench.py --variance f64 --steps 10 --warmup 2 --unpipelined-steps 5 --cpu-baseline 0 > $R/f64.json 2> $R/f64.err || exit 1
timeout -k 10 500 python -u bench.py --config D --steps 3 --warmup 1 --unpipelined-steps 1 --single-job-dist 1 --cpu-baseline 0 > $R/D.json 2> $R/D.err || exit 1
for f in C f64 D; do python3 -c "import json;d=json.load(open('$R/$f.json'));print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], (d.get('unpipelined') or {}).get('ms_per_step'), (d.get('single_job') or {}))"; done
