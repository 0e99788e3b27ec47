# round 3, call p: config B regression bisect — round-2 end (5f44290), session start (0e11326), HEAD
set -o pipefail
R=$GRAFT_REPO_ROOT/gpurun_out/r03p; mkdir -p $R
cd /tmp && export TMPDIR=/tmp
B="--config B --steps 100 --warmup 5 --unpipelined-steps 0 --cpu-baseline 0"
for w in 5f44290 0e11326; do
  cd "$GRAFT_REPO_ROOT/tools/_p/w_$w"
  timeout -k 10 200 python -u bench.py $B > $R/B_$w.json 2>> $R/B.err || exit 1
  python3 -c "import json;d=json.load(open('$R/B_$w.json'));print('B $w', d['value'], d['ms_per_step'])"
done
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u bench.py $B > $R/B_head.json 2>> $R/B.err || exit 1
python3 -c "import json;d=json.load(open('$R/B_head.json'));print('B HEAD', d['value'], d['ms_per_step'])"
timeout -k 10 60 python -u tools/probe_queues.py 12 > $R/queues.json 2>&1; cat $R/queues.json
timeout -k 10 200 python -u bench.py $B --pipeline 0 > $R/B_head_p0.json 2>> $R/B.err || exit 1
python3 -c "import json;d=json.load(open('$R/B_head_p0.json'));print('B HEAD pipeline 0', d['value'], d['ms_per_step'])"
