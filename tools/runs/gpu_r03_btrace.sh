# round 3: kernel trace of config B's job stream (fits_ahead 1 and 2) — where a 4.3-5.9 ms job goes
set -o pipefail
R=gpurun_out/r03btrace; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for a in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/prof$a -o run -- python3 bench.py --config B --fits-ahead $a --steps 30 --warmup 5 --unpipelined-steps 0 --cpu-baseline 0 > $R/B$a.json 2> $R/B$a.err || exit 1
  python3 -c "import json;d=json.loads(open('$R/B$a.json').read().strip().splitlines()[-1]);print('B ahead $a', round(d['value']), round(d['ms_per_step'],3))"
done
timeout -k 10 120 python3 tools/probe_fit.py 1024 2>&1 | grep fit
