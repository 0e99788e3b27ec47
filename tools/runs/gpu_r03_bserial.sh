# round 3: config B strictly one job after another (--pipeline 0) vs the job stream
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03bs
for p in 0 1 0 1; do
  timeout -k 10 200 python -u bench.py --config B --pipeline $p --steps 100 --warmup 5 --unpipelined-steps 0 --cpu-baseline 0 > gpurun_out/r03bs/B_$p.json 2> gpurun_out/r03bs/B_$p.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r03bs/B_$p.json'));print('B pipeline $p', round(d['value']), round(d['ms_per_step'],3), d.get('fits_ahead'), d['api'])"
done
