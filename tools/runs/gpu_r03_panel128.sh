# round 3: 128-row skinny panel kernel (GP2D_PANEL_ROWS=128) vs the 32-row one: factor parity,
# fit times, headline bench (pipelined + unpipelined), config B
set -o pipefail
R=gpurun_out/r03p128; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
GP2D_PANEL_ROWS=128 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py -x -q --timeout 120 --timeout-method thread > $R/tests.log 2>&1
rc=$?; tail -1 $R/tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
for pr in 32 128; do
  echo "rows=$pr"; GP2D_PANEL_ROWS=$pr timeout -k 10 240 python -u tools/probe_fit.py 4096 1024 2>&1 | grep "fused=False" || exit 1
done
for pr in 32 128 32 128; do
  GP2D_PANEL_ROWS=$pr timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 > $R/head_$pr.json 2> $R/head_$pr.err || exit 1
  python3 -c "import json;d=json.load(open('$R/head_$pr.json'));print('head rows $pr', round(d['value']), round(d['ms_per_step'],2), round(d['roofline']['avg_launch_ms'],4), round(d['unpipelined']['ms_per_step'],2), round(d['single_job']['ms'],2))"
done
for pr in 32 128; do
  GP2D_PANEL_ROWS=$pr timeout -k 10 200 python -u bench.py --config B --steps 100 --warmup 5 --unpipelined-steps 0 --cpu-baseline 0 > $R/B_$pr.json 2> $R/B_$pr.err || exit 1
  python3 -c "import json;d=json.load(open('$R/B_$pr.json'));print('B rows $pr', round(d['value']), round(d['ms_per_step'],3))"
done
