# round 3, call v: factor parity on the final diagonal kernel; int8 GEMM ring depth at the bench
# configuration (GP2D_IGEMM_NST 4 vs 5); config E settings in flight (1/2/3); config B fits ahead (1/2)
set -o pipefail
R=gpurun_out/r03v; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $R/tests.log 2>&1
rc=$?; tail -1 $R/tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
for v in 4 5 4 5; do
  GP2D_IGEMM_NST=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 > $R/nst$v.json 2> $R/nst$v.err || exit 1
  python3 -c "import json;d=json.load(open('$R/nst$v.json'));print('nst $v', round(d['value']), round(d['ms_per_step'],2), round(d['roofline']['avg_launch_ms'],4), round(d['roofline']['frac'],4), round(d['unpipelined']['ms_per_step'],2), round(d['unpipelined']['avg_launch_ms'],4), round(d['unpipelined']['roofline_frac'],4))"
done
for c in 1 2 3; do
  timeout -k 10 300 python -u bench.py --config E --sweep-concurrent $c --cpu-baseline 0 > $R/E_$c.json 2> $R/E_$c.err || exit 1
  python3 -c "import json;d=json.load(open('$R/E_$c.json'));print('E conc $c', d['value'], d['unit'], d['ms_per_step'])"
done
for a in 1 2; do
  timeout -k 10 200 python -u bench.py --config B --fits-ahead $a --steps 100 --warmup 5 --unpipelined-steps 0 --cpu-baseline 0 > $R/B_$a.json 2> $R/B_$a.err || exit 1
  python3 -c "import json;d=json.load(open('$R/B_$a.json'));print('B ahead $a', round(d['value']), round(d['ms_per_step'],3))"
done
