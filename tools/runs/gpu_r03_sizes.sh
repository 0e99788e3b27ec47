# round 3: throughput over problem sizes (df kernel, one MI355X, pipelined job stream; N_train 1024
# uses jobs back to back like config B)
set -o pipefail
R=gpurun_out/r03sizes; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in "1024 128 0" "1024 256 0" "2048 256 1" "4096 256 1" "4096 512 1" "8192 256 1" "8192 512 1"; do
  set -- $cfg
  timeout -k 10 400 python -u bench.py --ntrain $1 --grid $2 --fits-ahead $3 --steps 8 --warmup 2 --unpipelined-steps 3 --cpu-baseline 0 > $R/n$1_g$2.json 2> $R/n$1_g$2.err || exit 1
  python3 -c "import json;d=json.load(open('$R/n$1_g$2.json'));u=d.get('unpipelined') or {};print('N_train $1 grid $2^2 ahead $3:', '%.3e pts/s' % d['value'], '%.1f ms/job' % d['ms_per_step'], 'GEMM frac %.3f' % d['roofline']['frac'], 'unpipelined %.1f ms' % (u.get('ms_per_step') or 0), 'single %.1f ms' % d['single_job']['ms'])"
done
