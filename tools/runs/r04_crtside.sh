# CRT stream (chunk c's CRT + finalize beside chunk c+1's K* kernel): parity, then A/B in the bench
set -o pipefail
R=gpurun_out/r04_crtside
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_ozaki.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || exit 1
for i in 1 2; do
  GP2D_OZ_CRT_SIDE=1 timeout -k 10 200 python -u bench.py --steps 60 --warmup 3 --cpu-baseline 0 > $R/on_$i.json 2> $R/on_$i.err || exit 1
  GP2D_OZ_CRT_SIDE=0 timeout -k 10 200 python -u bench.py --steps 60 --warmup 3 --cpu-baseline 0 > $R/off_$i.json 2> $R/off_$i.err || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/prof -o trace -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline 0 --unpipelined-steps 0 > $R/prof_bench.json 2> $R/prof.err
