# CRT with the next plane group's loads issued before this group's arithmetic (build/libgp2d_crtpipe.so)
# vs the product library: parity on the variant, bench A/B, kernel trace of each
set -o pipefail
R=gpurun_out/r04_crtpipe
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
V=$PWD/build/libgp2d_crtpipe.so
GP2D_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_ozaki.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 3 --cpu-baseline 0 --unpipelined-steps 10 > $R/base_$i.json 2> $R/base_$i.err || exit 1
  GP2D_LIB=$V timeout -k 10 200 python -u bench.py --steps 100 --warmup 3 --cpu-baseline 0 --unpipelined-steps 10 > $R/pipe_$i.json 2> $R/pipe_$i.err || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $R/prof_base -o run -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline 0 --unpipelined-steps 0 > $R/prof_base.json 2> $R/prof_base.err || exit 1
GP2D_LIB=$V timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $R/prof_pipe -o run -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline 0 --unpipelined-steps 0 > $R/prof_pipe.json 2> $R/prof_pipe.err || exit 1
