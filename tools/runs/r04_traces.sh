# Kernel traces: config D's fit (engine.fit, fit_distributed P = 1, one rank's P = 8 share) and
# a pipelined headline job stream (which fit kernels slow the int8 GEMM)
set -o pipefail
R=gpurun_out/r04_traces
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/dfit -o run -- python -u tools/probe_dfit.py --sizes 16384 --reps 1 --emulate 8 > $R/dfit.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/bench -o run -- python -u bench.py --steps 20 --warmup 2 --unpipelined-steps 4 --cpu-baseline 0 > $R/bench.json 2> $R/bench.err || exit 1
