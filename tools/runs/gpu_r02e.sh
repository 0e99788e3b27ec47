set -o pipefail
mkdir -p gpurun_out/r02e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-baseline 0 > gpurun_out/r02e/bench.json 2> gpurun_out/r02e/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02e/prof -o run -- python -u bench.py --steps 4 --warmup 1 --cpu-baseline 0 > gpurun_out/r02e/prof.log 2>&1
