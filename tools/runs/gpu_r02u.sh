set -o pipefail
mkdir -p gpurun_out/r02u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u bench.py --cpu-baseline 0 --steps 20 > gpurun_out/r02u/a.json 2>/dev/null && \
timeout -k 10 200 python -u bench.py --cpu-baseline 0 --steps 20 --unpipelined-steps 20 > gpurun_out/r02u/b.json 2>/dev/null && \
timeout -k 10 200 python -u bench.py --cpu-baseline 0 --steps 20 > gpurun_out/r02u/c.json 2>/dev/null
