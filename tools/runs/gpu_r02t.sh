set -o pipefail
mkdir -p gpurun_out/r02t
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="bench.py --cpu-baseline 0 --steps 20"
timeout -k 10 200 python -u $B > gpurun_out/r02t/base.json 2>/dev/null && \
GP2D_FIT_PRIORITY=low timeout -k 10 200 python -u $B > gpurun_out/r02t/fitlow.json 2>/dev/null && \
GP2D_PREDICT_PRIORITY=high timeout -k 10 200 python -u $B > gpurun_out/r02t/predhigh.json 2>/dev/null && \
GP2D_FIT_PRIORITY=low GP2D_PREDICT_PRIORITY=high timeout -k 10 200 python -u $B > gpurun_out/r02t/both.json 2>/dev/null && \
timeout -k 10 200 python -u $B --pipeline 0 > gpurun_out/r02t/nopipe.json 2>/dev/null
