set -o pipefail
R=gpurun_out/r04_dfit3
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/trace -o run -- python -u tools/probe_dfit.py --sizes 16384 --reps 1 --emulate 8 > $R/trace.log 2>&1 || exit 1
