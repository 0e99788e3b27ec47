set -o pipefail
mkdir -p gpurun_out/r02f
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02f/profD -o run -- python -u tools/probe_fit.py 16384 > gpurun_out/r02f/profD.log 2>&1
