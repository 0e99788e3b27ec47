# one N_train = 4096 fit under a kernel trace after the panel-shape change (tools/fit_trace.py)
set -o pipefail
R=gpurun_out/r04_fit4096
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace -d $R/tr -o run -- python3 tools/probe_potrf_sched.py --sizes 4096 > $R/fit.log 2>&1 || exit 1
