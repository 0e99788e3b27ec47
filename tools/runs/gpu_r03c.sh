# round 3, call c: distributed-factor probe (P=1 timings, per-rank share of P=2/8, the owners' chain)
set -o pipefail
R=gpurun_out/r03c; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u tools/probe_dfit.py > $R/probe_dfit.log 2>&1; echo "probe rc $?"; tail -4 $R/probe_dfit.log
