# round 3, call j: the shared-card phase-order effect: two processes on the
# one card, each running unpipelined → pipelined → unpipelined jobs, memory stats per phase
set -o pipefail
R=gpurun_out/r03j; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 python -u tools/probe_phases.py --jobs 8 > $R/p0.log 2>&1 &
P0=$!
timeout -k 10 240 python -u tools/probe_phases.py --jobs 8 > $R/p1.log 2>&1 &
P1=$!
wait $P0; r0=$?; wait $P1; r1=$?
echo "rc $r0 $r1"; cat $R/p0.log $R/p1.log | grep phase | cut -c1-200
