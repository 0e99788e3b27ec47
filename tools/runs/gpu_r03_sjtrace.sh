# round 3: kernel traces of N=4096 fits issued from the current (null) stream and from
# high-priority side streams in one process (tools/probe_single_job.py PROBE_ONLY)
set -o pipefail
R=$GRAFT_REPO_ROOT/gpurun_out/r03sj2; mkdir -p $R
cd /tmp && export TMPDIR=/tmp
export PROBE_ONLY=main,side,side2,normal,main
timeout -k 10 240 rocprofv3 --kernel-trace -f csv -d $R/seq -o trace -- python3 $GRAFT_REPO_ROOT/tools/probe_single_job.py 4096 256 > $R/seq.log 2>&1 || exit 1
grep "fit alone" $R/seq.log
