# round-4 profile set: PMC passes + kernel-trace summary + bench (tools/profile_round.sh), the
# exact driver bench command under a kernel trace, and one config-D fit's kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/profile_round.sh r04 ozaki > gpurun_out/r04_profile_round.log 2>&1 || exit 1
R=gpurun_out/r04_exact
mkdir -p $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $R/bench.json 2> $R/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/fitD -o run -- python3 tools/probe_potrf_sched.py --sizes 16384 --reps 2 > $R/fitD.log 2>&1 || exit 1
