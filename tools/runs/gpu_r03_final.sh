# round 3, final profile set on the final code: PMC passes (clock / MFMA busy, FETCH, WRITE) of the
# unpipelined bench, kernel-trace summary of the default bench, the EXACT driver bench command
# under rocprofv3 --kernel-trace --stats with its timed-region average (tools/rocprof_timed.py)
set -o pipefail
R=r03final
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 bash tools/profile_round.sh $R ozaki > gpurun_out/$R.log 2>&1 || { echo "profile_round rc $?"; tail -5 gpurun_out/$R.log; exit 1; }
tail -1 gpurun_out/$R/bench_ozaki.json | cut -c1-300
O=gpurun_out/$R
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/exact -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_exact.json 2> $O/bench_exact.err || exit 1
python3 tools/rocprof_timed.py "$(find $O/exact -name '*kernel_trace.csv' | head -n 1)" $O/bench_exact.json $O/timed.json; echo "timed rc $?"
