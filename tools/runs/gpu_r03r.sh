# round 3, call r: diagonal-kernel phase breakdown, fit times (N=4096, 16384), kernel trace of N=4096 fits
set -o pipefail
R=gpurun_out/r03r; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 ./tools/microbench/diag_bench > $R/diag_bench.txt 2>&1 || exit 1
cat $R/diag_bench.txt
timeout -k 10 240 python -u tools/probe_fit.py 4096 16384 > $R/probe_fit.txt 2>&1 || exit 1
cat $R/probe_fit.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/prof -o fit -- python -u tools/probe_fit.py 4096 > $R/prof.log 2>&1 || exit 1
find $R/prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-160
