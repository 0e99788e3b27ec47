# round 3 re-entry: full GPU suite, smoke and the default bench on the restored tree
set -o pipefail
R=gpurun_out/r03rc; mkdir -p $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/tests.log 2>&1 || { tail -30 $R/tests.log; exit 1; }
tail -2 $R/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $R/smoke.txt 2>&1 || { tail -20 $R/smoke.txt; exit 1; }
tail -2 $R/smoke.txt
timeout -k 10 400 python -u bench.py > $R/bench.json 2> $R/bench.err || { tail -20 $R/bench.err; exit 1; }
cut -c1-600 $R/bench.json
# D fit (n = 32768) per-kernel breakdown: where the 418 ms go (SYRK / TRTRI / chain)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/profD -o fit -- python -u tools/probe_fit.py 16384 > $R/profD.log 2>&1 || { tail -5 $R/profD.log; exit 1; }
tail -3 $R/profD.log
find $R/profD -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-160 | head -20
