# round 3, end of the re-entry session: full GPU suite, smoke, the exact driver bench command under
# rocprofv3 --kernel-trace --stats (timed-region GEMM average, tools/rocprof_timed.py), fit times
set -o pipefail
R=gpurun_out/r03e2; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/tests.log 2>&1 || { tail -30 $R/tests.log; exit 1; }
tail -2 $R/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $R/smoke.txt 2>&1 || { tail -20 $R/smoke.txt; exit 1; }
tail -2 $R/smoke.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $R/exact -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $R/bench_exact.json 2> $R/bench_exact.err || { tail -20 $R/bench_exact.err; exit 1; }
cut -c1-400 $R/bench_exact.json
python3 tools/rocprof_timed.py "$(find $R/exact -name '*kernel_trace.csv' | head -n 1)" $R/bench_exact.json $R/timed.json; echo "timed rc $?"
cp "$(find $R/exact -name '*kernel_stats.csv' | head -n 1)" $R/kernel_stats.csv
rm -rf $R/exact
timeout -k 10 240 python -u tools/probe_fit.py 4096 16384 > $R/fit.txt 2>&1 || exit 1
grep -v amdgpu.ids $R/fit.txt
# the K = 256 SYRK alone under PMC (clock, MFMA busy, wave states)
timeout -k 10 300 bash tools/microbench/pmc_syrk.sh > $R/pmc_syrk.txt 2>&1 || { tail -20 $R/pmc_syrk.txt; exit 1; }
cat $R/pmc_syrk.txt
