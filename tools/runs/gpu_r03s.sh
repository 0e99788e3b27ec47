# round 3, call s: block-lower 82 KB LDS diagonal kernel (fits beside one SYRK workgroup):
# diag_bench vs the register kernel, factor parity tests, fit times, kernel trace of N=4096 fits
set -o pipefail
R=gpurun_out/r03s; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 ./tools/microbench/diag_bench > $R/diag_bench.txt 2>&1 || exit 1
cat $R/diag_bench.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_distributed.py -x -q --timeout 120 --timeout-method thread > $R/tests.log 2>&1
rc=$?; tail -3 $R/tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 240 python -u tools/probe_fit.py 4096 16384 > $R/probe_fit.txt 2>&1 || exit 1
cat $R/probe_fit.txt
timeout -k 10 240 rocprofv3 --kernel-trace -d $R/prof -o fit -- python -u tools/probe_fit.py 4096 > $R/prof.log 2>&1 || exit 1
