# round 3, call b: distributed factor (one job over ranks) — GPU tests, one-process probe
set -o pipefail
R=gpurun_out/r03b; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 240 --timeout-method thread -k "distributed_fit" > $R/dfit_tests.log 2>&1
rc=$?; echo "dfit tests rc $rc"; tail -3 $R/dfit_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/probe_dfit.py > $R/probe_dfit.log 2>&1; echo "probe rc $?"; cat $R/probe_dfit.log | tail -4
