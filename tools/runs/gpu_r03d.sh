# round 3, call d: single-stream owner panel — distributed-fit GPU tests + probe
set -o pipefail
R=gpurun_out/r03d; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 240 --timeout-method thread -k "distributed_fit" > $R/dfit_tests.log 2>&1
rc=$?; echo "dfit tests rc $rc"; tail -3 $R/dfit_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u tools/probe_dfit.py > $R/probe_dfit.log 2>&1; echo "probe rc $?"; tail -2 $R/probe_dfit.log
