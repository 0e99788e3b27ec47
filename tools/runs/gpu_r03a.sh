# round 3, call a: full GPU suite, int8 vendor yardstick, phase-order probe, default bench
set -o pipefail
R=gpurun_out/r03a; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $R/gpu_tests.log 2>&1
rc=$?; echo "tests rc $rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/yardstick_int8.py > $R/yardstick.log 2>&1 && \
timeout -k 10 300 python -u tools/probe_phases.py --jobs 10 > $R/phases.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $R/bench.json 2> $R/bench.err
