# round 3, call u: trailing-update schedules A/B (GP2D_SYRK_SPLIT 0: one K=256 SYRK per pair,
# 2: panel k's K=128 SYRK from the pair's start + panel k+1's after it); factor tests in mode 2
set -o pipefail
R=gpurun_out/r03u; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
GP2D_SYRK_SPLIT=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $R/tests.log 2>&1
rc=$?; tail -2 $R/tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
for s in 0 2 0 2; do
  echo "split=$s"; GP2D_SYRK_SPLIT=$s timeout -k 10 240 python -u tools/probe_fit.py 4096 16384 2>&1 | grep -v amdgpu.ids || exit 1
done
GP2D_SYRK_SPLIT=2 timeout -k 10 240 rocprofv3 --kernel-trace -d $R/prof -o fit -- python -u tools/probe_fit.py 4096 > $R/prof.log 2>&1 || exit 1
