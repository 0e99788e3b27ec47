# round 3, call t: diag kernel panel readlane depth (0/1/2/4) and load loop; trailing SYRK
# head/rest split A/B (GP2D_SYRK_SPLIT); factor tests
set -o pipefail
R=gpurun_out/r03t; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in diag_bench_rl0 diag_bench_rl1 diag_bench diag_bench_rl4; do
  timeout -k 10 60 ./tools/microbench/$v > $R/$v.txt 2>&1 || exit 1
  echo "== $v"; grep -E "blocked|phases|panels" $R/$v.txt
done
GP2D_SYRK_SPLIT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $R/tests.log 2>&1
rc=$?; tail -2 $R/tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
for s in 0 1 0 1; do
  echo "split=$s"; GP2D_SYRK_SPLIT=$s timeout -k 10 240 python -u tools/probe_fit.py 4096 16384 2>&1 | grep -v amdgpu.ids || exit 1
done
GP2D_SYRK_SPLIT=1 timeout -k 10 240 rocprofv3 --kernel-trace -d $R/prof -o fit -- python -u tools/probe_fit.py 4096 > $R/prof.log 2>&1 || exit 1
