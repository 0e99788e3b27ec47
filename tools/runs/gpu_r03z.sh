# round 3, call z: POTRF look-ahead 2 (GP2D_POTRF_LA=2: block columns k+3, k+4 updated on aux, the
# SYRK over columns >= k+5 no longer on the chain) vs the current schedule
set -o pipefail
R=gpurun_out/r03z; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
GP2D_POTRF_LA=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py -x -q --timeout 120 --timeout-method thread > $R/tests.log 2>&1
rc=$?; tail -1 $R/tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
for la in 1 2 1 2; do
  echo "la=$la"; GP2D_POTRF_LA=$la timeout -k 10 240 python -u tools/probe_fit.py 4096 16384 1024 2>&1 | grep -v amdgpu.ids || exit 1
done
GP2D_POTRF_LA=2 timeout -k 10 240 rocprofv3 --kernel-trace -d $R/prof -o fit -- python -u tools/probe_fit.py 4096 > $R/prof.log 2>&1 || exit 1
