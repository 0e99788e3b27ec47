# round 3, call y: TRTRI products split at K/2 where one round of long-K tiles would run
# (trtri_ksplit): factor parity (LAPACK, fused = potrf + trtri bit for bit), fit times, trace
set -o pipefail
R=gpurun_out/r03y; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py tests/test_gpu_lml.py -x -q --timeout 120 --timeout-method thread > $R/tests.log 2>&1
rc=$?; tail -1 $R/tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 240 python -u tools/probe_fit.py 4096 16384 1024 2>&1 | grep -v amdgpu.ids | tee $R/probe_fit.txt || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace -d $R/prof -o fit -- python -u tools/probe_fit.py 4096 > $R/prof.log 2>&1 || exit 1
