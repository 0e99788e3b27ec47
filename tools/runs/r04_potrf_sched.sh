# POTRF trailing-update schedules A/B (pairs / four panels / four panels + head-rest split)
set -o pipefail
mkdir -p gpurun_out/r04_sched
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -k "schedules or potrf" --timeout 150 --timeout-method thread > gpurun_out/r04_sched/tests.log 2>&1 || exit 1
for v in "2 0" "4 0" "4 1" "2 1"; do
  set -- $v
  GP2D_POTRF_G=$1 GP2D_POTRF_SPLIT=$2 timeout -k 10 240 python -u tools/probe_potrf_sched.py --sizes 4096,8192,16384 >> gpurun_out/r04_sched/sched.jsonl 2>> gpurun_out/r04_sched/sched.err || exit 1
done
