# POTRF schedules, round 2: G = 8 (K = 1024) and the small sizes
set -o pipefail
mkdir -p gpurun_out/r04_sched2
cd "$GRAFT_REPO_ROOT"
for v in "2 0" "4 1" "8 1" "8 0"; do
  set -- $v
  GP2D_POTRF_G=$1 GP2D_POTRF_SPLIT=$2 timeout -k 10 240 python -u tools/probe_potrf_sched.py --sizes 1024,2048,4096,8192,16384 >> gpurun_out/r04_sched2/sched.jsonl 2>> gpurun_out/r04_sched2/sched.err || exit 1
done
