# headline bench under each POTRF trailing-update schedule (the pipelined job stream's fit)
set -o pipefail
R=gpurun_out/r04_bench_sched
mkdir -p $R
cd "$GRAFT_REPO_ROOT"
for v in "2 0" "4 1" "4 0" "2 0" "4 1"; do
  set -- $v
  GP2D_POTRF_G=$1 GP2D_POTRF_SPLIT=$2 timeout -k 10 200 python -u bench.py --steps 40 --warmup 3 --unpipelined-steps 10 --cpu-baseline 0 > $R/g$1s$2.json 2>> $R/err.log || exit 1
  python -c "import json;d=json.load(open('$R/g$1s$2.json'));print('G=$1 split=$2',round(d['ms_per_step'],2),round(d['unpipelined']['ms_per_step'],2),round(d['roofline']['avg_launch_ms'],4),round(d['single_job']['ms'],2))" >> $R/summary.txt
done
