# new panel shapes (product) vs the previous 32x128 panels (build/libgp2d_oldpanel.so) on one box:
# headline pipelined + unpipelined, fit times
set -o pipefail
R=gpurun_out/r04_panel_ab
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=$PWD/build/libgp2d_oldpanel.so
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 60 --warmup 2 --cpu-baseline 0 --unpipelined-steps 10 > $R/new_$i.json 2> $R/new_$i.err || exit 1
  GP2D_LIB=$O timeout -k 10 200 python -u bench.py --steps 60 --warmup 2 --cpu-baseline 0 --unpipelined-steps 10 > $R/old_$i.json 2> $R/old_$i.err || exit 1
done
timeout -k 10 200 python -u tools/probe_potrf_sched.py --sizes 1024,4096 > $R/fit_new.jsonl 2> $R/fit_new.err || exit 1
GP2D_LIB=$O timeout -k 10 200 python -u tools/probe_potrf_sched.py --sizes 1024,4096 > $R/fit_old.jsonl 2> $R/fit_old.err || exit 1
