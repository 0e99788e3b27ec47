# chain column update split (diagonal-block rows on crit, the rows below on aux beside the diagonal
# kernel): factorisation tests, fit latency per size, same-box A/B vs build/libgp2d_oldpanel.so? no:
# vs build/libgp2d_prevsplit.so (the committed sources before the split)
set -o pipefail
R=gpurun_out/r04_split_upd
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=$PWD/build/libgp2d_prevsplit.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batched.py tests/test_gpu_configs.py tests/test_gpu_jobs.py tests/test_gpu_lml.py -x -q --timeout 300 --timeout-method thread > $R/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe_potrf_sched.py --sizes 1024,2048,4096,8192,16384 > $R/fit_new.jsonl 2> $R/fit_new.err || exit 1
GP2D_LIB=$O timeout -k 10 300 python -u tools/probe_potrf_sched.py --sizes 1024,2048,4096,8192,16384 > $R/fit_old.jsonl 2> $R/fit_old.err || exit 1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 40 --warmup 2 --cpu-baseline 0 --unpipelined-steps 10 > $R/new_$i.json 2> $R/new_$i.err || exit 1
  GP2D_LIB=$O timeout -k 10 200 python -u bench.py --steps 40 --warmup 2 --cpu-baseline 0 --unpipelined-steps 10 > $R/old_$i.json 2> $R/old_$i.err || exit 1
done
for c in B E; do
  timeout -k 10 300 python -u bench.py --config $c --cpu-baseline 0 > $R/config_$c.json 2> $R/config_$c.err || exit 1
  GP2D_LIB=$O timeout -k 10 300 python -u bench.py --config $c --cpu-baseline 0 > $R/config_${c}_old.json 2> $R/config_${c}_old.err || exit 1
done
