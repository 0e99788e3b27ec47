# round 3, call e: full GPU suite; rocprofv3 kernel trace of the EXACT driver bench command;
# two-rank bench rehearsal (gloo, one card) incl. the distributed-fit single job; config D on one
# GPU with the distributed single job at P = 1
set -o pipefail
R=gpurun_out/r03e; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $R/gpu_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -2 $R/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $R/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $R/bench_prof.json 2> $R/bench_prof.err
rc=$?; echo "prof rc $rc"; if [ $rc -ne 0 ]; then exit $rc; fi
python3 tools/rocprof_timed.py "$(find $R/prof -name '*kernel_trace.csv' | head -n 1)" $R/bench_prof.json $R/timed.json > /dev/null; echo "timed rc $?"
GP2D_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 4 --warmup 2 > $R/n2.json 2> $R/n2.err
echo "n2 rc $?"
timeout -k 10 400 python -u bench.py --config D --steps 2 --warmup 1 --unpipelined-steps 0 --single-job-dist 1 > $R/configD.json 2> $R/configD.err
echo "D rc $?"
