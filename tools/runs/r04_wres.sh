# tiled W residue planes + scale pass without L1 on the a-priori path: full GPU suite, fit times, bench
set -o pipefail
R=gpurun_out/r04_wres
mkdir -p $R
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $R/gpu_tests.log 2>&1 || exit 1
timeout -k 10 240 python -u tools/probe_potrf_sched.py --sizes 4096,16384 > $R/fit.jsonl 2> $R/fit.err || exit 1
timeout -k 10 300 python -u bench.py --steps 40 --warmup 3 --unpipelined-steps 10 --cpu-baseline 0 > $R/bench.json 2> $R/bench.err || exit 1
