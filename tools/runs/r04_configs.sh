# BASELINE configs B / C / D / E on one GPU with the library's own defaults (no bench overrides)
set -o pipefail
R=gpurun_out/r04_configs
mkdir -p $R
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u bench.py --config B --steps 100 --warmup 3 --cpu-baseline 0 > $R/B.json 2> $R/B.err || exit 1
timeout -k 10 200 python -u bench.py --config E --warmup 1 > $R/E.json 2> $R/E.err || exit 1
timeout -k 10 200 python -u bench.py --config C --steps 40 --warmup 3 --unpipelined-steps 10 --cpu-baseline 0 > $R/C.json 2> $R/C.err || exit 1
timeout -k 10 300 python -u bench.py --config D --warmup 1 --unpipelined-steps 2 --single-job-dist 1 > $R/D.json 2> $R/D.err || exit 1
