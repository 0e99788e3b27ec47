set -o pipefail
mkdir -p gpurun_out/crt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for g in 4 8 16 4 8 16; do
  GP2D_LIB=$PWD/gpurun_libs/libgp2d_crt$g.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/crt/g$g -o run -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline 0 --unpipelined-steps 0 > gpurun_out/crt/g$g.log 2>&1 || exit 1
  python3 - gpurun_out/crt/g$g/run_kernel_stats.csv $g <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "crt_colsq" in r["Name"] or "igemm" in r["Name"]:
        print(sys.argv[2], r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e3)
PY
done
