set -o pipefail
mkdir -p gpurun_out/r02g
for R in 0 8 32; do
  echo "== GP2D_RESERVE_CUS=$R" >> gpurun_out/r02g/reserve.log
  GP2D_RESERVE_CUS=$R timeout -k 10 200 python -u tools/probe_fit.py 4096 16384 >> gpurun_out/r02g/reserve.log 2>&1 || exit 1
done
