set -o pipefail
mkdir -p gpurun_out/r02p
for C in 0 64 128 192; do
  echo "== GP2D_INV_CUS=$C" >> gpurun_out/r02p/inv.log
  GP2D_INV_CUS=$C timeout -k 10 200 python -u tools/probe_fit.py 4096 >> gpurun_out/r02p/inv.log 2>&1 || exit 1
done
