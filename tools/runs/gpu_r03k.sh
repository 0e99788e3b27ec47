# round 3, call k: POTRF with the trailing SYRK confined to k CUs (GP2D_BULK_CUS) — fit time at
# N = 4096 and 16384
set -o pipefail
R=gpurun_out/r03k; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for k in 0 192 128 96 64; do
  if [ $k -gt 0 ]; then export GP2D_BULK_CUS=$k; else unset GP2D_BULK_CUS; fi
  echo "bulk_cus=$k" >> $R/fit.log
  timeout -k 10 120 python -u tools/probe_fit.py 4096 16384 >> $R/fit.log 2>&1 || exit 1
done
cat $R/fit.log | grep -v amdgpu.ids
