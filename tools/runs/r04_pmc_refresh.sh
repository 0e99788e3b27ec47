# refresh the int8 GEMM's PMC record at HEAD (after the IgemmZ prologue): clock + MFMA busy,
# FETCH_SIZE, WRITE_SIZE in separate passes on the unpipelined bench (tools/profile_round.sh step 1)
set -euo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04_pmc_refresh
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="bench.py --steps 1 --warmup 1 --cpu-baseline 0 --pipeline 0 --variance ozaki"
csv() { find "$1" -name "*counter_collection.csv" | head -n 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -f csv -d "$OUT/pmc_clock" -o run -- python3 $B > "$OUT/pmc_clock.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/pmc_fetch" -o run -- python3 $B > "$OUT/pmc_fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT/pmc_write" -o run -- python3 $B > "$OUT/pmc_write.log" 2>&1
python3 tools/pmc_igemm.py "$(csv "$OUT/pmc_clock")" "$(csv "$OUT/pmc_fetch")" "$(csv "$OUT/pmc_write")" "$OUT/pmc_traffic_ozaki.json" > /dev/null
cat "$OUT/pmc_traffic_ozaki.json"
