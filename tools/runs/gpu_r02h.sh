set -o pipefail
R=r02h
OUT=gpurun_out/$R
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="bench.py --steps 1 --warmup 1 --cpu-baseline 0 --pipeline 0"
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -f csv -d $OUT/pmc_clock -o run -- python3 $B > $OUT/pmc_clock.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/pmc_fetch -o run -- python3 $B > $OUT/pmc_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/pmc_write -o run -- python3 $B > $OUT/pmc_write.log 2>&1 && \
python3 tools/pmc_igemm.py $(find $OUT/pmc_clock -name "*counter_collection.csv" | head -n 1) $(find $OUT/pmc_fetch -name "*counter_collection.csv" | head -n 1) $(find $OUT/pmc_write -name "*counter_collection.csv" | head -n 1) $OUT/pmc_igemm.json > /dev/null
