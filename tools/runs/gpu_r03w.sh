# round 3, call w: counter list; wave-state breakdown of the int8 GEMM at the bench configuration
set -o pipefail
R=gpurun_out/r03w; mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 60 rocprofv3 -L > $R/counters.txt 2>&1 || true
B="bench.py --steps 1 --warmup 1 --cpu-baseline 0 --pipeline 0 --unpipelined-steps 0"
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -f csv -d $R/pmc_waves -o run -- python3 $B > $R/pmc_waves.log 2>&1 || exit 1
ls -R $R/pmc_waves | head
