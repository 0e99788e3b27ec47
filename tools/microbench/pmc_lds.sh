#!/bin/bash
# LDS counters of one igemm variant (one pass): bank conflicts vs LDS instruction cycles.
# usage (GPU box, repo root): bash tools/microbench/pmc_lds.sh FULL
export TMPDIR=/tmp
cd tools/microbench
for v in "$@"; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAVE_CYCLES SQ_BUSY_CYCLES -f csv -d ../../gpurun_out/pmcl_$v -o run -- ./igemm_$v > /dev/null 2>&1 || exit 1
  f=$(find ../../gpurun_out/pmcl_$v -name "*counter_collection.csv" | head -n 1)
  python3 - "$f" "$v" <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "igemm" in r["Kernel_Name"]:
        d[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in d.items()}
print(sys.argv[2], {k: f"{v:.4g}" for k, v in sorted(m.items())})
PY
done
