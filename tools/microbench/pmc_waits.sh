#!/bin/bash
# Wave-state breakdown of one igemm variant (SQ counters, one pass):
# usage (GPU box, repo root): bash tools/microbench/pmc_waits.sh FULL
export TMPDIR=/tmp
cd tools/microbench
for v in "$@"; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM -f csv -d ../../gpurun_out/pmcw_$v -o run -- ./igemm_$v > /dev/null 2>&1 || exit 1
  f=$(find ../../gpurun_out/pmcw_$v -name "*counter_collection.csv" | head -n 1)
  python3 - "$f" "$v" <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "igemm" in r["Kernel_Name"]:
        d[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in d.items()}
w = m["SQ_WAVE_CYCLES"]
print(sys.argv[2], " ".join(f"{k[3:]}={v / w:.3f}" for k, v in sorted(m.items()) if k != "SQ_WAVE_CYCLES"), f"wave_cycles={w:.3e}")
PY
done
