#!/bin/bash
# Per-variant GEMM microbench under rocprofv3: cycles (GRBM_GUI_ACTIVE/8), clock and MFMA
# busy fraction.  usage (GPU box, repo root): bash tools/microbench/pmc_clock.sh FULL V2 ...
export TMPDIR=/tmp
cd tools/microbench
for v in "$@"; do
  t=$(timeout -k 10 60 ./igemm_$v > run_$v.txt && head -n 1 run_$v.txt && tail -n 1 run_$v.txt >&2) || exit 1
  timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES -f csv -d ../../gpurun_out/pmc_$v -o run -- ./igemm_$v > /dev/null 2>&1 || exit 1
  f=$(find ../../gpurun_out/pmc_$v -name "*counter_collection.csv" | head -n 1)
  python3 - "$f" "$t" <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "igemm" in r["Kernel_Name"]:
        d[r["Counter_Name"]].append(float(r["Counter_Value"]))
cyc = sum(d["GRBM_GUI_ACTIVE"]) / len(d["GRBM_GUI_ACTIVE"]) / 8
mf = sum(d["SQ_VALU_MFMA_BUSY_CYCLES"]) / len(d["SQ_VALU_MFMA_BUSY_CYCLES"])
ms = float(sys.argv[2].split(":")[1].split("ms")[0])
print(f"{sys.argv[2]} | cycles {cyc/1e3:.0f}k clock {cyc/ms/1e6:.2f} GHz mfma-busy {mf/cyc/1024:.2f}")
PY
done
