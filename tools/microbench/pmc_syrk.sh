#!/bin/bash
# The K = 256 POTRF SYRK alone (syrk_bench, SYRK_K=256) under rocprofv3 PMC: clock, MFMA busy and
# the wave-state breakdown per launch size.  usage (GPU box, repo root): bash tools/microbench/pmc_syrk.sh
export TMPDIR=/tmp
cd tools/microbench
B=./syrk_epi1
P1="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES"
P2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM"
i=0
for pass in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $pass -f csv -d ../../gpurun_out/pmcs_$i -o run -- $B > ../../gpurun_out/pmcs_$i.txt 2>&1 || exit 1
  f=$(find ../../gpurun_out/pmcs_$i -name "*counter_collection.csv" | head -n 1)
  python3 - "$f" <<'PY'
import csv, sys, collections
d = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    if "gemm_f64" in r["Kernel_Name"]:
        d[int(r["Grid_Size"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for g, c in sorted(d.items()):
    m = {k: sum(v) / len(v) for k, v in c.items()}
    if "GRBM_GUI_ACTIVE" in m:
        cyc = m["GRBM_GUI_ACTIVE"] / 8
        print(f"grid {g}: cycles {cyc/1e3:.0f}k mfma-busy {m['SQ_VALU_MFMA_BUSY_CYCLES']/cyc/1024:.3f} "
              f"sq-busy {m['SQ_BUSY_CYCLES']/cyc:.3f} waves {m['SQ_WAVES']:.0f}")
    else:
        w = m["SQ_WAVE_CYCLES"]
        print(f"grid {g}:", " ".join(f"{k[3:]}={v / w:.3f}" for k, v in sorted(m.items()) if k != "SQ_WAVE_CYCLES"))
PY
done
grep 'm=' ../../gpurun_out/pmcs_1.txt
