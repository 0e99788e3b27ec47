"""Clock, MFMA-busy fraction and HBM traffic per launch of the int8 variance GEMM at the bench
configuration, from three rocprofv3 --pmc passes (tools/profile_round.sh):
  pass 1: GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES
  pass 2: FETCH_SIZE      pass 3: WRITE_SIZE
Per /opt/skills/guides/MI355X_MICROARCH.md: effective clock = GRBM_GUI_ACTIVE / 8 / duration
(the counter sums the 8 XCDs); SQ_VALU_MFMA_BUSY_CYCLES sums the busy cycles of every SIMD
(256 CUs × 4), so busy fraction = it / (GRBM_GUI_ACTIVE / 8 × 1024); FETCH_SIZE doubled
(gfx950 16-B/lane reads), WRITE_SIZE exact.

usage: python tools/pmc_igemm.py CLOCK_CSV FETCH_CSV WRITE_CSV OUT_JSON [n] [ncols] [nmod]
"""
import csv
import json
import sys
from collections import defaultdict

PAT = "igemm_nt_mod_"   # the persistent (default) and one-tile forms


def per_dispatch(path):
    d = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if PAT in r["Kernel_Name"]:
            k = r["Dispatch_Id"]
            d[k][r["Counter_Name"]] = d[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            d[k]["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return list(d.values())


def mean(xs):
    return sum(xs) / len(xs)


def main():
    clk, fet, wri, out = sys.argv[1:5]
    n = int(sys.argv[5]) if len(sys.argv) > 5 else 8192
    ncols = int(sys.argv[6]) if len(sys.argv) > 6 else 16384
    c = per_dispatch(clk)
    cyc = [x["GRBM_GUI_ACTIVE"] / 8 for x in c]
    ghz = [cy / x["_ns"] for cy, x in zip(cyc, c)]
    busy = [x["SQ_VALU_MFMA_BUSY_CYCLES"] / (cy * 1024) for cy, x in zip(cyc, c)]
    f = [2.0 * 1024.0 * x["FETCH_SIZE"] for x in per_dispatch(fet)]
    w = [1024.0 * x["WRITE_SIZE"] for x in per_dispatch(wri)]
    alg = n * (n + 256) / 2 + 2 * n * ncols    # W lower half + K* plane read, C plane written
    res = {"kernel": PAT, "launches": len(c), "duration_ms_pmc_pass": mean([x["_ns"] for x in c]) / 1e6,
           "cycles_per_launch": mean(cyc), "clock_ghz": mean(ghz), "mfma_busy_fraction": mean(busy),
           "sq_busy_cycles_per_launch": mean([x.get("SQ_BUSY_CYCLES", 0.0) for x in c]),
           "fetch_bytes_per_launch": mean(f), "write_bytes_per_launch": mean(w),
           "hbm_bytes_per_launch": mean(f) + mean(w), "algorithmic_bytes_per_launch": alg,
           "traffic_over_algorithmic": (mean(f) + mean(w)) / alg,
           "read_over_algorithmic_read": mean(f) / (n * (n + 256) / 2 + n * ncols),
           "correction": "FETCH_SIZE x2 (gfx950 16-B/lane reads), KiB->B; clock = GRBM_GUI_ACTIVE/8/duration"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
