"""HBM traffic per launch of the dominant kernel from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE), corrected per /opt/skills/guides/MI355X_MICROARCH.md §HBM:
FETCH_SIZE (KiB) reports half of the bytes of 16-B-per-lane coalesced reads on gfx950
(doubled here); WRITE_SIZE (KiB) is exact for 16-B streaming stores.

usage: python tools/pmc_traffic.py FETCH_CSV WRITE_CSV OUT_JSON [kernel-substring] [n] [ncols]
"""
import csv
import json
import sys


def per_launch(path, counter, pattern):
    vals = []
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] == counter and pattern in row["Kernel_Name"]:
            vals.append(float(row["Counter_Value"]))
    return vals


def main():
    fetch_csv, write_csv, out = sys.argv[1:4]
    pat = sys.argv[4] if len(sys.argv) > 4 else "gemm_f64_kernel<false, 1>"
    n = int(sys.argv[5]) if len(sys.argv) > 5 else 8192
    ncols = int(sys.argv[6]) if len(sys.argv) > 6 else 16384
    f = per_launch(fetch_csv, "FETCH_SIZE", pat)
    w = per_launch(write_csv, "WRITE_SIZE", pat)
    fetch_b = 2.0 * 1024.0 * sum(f) / len(f)
    write_b = 1024.0 * sum(w) / len(w)
    if "igemm" in pat:  # int8 residue planes: W lower half + K* chunk (read) + residue plane (written)
        alg = 1.0 * (n * (n + 256) / 2 + n * ncols + n * ncols)
    else:               # fp64: W lower half + K* chunk + partials
        alg = 8.0 * (n * (n + 128) / 2 + n * ncols + (n // 128) * ncols)
    res = {"kernel": pat, "launches_fetch": len(f), "launches_write": len(w),
           "fetch_bytes_per_launch_raw": 1024.0 * sum(f) / len(f), "fetch_bytes_per_launch": fetch_b,
           "write_bytes_per_launch": write_b, "hbm_bytes_per_launch": fetch_b + write_b,
           "algorithmic_bytes_per_launch": alg, "traffic_over_algorithmic": (fetch_b + write_b) / alg,
           "correction": "FETCH_SIZE x2 (gfx950 16-B/lane reads), KiB->B"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
