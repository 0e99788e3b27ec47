"""The dominant kernel's average duration over bench.py's TIMED region, from a rocprofv3
--kernel-trace of the exact bench command (the roofline must reproduce
from profiles/).  bench.py's one-rank run launches, in order: `warmup` + `unpipelined_steps`
unpipelined jobs, `warmup` pipelined warmup jobs, the `steps` timed jobs, then the single-job
reps; every job launches the same number of int8 GEMMs (nmod × chunks), so the timed region
is a fixed index range of the kernel's dispatches.

    python tools/rocprof_timed.py <kernel_trace.csv> <bench.json> [out.json]
    python tools/rocprof_timed.py profiles/r03_bench_exact_igemm_dispatches.csv profiles/r03_bench_exact_prof.json
"""
import csv
import json
import sys


def main():
    trace, bench = sys.argv[1], sys.argv[2]
    b = json.loads(open(bench).read().strip().splitlines()[-1])
    roof = b["roofline"]
    per_job = roof["launches"] // b["steps"]
    up = (b.get("unpipelined") or {}).get("steps", 0)
    warm = b["warmup"]
    durs = []
    with open(trace) as f:
        rows = list(csv.DictReader(f))
    if "duration_ns" in rows[0]:   # the reduced per-dispatch file kept in profiles/ (GEMM only, in order)
        rows = [{"Kernel_Name": "igemm_nt_mod_kernel", "Start_Timestamp": r["start_ns"],
                 "End_Timestamp": str(int(r["start_ns"]) + int(r["duration_ns"]))} for r in rows]
    key_s = "Start_Timestamp" if "Start_Timestamp" in rows[0] else "start_timestamp"
    key_e = "End_Timestamp" if "End_Timestamp" in rows[0] else "end_timestamp"
    key_n = "Kernel_Name" if "Kernel_Name" in rows[0] else "kernel_name"
    rows.sort(key=lambda r: int(r[key_s]))
    marks = [int(r[key_s]) for r in rows if "trace_mark_kernel" in r[key_n]]
    starts = []
    for r in rows:
        if "igemm_nt_mod_kernel" in r[key_n]:
            durs.append((int(r[key_e]) - int(r[key_s])) * 1e-6)
            starts.append(int(r[key_s]))
    skip_up = warm * per_job
    up_rng = (skip_up, skip_up + up * per_job)
    t_lo = up_rng[1] + warm * per_job
    t_rng = (t_lo, t_lo + b["steps"] * per_job)
    if len(marks) >= 2:   # bench.py GP2D_TRACE_MARKS=1: the launches that start inside the marks
        idx = [i for i, t in enumerate(starts) if marks[0] <= t <= marks[1]]
        if len(idx) != b["steps"] * per_job:
            print(f"warning: {len(idx)} launches between the marks, expected {b['steps'] * per_job}", file=sys.stderr)
        t_rng = (idx[0], idx[-1] + 1)

    def avg(a, z):
        seg = durs[a:z]
        return sum(seg) / len(seg) if seg else None
    out = {"launches_total": len(durs), "per_job": per_job,
           "timed_range": t_rng, "timed_avg_ms": avg(*t_rng),
           "unpipelined_range": up_rng, "unpipelined_avg_ms": avg(*up_rng),
           "bench_avg_launch_ms": roof["avg_launch_ms"],
           "bench_unpipelined_avg_launch_ms": (b.get("unpipelined") or {}).get("avg_launch_ms"),
           "ops_per_launch": roof["ops_per_launch"], "peak_tops": roof["peak"]}
    if out["timed_avg_ms"]:
        out["frac_from_trace"] = roof["ops_per_launch"] / (out["timed_avg_ms"] * 1e-3) / 1e12 / roof["peak"]
    if out["unpipelined_avg_ms"]:
        out["unpipelined_frac_from_trace"] = roof["ops_per_launch"] / (out["unpipelined_avg_ms"] * 1e-3) / 1e12 / \
            roof["peak"]
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(s + "\n")


if __name__ == "__main__":
    main()
