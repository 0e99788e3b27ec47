"""Kernels a rocprofv3 kernel trace shows between bench.py's two trace marks (GP2D_TRACE_MARKS=1:
trace_mark_kernel tag 1 at t0, tag 2 after the timed jobs were queued) — the timed region's kernel
mix, and any kernel that is not the engine's own (a framework kernel on the hot path).
usage: python tools/timed_kernels.py <kernel_trace.csv> [out.json]"""
import collections
import csv
import json
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
name = "Kernel_Name" if "Kernel_Name" in rows[0] else "kernel_name"
ks, ke = ("Start_Timestamp", "End_Timestamp") if "Start_Timestamp" in rows[0] else ("start_timestamp", "end_timestamp")
marks = sorted(int(r[ks]) for r in rows if "trace_mark_kernel" in r[name])
if len(marks) < 2:
    sys.exit("need two trace_mark_kernel dispatches (run bench.py with GP2D_TRACE_MARKS=1)")
t0, t1 = marks[0], marks[1]
# the second mark is queued after the last timed job: everything that STARTS between them
# belongs to the timed jobs, plus the kernels still running on other streams at the second mark
inside = [r for r in rows if t0 <= int(r[ks]) <= t1 and "trace_mark_kernel" not in r[name]]
agg = collections.OrderedDict()
for r in sorted(inside, key=lambda r: int(r[ks])):
    n = r[name].split("(")[0]
    a = agg.setdefault(n, [0, 0])
    a[0] += 1
    a[1] += int(r[ke]) - int(r[ks])
foreign = {n: c for n, (c, _) in agg.items() if not ("gp2d::" in n or "__amd_rocclr" in n)}
out = {"window_ms": (t1 - t0) / 1e6, "kernels": {n: {"calls": c, "busy_ms": d / 1e6} for n, (c, d) in agg.items()},
       "non_engine_kernels": foreign}
print(json.dumps(out, indent=1))
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
