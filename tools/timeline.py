"""Per-step kernel timeline from a rocprofv3 --kernel-trace CSV (dev tool).

usage: python tools/timeline.py kernel_trace.csv|results.db [first_kernel_substring] [step_index]
Splits the trace at every launch of the step's first kernel (default assemble_vec_kernel),
takes step `step_index` (default −2: the last complete one) and prints, per kernel family: launches, first start, last end
(ms from the step start) and summed duration — i.e. what overlapped with what."""
import csv
import sys
from collections import OrderedDict


def short(name):
    name = name.split("(")[0]
    for k in ("void ", "gp2d::"):
        name = name.replace(k, "")
    return name[:60]


def main(path, first="assemble_vec_kernel", index="-2"):
    rows = []
    if path.endswith(".db"):   # rocpd SQLite output (rocprofv3's default format)
        import sqlite3
        c = sqlite3.connect(path)
        for s, e, n, q in c.execute("select start, end, name, queue_id from kernels"):
            rows.append((int(s), int(e), short(n), str(q)))
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                             r.get("Queue_Id", r.get("Stream_Id", "?"))))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if first in r[2]]
    if len(starts) < 2:
        print("need ≥ 2 steps")
        return
    i = int(index)
    a, b = starts[i], starts[i + 1]
    step = rows[a:b]
    t0 = step[0][0]
    fam = OrderedDict()
    for s, e, n, q in step:
        d = fam.setdefault((n, q), [0, 1e18, 0, 0.0])
        d[0] += 1
        d[1] = min(d[1], s - t0)
        d[2] = max(d[2], e - t0)
        d[3] += e - s
    print(f"step wall {(rows[b][0] - t0) / 1e6:.3f} ms ({len(step)} kernels)")
    print(f"{'kernel':60s} {'queue':>5s} {'n':>4s} {'first':>8s} {'last':>8s} {'busy':>8s}")
    for (n, q), (c, s, e, d) in fam.items():
        print(f"{n:60s} {q:>5s} {c:4d} {s / 1e6:8.3f} {e / 1e6:8.3f} {d / 1e6:8.3f}")


if __name__ == "__main__":
    main(*sys.argv[1:])
