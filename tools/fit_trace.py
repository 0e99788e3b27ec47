"""Per-kernel breakdown and the crit-stream timeline of one fit from a rocprofv3 kernel-trace
database (dev tool): python tools/fit_trace.py <results.db> [fit index] [crit rows]"""
import collections
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
fi = int(sys.argv[2]) if len(sys.argv) > 2 else 10
nrows = int(sys.argv[3]) if len(sys.argv) > 3 else 14
rows = con.execute("select name, start, end, queue_id, grid_x from kernels order by start").fetchall()
starts = [i for i, r in enumerate(rows) if "assemble_vec" in r[0]]
a = starts[fi]
b = starts[fi + 1] if fi + 1 < len(starts) else len(rows)
seg = rows[a:b]
t0 = seg[0][1]
t1 = max(r[2] for r in seg)
agg = collections.defaultdict(lambda: [0, 0.0])
for r in seg:
    agg[r[0].split("(")[0][-40:] + " q%s" % r[3]][0] += 1
    agg[r[0].split("(")[0][-40:] + " q%s" % r[3]][1] += (r[2] - r[1]) / 1e3
print("fit %d: wall %.2f ms, %d kernels" % (fi, (t1 - t0) / 1e6, len(seg)))
for k, v in sorted(agg.items(), key=lambda x: -x[1][1]):
    print("  %-50s %4d %9.1f us  avg %.1f" % (k, v[0], v[1], v[1] / v[0]))
diag = [r for r in seg if "potrf_diag" in r[0]]
print("  potrf span %.2f ms" % ((diag[-1][2] - t0) / 1e6))
crit = [r for r in seg if r[3] == diag[0][3]]
for lo in (0, len(crit) // 2):
    for r in crit[lo:lo + nrows]:
        print("    %-32s %8.1f +%7.1f  grid %d" % (r[0].split("(")[0][-30:], (r[1] - t0) / 1e3, (r[2] - r[1]) / 1e3, r[4]))
