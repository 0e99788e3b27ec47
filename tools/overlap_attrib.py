"""Which fit kernels slow the int8 variance GEMM in a pipelined job stream:
from a rocprofv3 kernel-trace database of `bench.py`, every `igemm_nt_mod_kernel` launch of the
timed (pipelined) region is classed by the fit kernels that run beside it — the trailing SYRK
(`gemm_f64_kernel<true, 0>`), the TRTRI products (`gemm_f64_kernel<false, 0>`), the
critical-path chain (`potrf_diag_kernel`, `gemm_f64_panel_kernel`) and the rest of the fit
(assembly, α, int8 preparation) — by the fraction of its duration each class overlaps.

    python tools/overlap_attrib.py <results.db> [first igemm launch of the window] [launches]

Default window: bench.py's timed region of 20 jobs (20 × 96 launches), which the three
single-job launches (3 × 96) follow.
"""
import collections
import sqlite3
import sys

CLASSES = [("syrk", lambda n: "gemm_f64_kernel<true" in n),
           ("trtri", lambda n: "gemm_f64_kernel<false" in n or "add_into" in n),
           ("chain", lambda n: "potrf_diag" in n or "gemm_f64_panel" in n),
           ("fit_other", lambda n: any(k in n for k in ("assemble_vec", "trmv", "sum_segments", "zero_upper",
                                                         "ozaki_w_", "put_diag")))]


def klass(name):
    for c, f in CLASSES:
        if f(name):
            return c
    return None


def main(db, first=None, count=20 * 96):
    con = sqlite3.connect(db)
    rows = con.execute("select name, start, end from kernels order by start").fetchall()
    ig = [(s, e) for n, s, e in rows if "igemm_nt_mod_kernel" in n]
    fit = collections.defaultdict(list)
    for n, s, e in rows:
        c = klass(n)
        if c:
            fit[c].append((s, e))
    if first is None:   # bench.py: the timed jobs, then 3 single jobs (12 moduli × 8 chunks each)
        first = max(0, len(ig) - count - 3 * 96)
    ig = ig[first:first + count]

    def overlap(a, b, ivs):
        tot = 0
        for s, e in ivs:
            if e <= a or s >= b:
                continue
            tot += min(b, e) - max(a, s)
        return tot

    # per class a sorted interval list; brute force over the window is fine (≈ 2k launches)
    lo, hi = ig[0][0], ig[-1][1]
    win = {c: [(s, e) for s, e in ivs if e > lo and s < hi] for c, ivs in fit.items()}
    buckets = collections.defaultdict(list)
    frac_sum = collections.defaultdict(float)
    total = 0.0
    for a, b in ig:
        d = b - a
        fr = {c: min(1.0, overlap(a, b, win.get(c, [])) / d) for c, _ in CLASSES}
        for c in fr:
            frac_sum[c] += fr[c] * d
        total += d
        dom = max(fr, key=fr.get)
        key = dom if fr[dom] > 0.25 else "alone"
        buckets[key].append(d / 1e3)
    print(f"{len(ig)} igemm launches, {total / 1e6:.2f} ms, avg {total / len(ig) / 1e3:.1f} us")
    for c, _ in CLASSES:
        print(f"  overlapped by {c:9s}: {frac_sum[c] / total:6.1%} of the GEMM time")
    for k in ("alone", "syrk", "trtri", "chain", "fit_other"):
        v = buckets.get(k, [])
        if v:
            v = sorted(v)
            print(f"  launches mostly beside {k:9s}: {len(v):5d}  avg {sum(v) / len(v):7.1f} us  "
                  f"median {v[len(v) // 2]:7.1f} us")
    # the displaced time: Σ (d − median alone) per class
    alone = sorted(buckets.get("alone", [])) or [0.0]
    base = alone[len(alone) // 2]
    print(f"  excess over the median lone launch ({base:.1f} us), by class:")
    for k in ("syrk", "trtri", "chain", "fit_other", "alone"):
        v = buckets.get(k, [])
        print(f"    {k:9s} {sum(x - base for x in v) / 1e3:8.2f} ms over {len(v)} launches")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None,
         int(sys.argv[3]) if len(sys.argv) > 3 else 20 * 96)
