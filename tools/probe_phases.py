"""Phase-order probe: the headline job run unpipelined (U1), then as a
pipelined krige_jobs stream (P), then unpipelined again (U2), in one process.  Per phase:
ms per job, the int8 GEMM launches' average (HIP events, gp2d_timing_*), and the caching
allocator's counters (torch.cuda.memory_stats) before and after — device allocations / frees,
alloc retries, reserved bytes.

    python tools/probe_phases.py [--jobs 10] [--ntrain 4096] [--grid 256] [--order U,P,U]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "2d-gp_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gp2d import data as D  # noqa: E402
from gp2d import engine as E  # noqa: E402

KEYS = ("num_device_alloc", "num_device_free", "num_alloc_retries", "num_sync_all_streams",
        "reserved_bytes.all.current", "allocated_bytes.all.current", "segment.all.current")


def mstats():
    s = torch.cuda.memory_stats()
    return {k: s.get(k, 0) for k in KEYS}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=10)
    ap.add_argument("--ntrain", type=int, default=4096)
    ap.add_argument("--grid", type=int, default=256)
    ap.add_argument("--order", default="U,P,U")
    ap.add_argument("--empty-cache", type=int, default=0, help="torch.cuda.empty_cache() between phases")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    x1, x2, u, v = D.synthetic_tracks(a.ntrain, seed=2016)
    xt = torch.tensor(np.stack([x1, x2], 1), device=dev)
    yt = torch.tensor(np.concatenate([u, v]), device=dev)
    _, _, xg = D.bbox_grid(x1, x2, a.grid, pad=5.0)
    xg = torch.tensor(xg, device=dev)
    spec = E.KernelSpec(kind="df", l_df=5.0)
    job = (spec, xt, yt, 0.0025, xg)

    def unpiped(k):
        for _ in range(k):
            gp = E.fit(spec, xt, yt, 0.0025, device=dev, variance="ozaki")
            E.Predictor(gp, 8192)(xg)

    def piped(k):
        for _ in E.krige_jobs([job] * k, variance="ozaki"):
            pass

    unpiped(1)
    piped(2)
    torch.cuda.synchronize()
    out = []
    for ph in a.order.split(","):
        if a.empty_cache:
            torch.cuda.empty_cache()
        before = mstats()
        E.timing_enable(True)
        E.timing_read()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        (unpiped if ph == "U" else piped)(a.jobs)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        kms, kl, _ = E.timing_read()
        E.timing_enable(False)
        after = mstats()
        rec = {"phase": ph, "ms_per_job": 1e3 * (t1 - t0) / a.jobs,
               "gemm_chunk_ms": kms / kl if kl else None,
               "delta": {k: after[k] - before[k] for k in KEYS}, "after": after}
        out.append(rec)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
