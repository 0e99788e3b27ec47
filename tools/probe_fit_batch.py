"""Batched fit latency: engine.fit_batch of B problems vs B engine.fit calls (one stream,
synchronised per call), per training-set size.  JSON lines: {n_train, B, batch_ms, lone_ms}."""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1024,4096")
    ap.add_argument("--batches", default="1,2,4,8")
    ap.add_argument("--variance", default="ozaki")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    for ntr in [int(v) for v in a.sizes.split(",")]:
        x1, x2, u, v = D.synthetic_tracks(ntr, seed=2016)
        x = torch.tensor(np.stack([x1, x2], 1), device=dev)
        y = torch.tensor(np.concatenate([u, v]), device=dev)
        for B in [int(v) for v in a.batches.split(",")]:
            probs = [(E.KernelSpec(kind="df", l_df=4.0 + 0.5 * b), x, y, 0.0025) for b in range(B)]
            E.fit_batch(probs, variance=a.variance)
            for k, xx, yy, nz in probs:
                E.fit(k, xx, yy, nz, variance=a.variance)
            torch.cuda.synchronize()
            tb, tl = [], []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                fits = E.fit_batch(probs, variance=a.variance)
                torch.cuda.synchronize()
                tb.append(1e3 * (time.perf_counter() - t0))
                del fits
                t0 = time.perf_counter()
                for k, xx, yy, nz in probs:
                    E.fit(k, xx, yy, nz, variance=a.variance)
                torch.cuda.synchronize()
                tl.append(1e3 * (time.perf_counter() - t0))
            print(json.dumps({"n_train": ntr, "B": B, "variance": a.variance, "batch_ms": min(tb),
                              "lone_ms": min(tl), "batch_ms_all": tb, "lone_ms_all": tl}), flush=True)


if __name__ == "__main__":
    main()
