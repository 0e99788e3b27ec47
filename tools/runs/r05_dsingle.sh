#!/bin/bash
# r05: why config D's single_job reading (9.4 s) is 3.6x its unpipelined jobs (2.58 s): one fresh
# krige_jobs job at a time, phase times (fit, check, predict) with and without the guard
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python3 - > gpurun_out/r05_dsingle.txt 2>&1 <<'PY'
import itertools, os, sys, time
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "2d-gp_amd")]
import numpy as np, torch
from gp2d import data as D, engine as E
x1, x2, u, v = D.synthetic_tracks(16384, seed=2016)
xt = torch.tensor(np.stack([x1, x2], 1), device="cuda"); yt = torch.tensor(np.concatenate([u, v]), device="cuda")
xg = torch.tensor(D.bbox_grid(x1, x2, 512, pad=5.0)[2], device="cuda")
spec = E.KernelSpec(kind="mixed", l_df=5.0, l_cf=5.0, ratio=0.5)
def sync(): torch.cuda.synchronize(); return time.perf_counter()
for guard in (True, False, True):
    for rep in range(2):
        t0 = sync(); gp = E.fit(spec, xt, yt, 0.0025, variance="ozaki", check=False, guard=guard); t1 = sync()
        gp.check(); t2 = sync()
        pr = E.Predictor(gp, 8192); mu, var = pr(xg); t3 = sync()
        g = gp.extra.get("guard") or {}
        print(f"guard={guard} rep={rep}: fit {1e3*(t1-t0):.0f} ms, check {1e3*(t2-t1):.0f} ms, predict {1e3*(t3-t2):.0f} ms, "
              f"bits {g.get('wbits')}/{g.get('kbits')} nmod {gp.extra['ozaki'][2]}, mem {torch.cuda.memory_reserved()/2**30:.1f} GiB", flush=True)
        del gp, pr, mu, var
    t0 = sync()
    for _ in E.krige_jobs([(spec, xt, yt, 0.0025, xg)], guard=guard) if False else E.krige_jobs([(spec, xt, yt, 0.0025, xg)]): pass
    t1 = sync(); print(f"krige_jobs one job: {1e3*(t1-t0):.0f} ms", flush=True)
PY
