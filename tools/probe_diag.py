"""Diagonal-block kernel probe (dev tool): gp2d_potrf at n = 128 (one potrf_diag_kernel per
call, HIP events over 200 calls), engine.fit medians, and the factor W of one N_train = 4096 fit
hashed for a bit comparison between library builds (GP2D_LIB).
usage: python tools/probe_diag.py [N_train ...]"""
import ctypes
import hashlib
import os
import sys
import time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "2d-gp_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from gp2d import _native as N  # noqa: E402
from gp2d import data as D  # noqa: E402
from gp2d import engine as E  # noqa: E402

L, dev, p = N.lib(), torch.device("cuda:0"), ctypes.c_void_p
s = p(torch.cuda.current_stream(dev).cuda_stream)
rng = np.random.default_rng(1)
G = rng.normal(size=(128, 128))
A0 = torch.tensor(G @ G.T / 128 + np.eye(128), device=dev)
A, dinv, info = A0.clone(), torch.empty((1, 128, 128), dtype=torch.float64, device=dev), torch.zeros(1, dtype=torch.int32, device=dev)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
for rep in range(3):
    ev[0].record()
    for _ in range(200):
        N.check(L.gp2d_potrf(p(A.data_ptr()), 128, 128, p(dinv.data_ptr()), p(info.data_ptr()), None, 0, s), "potrf")
    ev[1].record()
    torch.cuda.synchronize()
    print(f"potrf n=128 (one diagonal kernel): {1e3 * ev[0].elapsed_time(ev[1]) / 200:.2f} us per call", flush=True)
    A.copy_(A0)
if hasattr(L, "gp2d_debug_diag_stamps"):   # dev build with tools/microbench/diag_stamps.h
    st = (ctypes.c_ulonglong * 16)()
    N.check(L.gp2d_potrf(p(A.data_ptr()), 128, 128, p(dinv.data_ptr()), p(info.data_ptr()), None, 0, s), "potrf")
    torch.cuda.synchronize()
    L.gp2d_debug_diag_stamps(st)
    print("phase cycles (load P0 U0 P1 U1 P2 U2 P3 B C E dinv):", [st[i + 1] - st[i] for i in range(12)],
          "total", st[12] - st[0], flush=True)
    A.copy_(A0)

ks = E.KernelSpec(kind="df", l_df=5.0)
for i, ntr in enumerate([int(a) for a in sys.argv[1:]] or [4096]):
    x1, x2, u, v = D.synthetic_tracks(ntr, seed=2016)
    x = torch.tensor(np.stack([x1, x2], 1), device=dev)
    y = torch.tensor(np.concatenate([u, v]), device=dev)
    ts = []
    for r in range(7):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        gp = E.fit(ks, x, y, noise=0.0025, variance="ozaki")
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    print(f"fit N={ntr}: median {1e3 * np.median(ts[1:]):.2f} ms (min {1e3 * min(ts[1:]):.2f})", flush=True)
    if i == 0:
        N.check(L.gp2d_potrf(p(A.data_ptr()), 128, 128, p(dinv.data_ptr()), p(info.data_ptr()), None, 0, s), "potrf")
        for name, t in (("W", gp.W), ("L128", A), ("dinv128", dinv)):
            print(f"sha256 {name}: {hashlib.sha256(t.contiguous().cpu().numpy().tobytes()).hexdigest()}", flush=True)
    del gp
