"""Where a single N_train = 4096 fit's 12.4 ms go, by parts timed alone (dev tool, r06): the
Morton sort of the training points, the assembly, POTRF, TRTRI, α, the Ozaki preparation + guard,
and the whole engine.fit — each the median of 10 host-synchronised runs after warm-up.
usage: python tools/probe_fit_parts.py [N_train]"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "2d-gp_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gp2d import data as D  # noqa: E402
from gp2d import engine as E  # noqa: E402

NTR = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
dev = torch.device("cuda", 0)
E.warm_streams(dev)
x1, x2, u, v = D.synthetic_tracks(NTR, seed=2016)
X = torch.tensor(np.stack([x1, x2], 1), device=dev)
y = torch.tensor(np.concatenate([u, v]), device=dev)
spec = E.KernelSpec(kind="df", l_df=5.0)
L = E.N.lib()
P = E._ptr
s = E._stream_handle(dev)
npad, n = E.fit_layout(spec, NTR, "ozaki")
perm, Xs = E.morton_sort(X)
A = torch.empty((n, n), dtype=torch.float64, device=dev)
A0 = torch.empty_like(A)
dinv = torch.empty((n // 128, 128, 128), dtype=torch.float64, device=dev)
info = torch.zeros(1, dtype=torch.int32, device=dev)
wb = int(L.gp2d_trtri_workspace(n))
work = torch.empty(wb // 8 + 1, dtype=torch.float64, device=dev)
desc = spec.desc()


def med(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(1e3 * (time.perf_counter() - t0))
    return float(np.median(ts))


def assemble():
    E.N.check(L.gp2d_assemble(P(Xs), NTR, npad, P(Xs), NTR, npad, ctypes.byref(desc), 0.0025, 2, P(A0), n, s), "asm")


def potrf():
    A.copy_(A0)
    E.N.check(L.gp2d_potrf(P(A), n, n, P(dinv), P(info), None, 0, s), "potrf")


def copy_only():
    A.copy_(A0)


def trtri():
    E.N.check(L.gp2d_trtri(P(A), n, n, P(dinv), P(work), wb, s), "trtri")


assemble()
potrf()
Wsave = A.clone()


def trtri_fresh():
    A.copy_(Wsave)
    trtri()


out = {"n_train": NTR, "morton_sort_ms": med(lambda: E.morton_sort(X)), "assemble_ms": med(assemble),
       "copy_ms": med(copy_only), "potrf_plus_copy_ms": med(potrf), "trtri_plus_copy_ms": med(trtri_fresh),
       "fit_ozaki_ms": med(lambda: E.fit(spec, X, y, 0.0025, variance="ozaki")),
       "fit_f64_ms": med(lambda: E.fit(spec, X, y, 0.0025, variance="f64"))}
print(out, flush=True)
