"""CU-masked predict stream for a fit-bound job stream (dev tool): config B through
engine.krige_jobs with the predicts on a stream that excludes R CUs (hipExtStreamCreateWithCUMask,
called through ctypes), the fits on the usual unmasked side streams.
usage: python tools/probe_cumask_b.py R [R ...]   (R = 0: torch's default stream)"""
import ctypes
import itertools
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "2d-gp_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gp2d import data as D  # noqa: E402
from gp2d import engine as E  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
ncu = torch.cuda.get_device_properties(0).multi_processor_count
NTR, G = (int(os.environ.get("NTR", 1024)), int(os.environ.get("GRID", 128)))
x1, x2, u, v = D.synthetic_tracks(NTR, seed=2016)
xt = torch.tensor(np.stack([x1, x2], 1), device="cuda")
yt = torch.tensor(np.concatenate([u, v]), device="cuda")
xg = torch.tensor(D.bbox_grid(x1, x2, G, pad=5.0)[2], device="cuda")
spec = E.KernelSpec(kind="df", l_df=5.0)
job = (spec, xt, yt, 0.0025, xg)


def masked_stream(r, spread):
    words = (ncu + 31) // 32
    bits = [1] * ncu
    if r > 0:
        drop = range(0, ncu, ncu // r) if spread else range(ncu - r, ncu)
        for c in list(drop)[:r]:
            bits[c] = 0
    mask = (ctypes.c_uint32 * words)()
    for c, b in enumerate(bits):
        if b:
            mask[c // 32] |= 1 << (c % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), mask)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value)


def run(r, spread, ahead, jobs=40):
    st = masked_stream(r, spread) if r > 0 else torch.cuda.current_stream()
    with torch.cuda.stream(st):
        for _ in E.krige_jobs(itertools.repeat(job, 5), fits_ahead=ahead):
            pass
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in E.krige_jobs(itertools.repeat(job, jobs), fits_ahead=ahead):
            pass
        torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t) / jobs


def serial(jobs=20):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(jobs):
        gp = E.fit(spec, xt, yt, 0.0025, variance="ozaki")
        E.predict(gp, xg)
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t) / jobs


print(f"N_train {NTR}, grid {G}², {ncu} CUs; serial fit+predict: {serial():.2f} ms per job", flush=True)
for a in sys.argv[1:]:
    r = int(a)
    for spread in ((False, True) if r > 0 else (False,)):
        for ahead in (1, 2):
            print(f"  predict stream without {r:3d} CUs ({'spread' if spread else 'last'}), fits_ahead {ahead}: "
                  f"{run(r, spread, ahead):.2f} ms per job", flush=True)
