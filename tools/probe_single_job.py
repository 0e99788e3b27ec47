"""Single-job latency probe (dev tool): one fit + grid predict, host-synchronised after every job,
issued five ways — fit on the current stream / on engine.side_stream, through krige_jobs with
fits_ahead 1 and 0, and back to back without a per-job sync — to locate the gap between bench.py's
'single_job' and 'unpipelined' readings.  Also times the fit alone on each stream.
usage: python tools/probe_single_job.py [N_train] [grid]"""
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

NTR = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
G = int(sys.argv[2]) if len(sys.argv) > 2 else 256
REPS = 6
x1, x2, u, v = D.synthetic_tracks(NTR, seed=2016)
xt = torch.tensor(np.stack([x1, x2], 1), device="cuda")
yt = torch.tensor(np.concatenate([u, v]), device="cuda")
xg = torch.tensor(D.bbox_grid(x1, x2, G, pad=5.0)[2], device="cuda")
spec = E.KernelSpec(kind="df", l_df=5.0)
job = (spec, xt, yt, 0.0025, xg)
main = torch.cuda.current_stream()
E.FUSED_INVERSE = os.environ.get("PROBE_FUSED") == "1"   # gp2d_potrf_inv instead of potrf + trtri
side = E.side_stream(xt.device)
pred = [None]


def predict(gp):
    if pred[0] is None or not pred[0].fits(gp):
        pred[0] = E.Predictor(gp, 8192)
    pred[0].gp = gp
    return pred[0](xg)


def job_main():
    gp = E.fit(spec, xt, yt, 0.0025, check=False, variance="ozaki")
    out = predict(gp)
    gp.check()
    return out


def job_side():
    side.wait_stream(main)
    with torch.cuda.stream(side):
        gp = E.fit(spec, xt, yt, 0.0025, check=False, variance="ozaki")
    main.wait_stream(side)
    gp.record_stream(main)
    out = predict(gp)
    gp.check()
    return out


def jobs_api(ahead):
    def run():
        for out in E.krige_jobs(itertools.repeat(job, 1), fits_ahead=ahead):
            pass
    return run


enq = []   # host time of each fit_only enqueue (ms)


def fit_only(stream, join=None):
    def run():
        if stream is not main:
            stream.wait_stream(main)
        t = time.perf_counter()
        with torch.cuda.stream(stream):
            gp = E.fit(spec, xt, yt, 0.0025, check=False, variance="ozaki", join=join)
        enq.append(1e3 * (time.perf_counter() - t))
        torch.cuda.synchronize()
        return gp
    return run


def timed(fn, sync_each=True):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ts = []
    t0 = time.perf_counter()
    for _ in range(REPS):
        t = time.perf_counter()
        fn()
        if sync_each:
            torch.cuda.synchronize()
            ts.append(1e3 * (time.perf_counter() - t))
    torch.cuda.synchronize()
    tot = 1e3 * (time.perf_counter() - t0) / REPS
    return tot, (min(ts) if ts else float("nan"))


print(f"N_train {NTR}, grid {G}^2, {REPS} reps (ms per job: mean, min)")
normal = torch.cuda.Stream(xt.device)
side2 = E.side_stream(xt.device)
only = os.environ.get("PROBE_ONLY")   # e.g. 'main,side': those fit-alone cases only, in order (kernel traces)
if only:
    for case in only.split(","):
        enq.clear()
        name, _, j = case.partition("+")   # 'side+join': fit(join=True)
        tot, mn = timed(fit_only({"main": main, "side": side, "side2": side2, "normal": normal}[name], join=bool(j) or None))
        print(f"  fit alone, {case}: {tot:8.2f} {mn:8.2f}   host enqueue {np.mean(enq[2:]):6.2f} ms", flush=True)
        if os.environ.get("GP2D_LIB", "").endswith("libgp2d_chain.so"):   # last fit's diagonal-kernel chain
            import ctypes
            nb = 2 * NTR // 128
            buf = (ctypes.c_ulonglong * (2 * nb))()
            E.N.lib().gp2d_debug_chain_stamps(buf, 2 * nb)
            st = np.array(buf[:], dtype=np.float64).reshape(nb, 2) / 100.0   # µs (100 MHz)
            dur, gap = st[:, 1] - st[:, 0], st[1:, 0] - st[:-1, 1]
            print(f"      chain {st[-1, 1] - st[0, 0]:8.1f} us: diag avg {dur.mean():6.1f} us, gap avg "
                  f"{gap.mean():6.1f} us (first half {gap[:nb // 2].mean():6.1f}, second {gap[nb // 2:].mean():6.1f})",
                  flush=True)
    sys.exit(0)
for name, fn, se in [("fit alone, current stream", fit_only(main), True),
                     ("fit alone, side stream", fit_only(side), True),
                     ("fit alone, second side stream", fit_only(side2), True),
                     ("fit alone, normal-priority pool stream", fit_only(normal), True),
                     ("fit alone, current stream (again)", fit_only(main), True),
                     ("job, fit on current stream", job_main, True),
                     ("job, fit on side stream", job_side, True),
                     ("krige_jobs 1 job, fits_ahead 1", jobs_api(1), True),
                     ("krige_jobs 1 job, fits_ahead 0", jobs_api(0), True),
                     ("jobs back to back, current stream, no per-job sync", job_main, False),
                     ("job, fit on current stream (again)", job_main, True)]:
    tot, mn = timed(fn, se)
    print(f"  {name:55s} {tot:8.2f} {mn:8.2f}", flush=True)
