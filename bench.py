"""Headline benchmark: posterior grid points/s (fit + predict), N_train = 4096,
divergence-free 2-D SE vector kernel, 256×256 grid per GPU (BASELINE.json).

One "step" = one complete job: K_y assembly + POTRF + TRTRI + α + posterior mean AND
variance at every point of the job's grid.  Inputs are resident in HBM before the timed
region.  N = 1: successive jobs pipelined (engine.krige_jobs).  N > 1 (default: strong
scaling): the same 256×256 job grid sharded over the N ranks, job j fitted on rank j mod N
and its factor broadcast over RCCL (distributed.krige_jobs_sharded); --scaling weak gives
each rank its own 256×256 block with a replicated fit instead.

    python bench.py [--gpus N] [--steps K] [--warmup W]   (N > 1: starts the N ranks itself)
    torchrun --nproc-per-node N bench.py --gpus N ...     (--gpus must equal WORLD_SIZE)

Rank 0 prints ONE JSON line (the driver contract) with `roofline` (dominant
kernel: the variance contraction, timed live with HIP events on its stream) and
`cpu_baseline` (the numpy oracle on the host cores, bounded sample, N = 1 only).
"""
from __future__ import annotations

import argparse
import functools
import itertools
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "2d-gp_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

# GP2D_FORCE_COLLECTIVES=1 (tests only): take the multi-rank code paths — collectives,
# round-robin fits, the distributed single job — even at world size 1, so a one-GPU box can run
# them under the real RCCL backend (torchrun --nproc-per-node 1)
FORCE_COLLECTIVES = os.environ.get("GP2D_FORCE_COLLECTIVES") == "1"


def is_multi(ws: int) -> bool:
    return ws > 1 or FORCE_COLLECTIVES


METRIC = "posterior grid points/sec (fit+predict), N_train=4096, div-free 2D kernel"
FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 matrix (= vector) dense peak; measured 76.5 (tools/microbench)
HBM_PEAK_GBS = 8000.0
INT8_PEAK_TOPS = 5000.0   # MI355X dense int8 MFMA (2x bf16 2.5 PF); measured 4.7 POPS (tools/microbench/i8_mfma.hip)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed jobs (default 100; --config D: 4, E: 2 sweeps)")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--ntrain", type=int, default=4096)
    ap.add_argument("--grid", type=int, default=256)
    ap.add_argument("--kind", default="df")
    ap.add_argument("--grid-global", type=int, default=0,
                    help="strong scaling: ONE fixed G x G grid sharded over the ranks (0 = weak scaling, "
                         "--grid x --grid points per rank)")
    ap.add_argument("--config", default=None, choices=["B", "C", "D", "E", "E-noise"],
                    help="BASELINE.json config preset: B = df N=1024 128^2, C = mixed N=4096 256^2, "
                         "D = mixed N=16384, one 512^2 grid sharded over the ranks (strong scaling), "
                         "E = SURVEY's 64-setting (l_df, l_cf) sweep of LML + gradient at N=4096 (mixed), "
                         "settings dealt over the ranks (hyper.sweep); E-noise = the (l_df, noise) div-free sweep")
    ap.add_argument("--chunk", type=int, default=8192)
    ap.add_argument("--scaling", default="auto", choices=["auto", "weak", "strong"],
                    help="N>1: strong = the --grid x --grid job grid sharded over the ranks (auto's choice: "
                         "jobs fitted round robin, factor broadcast); weak = a --grid x --grid block per rank "
                         "(a --grid x (--grid·N) job grid)")
    ap.add_argument("--fit-mode", default=None, choices=["auto", "bcast", "replicate", "rr"],
                    help="N>1: every rank fits, no data-path collective (replicate, default); rank 0 "
                         "fits and W goes out by RCCL broadcast (bcast); whichever of the two the "
                         "warmup measured faster (auto); or job j fitted on rank j mod N only and its "
                         "factor broadcast, every rank predicting its shard of every job (rr, "
                         "distributed.krige_jobs_sharded)")
    ap.add_argument("--variance", default="ozaki", choices=["ozaki", "f64"],
                    help="variance contraction: exact INT8 Ozaki-II emulation (default) or FP64 MFMA")
    ap.add_argument("--kstar-ahead", type=int, default=-1,
                    help="ozaki: generate the K* residue planes on a side stream concurrently with the fit "
                         "(the mean stays K* alpha in fp64); 0 = inline per chunk after the fit; -1 (auto) = only while "
                         "non-root ranks wait for the factor broadcast (N>1, bcast)")
    ap.add_argument("--oz-skip", type=int, default=1,
                    help="ozaki: skip the all-zero K* slabs in the int8 GEMMs (exact; 0 = dense, for A/B)")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="issue each job's fit on a second stream, so job i+1's fit runs while job i's predict "
                         "does (the steps are independent fit+predict jobs, like the reference's per-time-window "
                         "krig.kriging loop); 0 = strictly one job after the other")
    ap.add_argument("--unpipelined-steps", type=int, default=20,
                    help="with --pipeline 1 on one rank: first time this many jobs strictly one after another "
                         "(reported under 'unpipelined', with the dominant kernel's roofline alone)")
    ap.add_argument("--cpu-baseline", type=int, default=-1,
                    help="time the numpy oracle on the host cores (N=1 only); -1 = only when N_train <= 4096")
    ap.add_argument("--cpu-sample-points", type=int, default=2048)
    ap.add_argument("--pmc-json", default=None)
    ap.add_argument("--fits-ahead", type=int, default=None,
                    help="N=1 job stream: fits in flight (engine.krige_jobs fits_ahead; default: the library's "
                         "engine.auto_fits_ahead for the job shape — 0 = each job's fit and predict back to back)")
    ap.add_argument("--batch-fits", type=int, default=None,
                    help="N=1 back-to-back job stream: fits per batched factorisation (engine.krige_jobs "
                         "batch_fits; default: the library's engine.auto_fit_batch)")
    ap.add_argument("--batch-ahead", type=int, default=None,
                    help="N=1 batched job stream: 1 = batch g+1's fit under batch g's predicts (engine.krige_jobs "
                         "batch_ahead; default: the library's)")
    ap.add_argument("--sweep-concurrent", type=int, default=None,
                    help="config E: streams the settings' fit + LML are queued on (hyper.sweep concurrent; "
                         "default: the library's hyper.auto_concurrent)")
    ap.add_argument("--sweep-batch", type=int, default=None,
                    help="config E: settings per batched factorisation (hyper.sweep batch; default: the "
                         "library's hyper.auto_batch)")
    ap.add_argument("--single-job-dist", type=int, default=0,
                    help="also time one job with distributed.fit_distributed at N = 1 (always at N > 1)")
    ap.add_argument("--f64-steps", type=int, default=5,
                    help="N = 1: also time this many jobs of the same stream on the strict FP64 engine (f64_value)")
    ap.add_argument("--dropin-steps", type=int, default=3,
                    help="N = 1: also time this many krig.Krig(...).fit(...).predict_device(grid) jobs (dropin)")
    a = ap.parse_args()
    if a.config == "B":
        a.kind, a.ntrain, a.grid = "df", 1024, 128
    elif a.config == "C":
        a.kind, a.ntrain, a.grid = "mixed", 4096, 256
    elif a.config == "D":
        a.kind, a.ntrain, a.grid_global = "mixed", 16384, 512
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if a.steps is None:   # config D: every rank owns at least two of the timed jobs' fits
        a.steps = {"D": max(4, 2 * ws), "E": 2, "E-noise": 2}.get(a.config, 100)
    if a.grid_global == 0 and is_multi(ws) and a.scaling in ("auto", "strong"):
        a.grid_global = a.grid   # N>1 default: one job grid sharded over the ranks
    if a.fit_mode is None:
        a.fit_mode = "rr" if (is_multi(ws) and a.grid_global > 0) else "replicate"
    return a


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` (N > 1) run without a launcher: start the N rank processes as ONE
    child `torch.distributed.run` (127.0.0.1 rendezvous, a free port) with this script's own
    arguments, before this process touches the GPU (the parent never initialises HIP and never
    execs), relay rank 0's JSON line to stdout and return the child's exit code.  The driver's
    command shape (`python3 bench.py --gpus N ...`) then measures N GPUs by itself; the
    reference's own parallelism is the job array, runKrig.py:7,14-17."""
    import signal
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    print(f"bench.py: --gpus {n} without WORLD_SIZE: launching {n} rank processes ({' '.join(cmd[1:7])} ...)",
          file=sys.stderr, flush=True)
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, start_new_session=True)
    try:
        for line in proc.stdout:   # rank 0 prints the one JSON line; anything else goes to stderr
            (sys.stdout if line.lstrip().startswith("{") else sys.stderr).write(line)
            sys.stdout.flush()
        return proc.wait()
    except BaseException:
        os.killpg(proc.pid, signal.SIGTERM)   # the child's own process group: the ranks go with it
        proc.wait()
        raise


def check_world(args) -> int | None:
    """World-size contract of --gpus, checked before any GPU call: returns the exit code of a
    run that must not proceed in this process (a self-launched N-rank child's, or 2 for a
    --gpus that contradicts the launcher's WORLD_SIZE), None to run here."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is None:
        return launch_ranks(args.gpus) if args.gpus > 1 else None
    if int(ws) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={ws} ranks", file=sys.stderr,
              flush=True)
        return 2
    return None


def setup_dist(args):
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if is_multi(ws):
        # one process per GPU; GP2D_DIST_BACKEND=gloo (and ranks sharing a device) only for
        # rehearsing the multi-rank path on a one-GPU box
        local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        # the library's factor streams take their hardware queues before RCCL's and torch's
        # streams are first used (engine.warm_streams; DESIGN.md §6 "bench state")
        from gp2d import engine as E
        E.warm_streams(torch.device("cuda", local))
        backend = os.environ.get("GP2D_DIST_BACKEND", "nccl")
        kw = {"device_id": torch.device("cuda", local)} if backend == "nccl" else {}
        dist.init_process_group(backend, **kw)
        if backend == "nccl":
            # the library's own RCCL communicator carries the data path (gp2d/comm.py): made here,
            # before any warmup, from an ncclUniqueId exchanged over torch.distributed's store
            from gp2d import comm as GC
            GC.get(torch.device("cuda", local))
        return dist.get_world_size(), dist.get_rank(), torch.device("cuda", local)
    from gp2d import engine as E
    E.warm_streams(torch.device("cuda", 0))
    return 1, 0, torch.device("cuda", 0)


def finish_dist():
    from gp2d import comm as GC
    dist.barrier()
    torch.cuda.synchronize()
    GC.shutdown()
    dist.destroy_process_group()


def barrier(ws):
    if is_multi(ws):
        dist.barrier()
    torch.cuda.synchronize()


def cpu_baseline(x, y, xg, kind, l, noise, sample_pts):
    """Oracle (numpy/OpenBLAS) on the host: full fit + a bounded sample of grid points,
    extrapolated linearly to the whole grid."""
    from oracle import gp2d_oracle as O
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        cores = os.cpu_count()
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp:
        cores = min(cores, int(omp))
    t0 = time.perf_counter()
    fit = O.OracleFit(x, y, kind, l, l, 1.0, noise, method="chol")
    t1 = time.perf_counter()
    fit.predict(xg[:sample_pts], chunk=sample_pts)
    t2 = time.perf_counter()
    M = xg.shape[0]
    total = (t1 - t0) + (t2 - t1) * (M / sample_pts)
    return {"value": M / total, "unit": "points/s", "cores": cores, "kind": "port",
            "sample": f"numpy oracle: full fit N_train={x.shape[0]} ({t1 - t0:.2f} s) + {sample_pts} of {M} "
                      f"grid points ({t2 - t1:.2f} s), predict extrapolated linearly; OpenBLAS threads={cores}"}


def _pmc_round(path: str, pmc: dict) -> str:
    """The round a PMC pass belongs to: its 'round' field, else the rNN prefix of the file or of
    its directory (profiles/r04_pmc_traffic_ozaki.json, gpurun_out/r04/pmc_traffic_ozaki.json)."""
    import re
    for part in (pmc.get("round"), os.path.basename(path), os.path.basename(os.path.dirname(path))):
        m = re.match(r"(r\d\d)", part or "")
        if m:
            return m.group(1)
    return "round unknown"


def config_e_settings(variant: str = "E"):
    """BASELINE config E's 64 settings.  'E' (SURVEY.md §8(d)): the mixed kernel (α = ½, noise
    0.0025) at 8 ℓ_df × 8 ℓ_cf log-spaced over [1, 10] km (ℓ_df-major); 'E-noise' (rounds 1-5's
    variant): the div-free kernel at 8 ℓ_df in [2, 12] km × 8 noise values in [1e-3, 5e-2].  The
    same grids as the committed fixtures (config_e_survey_share.npz, config_e_share.npz)."""
    if variant == "E":
        g = np.geomspace(1.0, 10.0, 8)
        return [dict(l_df=float(a), l_cf=float(b)) for a in g for b in g]
    return [dict(l_df=float(l), noise=float(nz)) for l in np.geomspace(2.0, 12.0, 8)
            for nz in np.geomspace(1e-3, 5e-2, 8)]


def run_sweep(args, ws, rank, dev):
    """Config E: one step = the whole 64-setting sweep (fit + LML + exact gradient per
    setting), settings dealt round robin over the ranks and the results all-reduced
    (hyper.sweep); value = settings per second for the whole job (strong scaling)."""
    from gp2d import data as D
    from gp2d import engine as E
    from gp2d import hyper as H
    x1, x2, u, v = D.synthetic_tracks(args.ntrain, seed=2016)
    xt = torch.tensor(np.stack([x1, x2], 1), device=dev)
    yt = torch.tensor(np.concatenate([u, v]), device=dev)
    settings = config_e_settings(args.config)
    survey = args.config == "E"
    ks = E.KernelSpec(kind="mixed", l_df=5.0, l_cf=5.0, ratio=0.5) if survey else E.KernelSpec(kind="df", l_df=5.0)

    # None: the library's default (hyper.auto_concurrent)
    conc = args.sweep_concurrent

    bsz = args.sweep_batch

    def sweep():
        return H.sweep(ks, xt, yt, settings, noise=0.0025, eval_gradient=True, device=dev, concurrent=conc,
                       batch=bsz)

    for _ in range(args.warmup):
        sweep()
    barrier(ws)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        vals, grads = sweep()
    barrier(ws)
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if is_multi(ws):
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    elapsed = float(dt.item())
    if rank == 0:
        n = 2 * E.padded_points(args.ntrain)
        # per setting: POTRF n³/3 + TRTRI n³/3 + K_y⁻¹ = WᵀW n³/3 (FP64 MFMA), the rest O(n²)
        per_gpu = len(settings) / ws * n ** 3 * args.steps / elapsed / 1e12
        grid = ("8 l_df x 8 l_cf log-spaced over [1, 10] km, mixed alpha=0.5, noise 0.0025 (SURVEY.md §8d)"
                if survey else "8 l_df in [2, 12] km x 8 noise in [1e-3, 5e-2], div-free")
        out = {
            "metric": f"hyperparameter settings/sec (fit + LML + gradient), 64-setting sweep, N_train={args.ntrain}, "
                      + ("mixed div-free + curl-free 2D kernel" if survey else "div-free 2D kernel"),
            "value": len(settings) * args.steps / elapsed, "unit": "settings/s", "n_gpus": ws, "world_size": ws,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (seeded drifter field, SURVEY.md §8d)",
            "config": {"workload": f"BASELINE config {args.config}: 64 settings ({grid}) x N_train={args.ntrain}, "
                                   f"LML + exact gradient per setting, settings dealt over {ws} GPU(s)",
                       "n_train": args.ntrain, "settings": len(settings), "parallelism": f"settings round robin x{ws}",
                       "sweep_batch": bsz if bsz is not None else
                       H.auto_batch(ks, xt, len(range(rank, len(settings), ws)), conc),
                       "sweep_concurrent": conc if conc is not None else
                       H.auto_concurrent(len(range(rank, len(settings), ws)), True)},
            "roofline": {"bound": "mfma", "achieved": per_gpu, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": per_gpu / FP64_PEAK_TFLOPS, "traffic": None,
                         "kernel": "whole sweep per GPU: POTRF + TRTRI + W^T W (n^3 FP64 flop per setting) / wall time"},
            "finite_settings": int(np.isfinite(vals).sum()),
        }
        print(json.dumps(out), flush=True)
    if is_multi(ws):
        finish_dist()


def comm_block(comm: dict, keys, per: int, ws: int, dev) -> dict:
    """The `comm` block of the N > 1 line: per collective kind, the HIP-event-timed milliseconds
    and the payload bytes this rank sent / received (distributed._timed), divided by `per` jobs,
    each the MAX over the ranks (all-reduce; every rank calls this)."""
    from gp2d import distributed as GD
    summ = GD.comm_summary(comm)
    vals = torch.tensor([[summ.get(k, {}).get(f, 0) for f in ("ms", "bytes_sent", "bytes_recv", "calls")]
                         for k in keys], dtype=torch.float64, device=dev)
    if is_multi(ws):
        dist.all_reduce(vals, op=dist.ReduceOp.MAX)
    out = {}
    for k, (ms, sent, recv, calls) in zip(keys, vals.tolist()):
        out[k] = {"ms_per_job_max_over_ranks": ms / per, "bytes_sent_per_job_max": sent / per,
                  "bytes_recv_per_job_max": recv / per, "calls_per_job": calls / per}
    return out


def single_job_distributed(args, ws, spec, xt, yt, noise, xg, m_all, dev, pred_cache, mean, var, reps):
    """One job with its FIT spread over the ranks too (distributed.fit_distributed: block-cyclic
    POTRF + TRTRI, panel broadcasts, W all-gathered), then each rank's grid shard predicted —
    the one-job multi-GPU reading of DESIGN.md §5 (config D).  One untimed warm job first."""
    from gp2d import distributed as GD
    from gp2d import engine as E

    def job():
        gp = GD.fit_distributed(spec, xt, yt, noise, dev, variance=args.variance)
        pr = pred_cache.get("pd")
        if pr is None or not pr.fits(gp):
            pr = E.Predictor(gp, args.chunk)
            pred_cache["pd"] = pr
        pr.gp = gp
        pr(xg, out=(mean, var))
        return gp

    job()
    barrier(ws)
    comm = {}
    tf = time.perf_counter()
    gp = GD.fit_distributed(spec, xt, yt, noise, dev, variance=args.variance, comm=comm)
    barrier(ws)
    fit_s = time.perf_counter() - tf
    del gp
    cblock = comm_block(comm, ("panel_bcast", "w_allgather", "alpha_allgather"), 1, ws, dev)
    ts = time.perf_counter()
    for _ in range(reps):
        job()
    barrier(ws)
    dts = torch.tensor([time.perf_counter() - ts, fit_s], dtype=torch.float64, device=dev)
    if is_multi(ws):
        dist.all_reduce(dts, op=dist.ReduceOp.MAX)
    ms = 1e3 * float(dts[0].item()) / reps
    return {"ms": ms, "value": m_all / (ms * 1e-3), "reps": reps, "fit_ms": 1e3 * float(dts[1].item()),
            "fit": f"distributed.fit_distributed over {ws} rank(s): 512-column block-cyclic POTRF + TRTRI, "
                   "panel broadcasts, W columns all-gathered",
            "comm": cblock}


def extra_readings_n1(args, spec, xt, yt, noise, xg, m_all):
    """N = 1 readings beside the headline, each timed on its own:
    * f64_value: the same job stream (engine.krige_jobs) with the strict FP64 variance engine;
    * dropin: the reference-shaped surface — krig.Krig(...).fit(X, obs) then predict_device(grid)
      (krig.py:471-574 / GP_plots.py:760-768), the variance engine its accuracy guard picks."""
    from gp2d import engine as E
    from gp2d import krig as K
    out = {}
    if args.f64_steps > 0:
        job = (spec, xt, yt, noise, xg)
        for _ in E.krige_jobs(itertools.repeat(job, 1), variance="f64", chunk=args.chunk):
            pass
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in E.krige_jobs(itertools.repeat(job, args.f64_steps), variance="f64", chunk=args.chunk):
            pass
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        out["f64_value"] = m_all * args.f64_steps / dt
        out["f64"] = {"value": m_all * args.f64_steps / dt, "ms_per_step": 1e3 * dt / args.f64_steps,
                      "steps": args.f64_steps, "api": "engine.krige_jobs(variance='f64')"}
    if args.dropin_steps > 0:
        # the drop-in object's default (variance='f64', the reference's arithmetic) and its opt-in
        # guarded int8 engine (variance='ozaki'), one job at a time each
        for key, variance in (("dropin", "ozaki"), ("dropin_f64", "f64")):
            def one():
                k = K.Krig(spec.kind, l_df=spec.l_df, l_cf=spec.l_cf, ratio=spec.ratio, noise=noise,
                           variance=variance).fit(xt, yt)
                mu, var = k.predict_device(xg)
                return k, mu, var
            k, _, _ = one()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.dropin_steps):
                k, _, _ = one()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            g = k.gp.extra.get("guard") or {}
            out[key] = {"value": m_all * args.dropin_steps / dt, "ms_per_step": 1e3 * dt / args.dropin_steps,
                        "steps": args.dropin_steps,
                        "api": f"krig.Krig(kind, l_df, noise, variance='{variance}').fit(X, obs).predict_device(grid)",
                        "variance_engine": k.variance if k.variance == "f64" else g.get("engine", "ozaki"),
                        "guard_bits": [g.get("wbits"), g.get("kbits")]}
    return out


def job_stream_shape(args, spec, m, api) -> dict:
    """fits_ahead / batch_fits / batch_ahead exactly as engine.krige_jobs resolved them for this
    job shape (None off the engine.krige_jobs path): a batch is used only with fits_ahead = 0, and
    batch_ahead only for a batch of more than one fit."""
    from gp2d import engine as E
    if api != "engine.krige_jobs":
        return {"fits_ahead": None, "batch_fits": None, "batch_ahead": None}
    fa = E.auto_fits_ahead(spec, args.ntrain, m, args.variance) if args.fits_ahead is None else args.fits_ahead
    if fa > 0:
        return {"fits_ahead": fa, "batch_fits": 1, "batch_ahead": False}
    bf = E.auto_fit_batch(spec, args.ntrain, args.variance) if args.batch_fits is None else args.batch_fits
    if bf <= 1:
        return {"fits_ahead": fa, "batch_fits": 1, "batch_ahead": False}
    ba = bool(args.batch_ahead) if args.batch_ahead is not None else \
        E.auto_batch_ahead(spec, args.ntrain, m, bf, args.variance)
    return {"fits_ahead": fa, "batch_fits": bf, "batch_ahead": ba}


def main():
    args = parse()
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    rc = check_world(args)
    if rc is not None:
        sys.exit(rc)
    ws, rank, dev = setup_dist(args)
    if args.config in ("E", "E-noise"):
        return run_sweep(args, ws, rank, dev)
    from gp2d import data as D
    from gp2d import distributed as GD
    from gp2d import engine as E
    E.N.lib().gp2d_ozaki_set_skip(int(args.oz_skip))

    G = args.grid
    x1, x2, u, v = D.synthetic_tracks(args.ntrain, seed=2016)
    x = np.stack([x1, x2], 1)
    y = np.concatenate([u, v])
    strong = args.grid_global > 0
    if strong:   # one fixed grid, sharded: per-rank work shrinks as 1/N
        G = args.grid_global
        _, _, xg_all = D.bbox_grid(x1, x2, G, pad=5.0)
    else:        # weak: each rank owns a G x G block of a G x (G N) grid
        _, _, xg_all = D.bbox_grid(x1, x2, G, pad=5.0, Gy=G * ws)
    m_all = xg_all.shape[0]
    lo, hi = D.shard_range(m_all, ws, rank)
    spec = E.KernelSpec(kind=args.kind, l_df=5.0, l_cf=5.0, ratio=1.0 if args.kind == "df" else 0.5)
    noise = 0.0025
    # inputs resident in HBM before the timed region
    xt = torch.tensor(x, device=dev)
    yt = torch.tensor(y, device=dev)
    xg = torch.tensor(xg_all[lo:hi], device=dev)
    m = hi - lo
    mean = torch.empty(2 * m, dtype=torch.float64, device=dev)
    var = torch.empty(2 * m, dtype=torch.float64, device=dev)
    pred_cache = {}
    side = E.side_stream(dev) if args.variance == "ozaki" else None
    cfg = {"mode": args.fit_mode if is_multi(ws) else "local", "ahead": False,
           "pipeline": bool(args.pipeline) and not is_multi(ws) or (bool(args.pipeline) and args.fit_mode == "replicate")
           or (is_multi(ws) and args.fit_mode == "rr"),
           "first": True}

    def set_mode(mode):
        cfg["mode"] = mode
        a = args.kstar_ahead
        cfg["ahead"] = args.variance == "ozaki" and (a == 1 or (a == -1 and is_multi(ws) and mode == "bcast"))

    stats = {}      # fits issued (engine.note_fit_issued): every timed job's fit must be issued after t0
    comm = {} if is_multi(ws) else None   # the N > 1 line's `comm` block (distributed._timed)

    fit_stream = E.side_stream(dev)
    main_stream = torch.cuda.current_stream(dev)

    def do_fit():
        if cfg["mode"] != "bcast" or rank == 0:   # bcast: rank 0 fits every job
            E.note_fit_issued(stats)
        if not cfg["pipeline"]:
            return GD.fit_sharded(spec, xt, yt, noise, dev, mode=cfg["mode"], variance=args.variance, check=False)
        # the fit is queued on its own stream behind the previous fit only, so it runs while
        # the previous job's predict (main stream) does; the predict waits for its own fit's event
        fit_stream.wait_stream(main_stream) if cfg["first"] else None
        cfg["first"] = False
        with torch.cuda.stream(fit_stream):
            gp = GD.fit_sharded(spec, xt, yt, noise, dev, mode=cfg["mode"], variance=args.variance, check=False)
        main_stream.wait_stream(fit_stream)
        return gp.record_stream(main_stream)

    def step():
        planes = None
        if cfg["ahead"]:   # K* planes depend on (X_train, grid, kernel) only: overlap them with the fit
            planes = E.kstar_planes(spec, xt, xg, noise, chunk=args.chunk, stream=side, out=pred_cache.get("k"))
            pred_cache["k"] = planes
        gp = do_fit()
        gp.check()   # status + the accuracy guard before the predict (the guard may re-prepare)
        gp.ready_on(main_stream)
        pr = pred_cache.get("p")
        if pr is None or not pr.fits(gp):
            pr = E.Predictor(gp, args.chunk)
            pred_cache["p"] = pr
        pr.gp = gp
        pr(xg, out=(mean, var), planes=planes)
        return gp

    probe = {}
    if is_multi(ws) and args.fit_mode == "auto":
        # measure one step in each mode (after a warm step of each), max over ranks, keep the faster
        for mode in ("bcast", "replicate"):
            set_mode(mode)
            step()
            barrier(ws)
            t = time.perf_counter()
            step()
            barrier(ws)
            dt_ = torch.tensor([time.perf_counter() - t], dtype=torch.float64, device=dev)
            dist.all_reduce(dt_, op=dist.ReduceOp.MAX)
            probe[mode] = 1e3 * float(dt_.item())
        set_mode(min(probe, key=probe.get))
    else:
        set_mode(cfg["mode"])
    unpiped = None
    if cfg["pipeline"] and not is_multi(ws) and args.unpipelined_steps > 0:
        # reference: the same jobs strictly one after another, measured BEFORE the timed region
        # (the dominant kernel's launch time without a concurrent fit = its roofline alone)
        cfg["pipeline"] = False
        for _ in range(args.warmup):
            step()
        barrier(ws)
        E.timing_enable(True)
        E.timing_read()
        tu0 = time.perf_counter()
        for _ in range(args.unpipelined_steps):
            step()
        barrier(ws)
        tu1 = time.perf_counter()
        ukms, uklaunch, ukflops = E.timing_read()
        E.timing_enable(False)
        unpiped = {"value": m_all * args.unpipelined_steps / (tu1 - tu0),
                   "ms_per_step": 1e3 * (tu1 - tu0) / args.unpipelined_steps, "steps": args.unpipelined_steps,
                   "kernel_ms": ukms, "kernel_launches": uklaunch, "kernel_flops": ukflops}
        cfg["pipeline"] = True
    # A job stream (engine.krige_jobs / distributed.krige_jobs_sharded) reads no job ahead before
    # its first next(), so warmup and timed jobs run on separate generators: the warmup one is
    # drained before the clock starts, and the timed one is created after t0 — every timed job's
    # fit (including the first, and at N > 1 the whole fill of the fit window) is inside the clock.
    stream, api = None, "engine.fit + Predictor"
    if cfg["mode"] == "rr":
        # the global grid on every rank; each job's fit on one rank, its shard predicted on all
        job = (spec, xt, yt, noise, torch.tensor(xg_all, device=dev))

        def stream(k):
            return GD.krige_jobs_sharded(itertools.repeat(job, k), variance=args.variance, chunk=args.chunk,
                                         stats=stats, comm=comm)
        api = "distributed.krige_jobs_sharded"
    elif cfg["pipeline"] and cfg["mode"] in ("local", "replicate") and not cfg["ahead"]:
        job = (spec, xt, yt, noise, xg)

        def stream(k):   # the shipped API for a sweep of jobs
            return E.krige_jobs(itertools.repeat(job, k), variance=args.variance, chunk=args.chunk, stats=stats,
                                fits_ahead=args.fits_ahead, batch_fits=args.batch_fits,
                                **({} if args.batch_ahead is None else {"batch_ahead": bool(args.batch_ahead)}))
        api = "engine.krige_jobs"
    trace = os.environ.get("GP2D_BENCH_TRACE") == "1"   # per-step wall times on stderr (diagnostics)

    def run_jobs(k, t_ref=None):
        it = stream(k) if stream is not None else (step() for _ in range(k))
        for i, _ in enumerate(it):
            if trace and t_ref is not None:
                torch.cuda.synchronize()
                print(f"[rank {rank}] step {i}: {1e3 * (time.perf_counter() - t_ref):.1f} ms since start",
                      file=sys.stderr, flush=True)

    # round robin: at least one warmup job per rank, so every rank has fitted before the clock
    warm = max(args.warmup, ws) if cfg["mode"] == "rr" else args.warmup
    run_jobs(warm)
    barrier(ws)
    E.timing_enable(True)
    E.timing_read()
    stats.clear()
    if comm is not None:
        comm.clear()
    marks = os.environ.get("GP2D_TRACE_MARKS") == "1"   # bracket the timed region in a kernel trace
    barrier(ws)
    t0 = time.perf_counter()
    if marks:
        E.N.lib().gp2d_trace_mark(1, E._stream_handle(dev))
    run_jobs(args.steps, t0)
    if marks:
        E.N.lib().gp2d_trace_mark(2, E._stream_handle(dev))
    barrier(ws)
    t1 = time.perf_counter()
    kms, klaunch, kflops = E.timing_read()
    E.timing_enable(False)
    # fits issued inside [t0, t1] on this rank (all of this rank's fits of the timed jobs)
    fit_times = stats.get("fit_issue_times", [])
    fits = torch.tensor([sum(t0 <= t <= t1 for t in fit_times), len(fit_times)], dtype=torch.float64, device=dev)
    dt = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if is_multi(ws):
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        dist.all_reduce(fits, op=dist.ReduceOp.SUM)
    elapsed = float(dt.item())
    ms_per_step = 1e3 * elapsed / args.steps
    value = m_all * args.steps / elapsed
    fits_expected = args.steps * (1 if cfg["mode"] in ("rr", "bcast") or not is_multi(ws) else ws)
    timed_fits = {"issued_in_window": int(fits[0].item()), "issued_total": int(fits[1].item()),
                  "expected": fits_expected, "warmup_jobs_run": warm}
    if timed_fits["issued_in_window"] != fits_expected or timed_fits["issued_total"] != fits_expected:
        raise RuntimeError(f"bench: timed region holds {timed_fits} fits, expected {fits_expected}")
    guard = (stats.get("guard") or [None])[0]   # the accuracy guard's decision for the first timed job
    comm_out = None
    if cfg["mode"] == "rr" and comm is not None:
        # every rank receives (or sends) every job's factor: bytes and HIP-event ms per job
        comm_out = comm_block(comm, ("bcast", "recv_prepare"), args.steps, ws, dev)
        comm_out["what"] = ("per timed job, MAX over ranks: the job's factor broadcast from its fitting rank (packed "
                            "W + alpha + X_train + the status block), RCCL on the comm stream under the predict; "
                            "recv_prepare: a receiving rank's int8 planes from the packed payload (no bytes)")
        from gp2d import comm as GC
        lc = GC.get(dev)
        comm_out["transport"] = ("the library's own RCCL communicator (gp2d_comm_init; gp2d_bcast on the comm stream)"
                                 if lc is not None else f"torch.distributed ({dist.get_backend()}) rehearsal")
        comm_out["library_calls"] = dict(lc.calls) if lc is not None else None

    # one job alone (unpipelined, its grid sharded over the ranks; at N > 1 fitted on rank 0 and
    # broadcast): the single-job reading beside the job-stream value
    reps = 1 if args.ntrain > 8192 else 3
    barrier(ws)
    ts = time.perf_counter()
    for _ in range(reps):
        if stream is not None:
            run_jobs(1)
        else:   # step(): its fit must wait for the previous job's predict (no overlap across reps)
            cfg["first"] = True
            step()
    barrier(ws)
    dts = torch.tensor([time.perf_counter() - ts], dtype=torch.float64, device=dev)
    if is_multi(ws):
        dist.all_reduce(dts, op=dist.ReduceOp.MAX)
    single_ms = 1e3 * float(dts.item()) / reps
    single_job = {"ms": single_ms, "value": m_all / (single_ms * 1e-3), "reps": reps,
                  "fit": "rank 0, factor broadcast" if is_multi(ws) else "local"}
    if is_multi(ws) or args.single_job_dist:
        try:
            single_job["distributed_fit"] = single_job_distributed(args, ws, spec, xt, yt, noise, xg, m_all, dev,
                                                                   pred_cache, mean, var, reps)
        except Exception as e:   # an informational reading: the timed value above stands without it
            single_job["distributed_fit"] = {"error": f"{type(e).__name__}: {e}"}

    # mean-only throughput (secondary, same fit; at most 20 jobs)
    mo_steps = min(args.steps, 20)
    barrier(ws)
    t2 = time.perf_counter()
    for _ in range(mo_steps):
        gp = GD.fit_sharded(spec, xt, yt, noise, dev, mode="replicate" if cfg["mode"] == "rr" else cfg["mode"],
                            variance=args.variance)
        if "p" not in pred_cache:   # the timed region ran through krige_jobs*: no Predictor yet
            pred_cache["p"] = E.Predictor(gp, args.chunk)
        pred_cache["p"].gp = gp
        pred_cache["p"](xg, compute_var=False, out=(mean, var))
    barrier(ws)
    t3 = time.perf_counter()
    mean_only = m_all * mo_steps / (t3 - t2)

    if rank != 0:
        if is_multi(ws):
            finish_dist()
        return

    achieved = kflops / (kms * 1e-3) / 1e12 if kms > 0 else None
    traffic = None   # the committed PMC pass was taken at the headline workload only
    headline = (args.kind, args.ntrain, G, strong) == ("df", 4096, 256, False)
    # the latest committed PMC pass of this engine (profiles/rNN_pmc_traffic_<engine>.json)
    import glob
    found = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r[0-9][0-9]_pmc_traffic_{args.variance}.json")))
    pmc_json = args.pmc_json or (found[-1] if found else "")
    traffic_source = None
    try:
        with open(pmc_json) as f:
            pmc = json.load(f)
        traffic = pmc.get("hbm_bytes_per_launch") if (headline or args.pmc_json) else None
        if traffic is not None:   # a separate builder run of rocprofv3 --pmc, not measured in this run
            traffic_source = (f"{os.path.relpath(pmc_json, ROOT)}: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes "
                              f"(separate runs, {_pmc_round(pmc_json, pmc)}) of this kernel at "
                              "this workload; not measured inside this bench run")
    except (OSError, ValueError):
        pass
    if args.variance == "ozaki":
        # dominant kernel = the nmod int8 GEMMs; executed int8 ops per launch = nmod × the
        # FP64-equivalent algorithmic count (one exact product per modulus)
        # — times the fraction the zero-slab skipping executes (all-zero K* tiles are skipped;
        # counted from the K* block flags, outside the timed region)
        nmod = int(pred_cache["p"].gp.extra["ozaki"][2])
        efrac = E.ozaki_executed_fraction(spec, xt, xg, noise, chunk=args.chunk) if args.oz_skip else 1.0
        ex = achieved * nmod * efrac if achieved else None
        roof = {"bound": "mfma", "achieved": ex, "peak": INT8_PEAK_TOPS,
                "unit": "TOP/s (int8)", "frac": (ex / INT8_PEAK_TOPS) if ex else None,
                "traffic": traffic, "traffic_source": traffic_source,
                "kernel": f"igemm_nt_mod_kernel x{nmod} moduli (Ozaki-II variance, exact)",
                "launches": klaunch * nmod, "avg_launch_ms": (kms / klaunch / nmod) if klaunch else None,
                "ops_per_launch": (kflops * efrac / klaunch) if klaunch else None,
                "executed_fraction_of_dense": efrac,
                "dense_equivalent_tops": achieved * nmod if achieved else None,
                "fp64_equivalent_tflops": achieved, "fp64_equivalent_frac_of_fp64_peak":
                    (achieved / FP64_PEAK_TFLOPS) if achieved else None}
        if unpiped and unpiped["kernel_ms"] > 0:
            ua = unpiped["kernel_flops"] / (unpiped["kernel_ms"] * 1e-3) / 1e12 * nmod * efrac
            unpiped["roofline_frac"] = ua / INT8_PEAK_TOPS
            unpiped["avg_launch_ms"] = unpiped["kernel_ms"] / unpiped["kernel_launches"] / nmod
    else:
        roof = {"bound": "mfma", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": (achieved / FP64_PEAK_TFLOPS) if achieved else None, "traffic": traffic,
                "traffic_source": traffic_source,
                "kernel": "gemm_f64_kernel<NN,COLSQ> (variance ‖L⁻¹k*‖²)",
                "launches": klaunch, "avg_launch_ms": (kms / klaunch) if klaunch else None,
                "flops_per_launch": (kflops / klaunch) if klaunch else None}
    out = {
        "metric": METRIC if (args.kind, args.ntrain) == ("df", 4096) else
        f"posterior grid points/sec (fit+predict), N_train={args.ntrain}, {args.kind} 2D kernel",
        "value": value,
        "unit": "points/s",
        "n_gpus": ws,
        "world_size": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f64" if args.variance == "f64" else "f64 (variance GEMM as exact int8 Ozaki-II)",
        "data": "synthetic (seeded drifter field, SURVEY.md §8d)",
        "config": {"workload": f"{args.kind} kernel, N_train={args.ntrain}, " +
                               (f"one {G}x{G} grid sharded over {ws} GPU(s)" if strong else f"{G}x{G} grid per GPU") +
                               ", fit+predict (mean+variance)" + (f" [BASELINE config {args.config}]" if args.config else ""),
                   "n_train": args.ntrain, ("grid_global" if strong else "grid_per_gpu"): f"{G}x{G}",
                   "points_total": m_all, "length_scale_km": 5.0, "noise": noise,
                   "parallelism": (f"grid-sharded x{ws}, job j fitted on rank j mod {ws}, factor broadcast "
                                   "(RCCL, packed W)" if cfg["mode"] == "rr" else
                                   f"grid-sharded x{ws}, factor {cfg['mode']}" +
                                   (" (RCCL broadcast of packed W)" if is_multi(ws) and cfg["mode"] == "bcast" else "")),
                   "fit_mode_probe_ms_per_step": probe or None, "kstar_ahead": cfg["ahead"]},
        "roofline": roof,
        "pipelined": cfg["pipeline"],
        "api": api,
        **job_stream_shape(args, spec, m, api),
        "unpipelined": unpiped,
        "single_job": single_job,
        "timed_fits": timed_fits,
        "mean_only_value": mean_only,
        "guard": guard,
    }
    if comm_out is not None:
        out["comm"] = comm_out
    if not is_multi(ws):
        out.update(extra_readings_n1(args, spec, xt, yt, noise, xg, m_all))
    if not is_multi(ws) and (args.cpu_baseline > 0 or (args.cpu_baseline < 0 and args.ntrain <= 4096)):
        out["cpu_baseline"] = cpu_baseline(x, y, xg_all, args.kind, 5.0, noise, args.cpu_sample_points)
    print(json.dumps(out), flush=True)
    if is_multi(ws):
        finish_dist()


if __name__ == "__main__":
    main()
