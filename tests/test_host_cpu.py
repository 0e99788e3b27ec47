"""CPU-side checks: the C-ABI library loads and exports every symbol of
include/gp2d.h, the host index/grid logic is bit-exact with the reference's
golden vectors, and the compute path fails loudly without a HIP device."""
import os
import re

import numpy as np
import pytest

from conftest import ROOT


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "gp2d.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(gp2d_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    from gp2d import _native
    L = _native.lib()
    syms = header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(_native.EXPORTS)
    assert L.gp2d_abi_version() == _native.ABI_VERSION == 11
    assert L.gp2d_padded_points(1) == 64 and L.gp2d_padded_points(64) == 64 and L.gp2d_padded_points(65) == 128


def test_kernel_diag_abi():
    import ctypes
    from gp2d import _native as N
    L = N.lib()
    k = N.vector_kernel_desc(N.KIND_MIXED, 2.0, 4.0, 0.25)
    assert L.gp2d_kernel_diag(ctypes.byref(k)) == pytest.approx(0.25 / 4 + 0.75 / 16, rel=1e-15)
    k = N.vector_kernel_desc(N.KIND_DIVFREE, 0.2)
    assert L.gp2d_kernel_diag(ctypes.byref(k)) == pytest.approx(25.0, rel=1e-15)  # plots/Cov_divFree.png peak
    a = N.ard_kernel_desc([0.8, 0.2], [[3, 4, 5], [10, 1.5, 2]])
    assert L.gp2d_kernel_diag(ctypes.byref(a)) == pytest.approx(1.0)
    assert L.gp2d_block_dim(ctypes.byref(a)) == 1 and L.gp2d_block_dim(ctypes.byref(k)) == 2


def test_argument_errors_are_reported():
    import ctypes
    from gp2d import _native as N
    L = N.lib()
    k = N.vector_kernel_desc(N.KIND_DIVFREE, -1.0)
    rc = L.gp2d_assemble(None, 1, 64, None, 1, 64, ctypes.byref(k), 0.0, 1, None, 128, None)
    assert rc < 0 and b"l_df" in L.gp2d_last_error()
    rc = L.gp2d_potrf(None, 100, 100, None, None, None, 0, None)
    assert rc < 0 and b"multiple of 128" in L.gp2d_last_error()
    one = ctypes.c_void_p(1)   # never dereferenced: the argument checks fail first
    rc = L.gp2d_gemm(0, 100, 128, 16, 1.0, one, 16, one, 128, 0.0, one, 128, None)
    assert rc < 0 and b"multiples of 128" in L.gp2d_last_error()
    rc = L.gp2d_transpose(one, 100, 100, one, None)
    assert rc < 0 and b"multiple of 64" in L.gp2d_last_error()
    assert L.gp2d_bcast(None, 0, 0, None, None) == 0            # nothing to send
    rc = L.gp2d_bcast(one, 8, 0, None, None)
    assert rc < 0 and b"communicator" in L.gp2d_last_error()
    # the library's own communicator: argument checks before RCCL is touched
    assert L.gp2d_comm_id_bytes() == 128                          # ncclUniqueId
    cm = ctypes.c_void_p()
    rc = L.gp2d_comm_init(ctypes.byref(cm), 2, one, 2, -1)
    assert rc < 0 and b"rank < nranks" in L.gp2d_last_error()
    rc = L.gp2d_allreduce(one, 4, 1, N.COMM_MIN, one, None)       # ncclUint8 is not a reduction type here
    assert rc < 0 and b"dtype" in L.gp2d_last_error()
    rc = L.gp2d_allreduce(one, 4, N.COMM_INT32, 7, one, None)
    assert rc < 0 and b"op" in L.gp2d_last_error()
    assert L.gp2d_allgather(None, None, 0, None, None) == 0       # nothing to gather
    rc = L.gp2d_sendrecv(None, 0, None, 0, 8, one, None)
    assert rc < 0 and b"NULL" in L.gp2d_last_error()
    assert L.gp2d_comm_destroy(None) == 0 and L.gp2d_stream_destroy(None) == 0
    rc = L.gp2d_bcast(one, 8, -1, one, None)
    assert rc < 0 and b"root" in L.gp2d_last_error()
    # distributed factor (one job over several GPUs): argument checks before any device work
    assert L.gp2d_dfact_sb() == 512
    assert L.gp2d_dfact_panel_doubles(1024) == 1024 * 512
    assert L.gp2d_dfact_workspace(1024) >= (4 * 128 * 128 + 512 * 1024) * 8
    rc = L.gp2d_dfact_panel(one, 768, 768, 0, one, one, one, 1 << 30, None)
    assert rc < 0 and b"multiple of 512" in L.gp2d_last_error()
    rc = L.gp2d_dfact_panel(one, 1024, 1024, 2, one, one, one, 1 << 30, None)
    assert rc < 0 and b"out of range" in L.gp2d_last_error()
    rc = L.gp2d_dfact_panel(one, 1024, 1024, 0, one, one, one, 8, None)
    assert rc < 0 and b"workspace" in L.gp2d_last_error()
    rc = L.gp2d_dfact_update(one, 1024, 1024, 0, one, 2, 2, 0, 2, None)
    assert rc < 0 and b"rank" in L.gp2d_last_error()
    rc = L.gp2d_dfact_invstep(one, 1024, 1022, 0, one, 1, 0, one, 1 << 30, None)
    assert rc < 0 and b"lda" in L.gp2d_last_error()
    rc = L.gp2d_dfact_invstep(one, 1024, 1024, 0, one, 1, 0, one, 8, None)
    assert rc < 0 and b"workspace" in L.gp2d_last_error()
    assert L.gp2d_dfact_update(one, 1024, 1024, 1, one, 1, 0, 0, 2, None) == 0   # no super-column after the last
    assert L.gp2d_copy2d(None, 1, None, 1, 0, 4, None) == 0
    rc = L.gp2d_copy2d(one, 2, one, 4, 3, 4, None)
    assert rc < 0 and b"leading dimension" in L.gp2d_last_error()
    rc = L.gp2d_zero_upper(one, 100, 100, None)
    assert rc < 0 and b"multiple of 128" in L.gp2d_last_error()


def test_ozaki_rejects_ratio_outside_unit_interval():
    """The Ozaki scale bound and CRT range check assume a convex mixed kernel:
    ratio outside [0, 1] is refused by every ozaki entry point, before any device work."""
    import ctypes
    from gp2d import _native as N
    L = N.lib()
    for r in (-0.25, 1.5):
        k = N.vector_kernel_desc(N.KIND_MIXED, 5.0, 5.0, r)
        assert L.gp2d_ozaki_nmod_apriori(8192, ctypes.byref(k), 0.0025, 0, 0) == -1
        nm = ctypes.c_int(0)
        one = ctypes.c_void_p(1)
        rc = L.gp2d_ozaki_prepare_async(one, 512, 512, ctypes.byref(k), 0.0025, 0, 0, one, one, ctypes.byref(nm), None)
        assert rc < 0 and b"ratio" in L.gp2d_last_error()
    k = N.vector_kernel_desc(N.KIND_MIXED, 5.0, 5.0, 0.5)
    assert L.gp2d_ozaki_nmod_apriori(8192, ctypes.byref(k), 0.0025, 0, 0) > 0


def test_no_cpu_fallback():
    import torch
    if torch.cuda.is_available():
        pytest.skip("HIP device present")
    from gp2d import engine as E
    from gp2d import NativeLibraryError
    with pytest.raises(NativeLibraryError):
        E.fit(E.KernelSpec(), np.zeros((4, 2)), np.zeros(8), 0.01)


def test_split_indices_bit_exact(golden):
    from gp2d import data as D
    g = golden("split_indices.npz")
    for step in (2, 3, 5):
        for n in g["sizes"]:
            s, t = D.split_indices(int(n), step)
            assert np.array_equal(t, g[f"test_{step}_{n}"])
            assert np.array_equal(s, np.arange(0, n, step))


def test_laser_split_and_grid(golden):
    from gp2d import data as D
    g = golden("laser_mixed_N256.npz")
    s, t = D.split_indices(int(g["n_raw"]), 3)
    assert np.array_equal(s, g["samples"]) and np.array_equal(t, g["test"])
    x, y, _, _ = D.laser_grid(g["xo"], g["yo"], g["xt"], g["yt"], dx=1.0)
    assert np.array_equal(x, g["x"]) and np.array_equal(y, g["y"])


def test_get_grid_bit_exact(golden):
    import krig
    g = golden("grids.npz")
    for i in range(int(g["ncases"])):
        X, tg, yg, xg = krig.getGrid(g[f"c{i}_to"], g[f"c{i}_yo"], g[f"c{i}_xo"], float(g[f"c{i}_dt"]),
                                     float(g[f"c{i}_dx"]), float(g[f"c{i}_xL"]), float(g[f"c{i}_yL"]))
        assert np.array_equal(X, g[f"c{i}_X"]) and np.array_equal(tg, g[f"c{i}_tg"])
        assert np.array_equal(yg, g[f"c{i}_yg"]) and np.array_equal(xg, g[f"c{i}_xg"])


def test_drifter_split_matches_reference_expression():
    from gp2d import data as D
    for nt, nd, ss, skip in [(96, 40, -2, 1), (96, 40, -1, 3), (50, 37, -4, 1), (50, 37, -1, 2)]:
        samples, testt, testd = D.drifter_split(nt, nd, ss, skip)
        # krig.py:304-316, verbatim numpy expressions
        ss_ = abs(ss)
        ref_s = np.arange(0, nt, ss_)
        if skip > 1:
            ref_tt = np.arange(nt)
            ref_td = np.array(list(set(np.arange(0, nd)) - set(np.arange(0, nd, skip))))
        else:
            ref_td = np.arange(0, nd)
            ref_tt = np.array(list(set(np.arange(0, nt)) - set(ref_s))) if ss_ > 1 else ref_s
        assert np.array_equal(samples, ref_s) and np.array_equal(testt, ref_tt) and np.array_equal(testd, ref_td)


def test_shard_ranges_cover_and_align():
    from gp2d import data as D
    for m in (1, 63, 64, 65, 65536, 262144 + 17):
        for w in (1, 2, 3, 4, 8):
            parts = [D.shard_range(m, w, r) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == m
            for (a, b), (c, d) in zip(parts, parts[1:]):
                assert b == c
            assert all(a % 64 == 0 or a == m for a, _ in parts)


@pytest.mark.parametrize("case", range(5))
def test_data_prep_bit_exact_on_tracks(golden, case):
    """krig's getData / boundData / projection / split / NaN filter / T,Y,X stacking vs the
    reference's own code (krig.py:50-77, 79-86, 274-381 exec'd by oracle/make_golden.py) on
    simulTracks coordinates with NaN tails and the hard-coded drifter-238 exclusion:
    bit-exact (SHA-256 of every output array)."""
    import hashlib
    from gp2d import krig as K
    g = golden("prep_tracks.npz")
    tr = K.Tracks(g["time"], g["lat"], g["lon"], g["u"], g["v"])
    st, et, ss, skip, la0, la1, lo0, lo1 = g[f"c{case}_args"]
    d = K._prepare(tr, int(st), int(et), (la0, la1), (lo0, lo1), int(ss), int(skip), drop_drifters=(238,))
    got = dict(X=d["X"], LL_o=d["LL_o"], obs=np.concatenate([d["vo"], d["uo"]], 1), Xt=d["Xt"], LL_t=d["LL_t"],
               obst=np.concatenate([d["vt"], d["ut"]], 1))
    for nm, a in got.items():
        a = np.ascontiguousarray(a, dtype=np.float64)
        assert tuple(a.shape) == tuple(g[f"c{case}_{nm}_shape"]), nm
        if a.shape[0]:
            assert np.array_equal(a[[0, -1]], g[f"c{case}_{nm}_rows"]), nm
        assert hashlib.sha256(a.tobytes()).digest() == g[f"c{case}_{nm}_sha256"].tobytes(), nm


@pytest.mark.parametrize("case", range(3))
def test_prior_window_bit_exact(golden, case):
    """scikit_prior's observation window (krig.py:146-167, exec'd by make_golden) — bit-exact."""
    from gp2d import krig as K
    g = golden("prior_window.npz")
    tc, tlim, x0, x1, xrange, comp = g[f"c{case}_args"]
    fm = {k: g[k] for k in ("Xo", "Xt", "obs", "test_points")}
    XT, u = K._prior_window(fm, np.array([tc]), tlim, (x0, x1), xrange, "u" if comp else "v")
    assert np.array_equal(XT, g[f"c{case}_XT"]) and np.array_equal(u, g[f"c{case}_u"])


def test_bench_scaling_defaults(monkeypatch):
    """bench.py: N = 1 runs the headline job; N > 1 defaults to strong scaling over the same
    256×256 job grid with round-robin fits; --scaling weak keeps a block per rank."""
    import sys
    import bench
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert (a.grid_global, a.fit_mode) == (0, "replicate")
    monkeypatch.setenv("WORLD_SIZE", "8")
    a = bench.parse()
    assert (a.grid_global, a.fit_mode) == (256, "rr")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--scaling", "weak"])
    a = bench.parse()
    assert (a.grid_global, a.fit_mode) == (0, "replicate")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--fit-mode", "bcast"])
    a = bench.parse()
    assert (a.grid_global, a.fit_mode) == (256, "bcast")


def test_ozaki_epilogue_reduction_exact():
    """The int8 GEMM epilogue's six-operation reduction (csrc/ozaki.hpp ozaki_mod_u32),
    emulated bit for bit: for every modulus of the table and biased sums v anywhere in
    [0, 2^32) (K < 2^17), y = v + (v >> 20)·(−(2^20 − 2^20 mod m)) mod 2^32 (v_mad_i32_i24),
    q = hi32(8y · ⌈2^29/m⌉) (v_mul_hi_u32_u24, both operands < 2^24), r = y − q·m gives
    0 ≤ r < m and r ≡ v (mod m)."""
    moduli = [256, 255, 253, 251, 247, 241, 239, 233, 229, 227, 223, 217, 211, 199, 197, 193, 191, 181, 179, 173]
    rng = np.random.default_rng(5)
    edges = np.array([0, 1, 2 ** 20 - 1, 2 ** 20, 2 ** 31 - 1, 2 ** 31, 2 ** 32 - 2 ** 15, 2 ** 32 - 1],
                     dtype=np.uint64)
    v = np.concatenate([edges, rng.integers(0, 2 ** 32, 400_000, dtype=np.uint64)])
    for m in moduli:
        neg_c = -((1 << 20) - (1 << 20) % m)
        magic = ((1 << 29) + m - 1) // m
        assert magic < (1 << 24)
        vh = v >> np.uint64(20)
        y = (v.astype(np.int64) + vh.astype(np.int64) * neg_c) % (1 << 32)   # mod 2^32 like the mad
        assert y.max() < (1 << 21)
        y8 = y << 3
        assert y8.max() < (1 << 24)
        q = (y8 * magic) >> 32
        r = y - q * m
        assert r.min() >= 0 and r.max() < m, m
        assert np.array_equal(r, (v % np.uint64(m)).astype(np.int64)), m
    # the bias keeps every sum of K products of centred int8 residues in [0, 2^32)
    for K, m in [(8192, 251), (32768, 193), (131071, 197)]:
        bias = ((K << 14) + m - 1) // m * m
        assert bias % m == 0 and bias - (K << 14) >= 0 and bias + (K << 14) < (1 << 32)


def test_ozaki_residue_low_bytes_exact():
    """The residue kernels' conversion-free byte (csrc/ozaki.hpp residue_low_m), emulated in
    fp64: for integers |x| < 2^51 and every modulus, q = rint(x·(1/m)) and
    (x + 1.5·2^52) − m·q is exact, lies in [2^52, 2^53), and the low byte of its bit pattern is
    the centred residue's two's-complement byte — the byte the int conversion gave
    (csrc/ozaki.hpp's former residue_byte: (int)(x − m·q) & 0xff)."""
    moduli = [256, 255, 253, 251, 247, 241, 239, 233, 229, 227, 223, 217, 211, 199, 197, 193, 191, 181, 179, 173]
    rng = np.random.default_rng(7)
    lim = 2.0 ** 51 - 1
    edges = np.array([0.0, 1.0, -1.0, 127.0, -128.0, 128.0, 2.0 ** 45, -2.0 ** 45, 2.0 ** 49 - 1, -(2.0 ** 49),
                      lim, -lim])
    x = np.concatenate([edges, np.rint(rng.uniform(-2.0 ** 49, 2.0 ** 49, 200_000)),
                        np.rint(rng.uniform(-2.0 ** 12, 2.0 ** 12, 50_000))])
    xm = x + 6755399441055744.0   # 1.5·2^52: exact for |x| < 2^51
    assert np.array_equal(xm - 6755399441055744.0, x)
    for m in moduli:
        q = np.rint(x * (1.0 / m))
        r = x - m * q              # the old path: |r| ≤ m/2, exact
        assert np.abs(r).max() <= m / 2, m
        rm = xm - m * q            # the new path (fma in the kernel; exact here as well)
        assert rm.min() >= 2.0 ** 52 and rm.max() < 2.0 ** 53, m
        assert np.array_equal(rm - 6755399441055744.0, r), m
        lo = rm.view(np.int64) & 0xFF
        assert np.array_equal(lo, r.astype(np.int64) & 0xFF), m
        c = np.mod(x.astype(np.int64), m)             # the residue in [0, m), integer arithmetic
        centred = np.where(c > m // 2, c - m, c)      # m = 256: ±128 share the byte 0x80
        assert np.array_equal(lo, centred & 0xFF), m


def test_factor_workspaces_cover_the_split_trtri():
    """gp2d_trtri / gp2d_potrf_inv workspaces (host functions, no device needed) include room
    for the high halves of the K-split TRTRI products (the lower levels' products with at most
    256 tiles per pair) on top of the T buffers, and grow with n."""
    from gp2d import _native as N
    L = N.lib()
    nb_ = 128
    prev_t = prev_f = 0
    for n in (128, 256, 640, 1024, 2048, 4096, 8192, 16384, 32768):
        nb = n // nb_
        t_base = (n // 2 + nb_) ** 2 * 8 + nb * nb_ * nb_ * 8
        t = int(L.gp2d_trtri_workspace(n))
        assert t >= t_base
        if nb >= 8:   # a level with g >= 4 exists: its products are split
            assert t > t_base, n
        f = int(L.gp2d_potrf_inv_workspace(n))
        assert t >= prev_t and f >= prev_f
        prev_t, prev_f = t, f
    assert int(L.gp2d_potrf_inv_workspace(128)) == 0


def test_factor_join_mode_is_per_thread_and_restorable():
    """gp2d_factor_join (host state only, no device needed): a negative argument queries, the
    previous mode is returned, and the mode belongs to the calling thread (engine.fit sets and
    restores it around one factorisation)."""
    import threading
    from gp2d import _native as N
    L = N.lib()
    assert L.gp2d_factor_join(-1) == 0
    assert L.gp2d_factor_join(1) == 0
    assert L.gp2d_factor_join(-1) == 1
    seen = []
    t = threading.Thread(target=lambda: seen.append(L.gp2d_factor_join(-1)))
    t.start()
    t.join()
    assert seen == [0]
    assert L.gp2d_factor_join(0) == 1
    assert L.gp2d_factor_join(-1) == 0


def test_job_shape_defaults_live_in_the_library():
    """engine.auto_fits_ahead / hyper.auto_concurrent: config B's small jobs
    run back to back, the headline / C / D shapes pipelined; a sweep overlaps only when there is a
    gradient and a next setting — and bench.py carries no per-config override."""
    from gp2d import engine as E
    from gp2d import hyper as H
    df, mixed = E.KernelSpec(kind="df"), E.KernelSpec(kind="mixed", ratio=0.5)
    assert E.auto_fits_ahead(df, 1024, 128 * 128) == 0
    assert E.auto_fits_ahead(df, 4096, 256 * 256) == 1
    assert E.auto_fits_ahead(mixed, 16384, 512 * 512) == 1
    assert H.auto_concurrent(8, True) == 2 and H.auto_concurrent(8, False) == 1 and H.auto_concurrent(1, True) == 1
    # batched factorisations: config B's back-to-back jobs 16 fits, N = 4096 job streams 8, config
    # E's sweep 16 settings (profiles/r04_bfit16_ab.jsonl, r04_ebatch_ab.jsonl); D-sized matrices
    # (8 GB each) are not batched
    assert E.auto_fit_batch(df, 1024) == 16 and E.auto_fit_batch(df, 4096) == 8 and E.auto_fit_batch(mixed, 16384) == 1
    x = np.zeros((4096, 2))
    assert H.auto_batch(df, x, 64) == 16 and H.auto_batch(df, x, 8) == 8 and H.auto_batch(df, x, 3) == 3
    assert H.auto_batch(df, x, 1) == 1
    assert H.auto_batch(df, x, 8, concurrent=2) == 1
    # config B's batches overlap the next batch's fit with their predicts (8.8e6 vs 7.8e6 points/s);
    # a tiny grid beside FLOP-bound N = 4096 batches does not
    assert E.auto_batch_ahead(df, 1024, 128 * 128, 8) and not E.auto_batch_ahead(df, 4096, 32 * 32, 8)
    assert not E.auto_batch_ahead(df, 1024, 128 * 128, 1)
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert "a.fits_ahead = 0" not in src and "sweep_concurrent or 2" not in src


def test_fit_batch_rejects_more_than_64_problems():
    """engine.fit_batch / gp2d_potrf_batched take at most 64 problems per batch (checked on the
    host before any device work)."""
    from gp2d import engine as E
    k = E.KernelSpec(kind="df")
    with pytest.raises(ValueError, match="at most 64"):
        E.fit_batch([(k, np.zeros((10, 2)), np.zeros(20), 0.01)] * 65)
    assert E.fit_batch([]) == []


def test_ozaki_split_residues_of_wide_w_rows_exact():
    """The W residue kernel above 50 bits (csrc/ozaki.hpp ozaki_w_res_kernel, pw ≤ 60), emulated
    in fp64: x = xh·2^26 + xl exactly, the centred residues rh, rl by one fma each, and
    t = rh·(2^26 mod m, centred) + rl reduced once more gives, for every modulus, the residue of
    x itself (checked against Python's exact integers)."""
    moduli = [256, 255, 253, 251, 247, 241, 239, 233, 229, 227, 223, 217, 211, 199, 197, 193, 191, 181, 179, 173]
    rng = np.random.default_rng(11)
    lim = 2.0 ** 60
    x = np.concatenate([np.array([0.0, 1.0, -1.0, 2.0 ** 59, -(2.0 ** 59), lim - 2 ** 8, -(lim - 2 ** 8)]),
                        np.rint(rng.uniform(-lim, lim, 100_000)), np.rint(rng.uniform(-2.0 ** 52, 2.0 ** 52, 20_000))])
    xh = np.rint(np.ldexp(x, -26))
    xl = x - np.ldexp(xh, 26)
    assert np.array_equal(np.ldexp(xh, 26) + xl, x) and np.abs(xl).max() <= 2 ** 25
    exact = [int(v) for v in x]
    for m in moduli:
        c26 = (1 << 26) % m
        c26 = c26 - m if 2 * c26 > m else c26
        rh = xh - m * np.rint(xh * (1.0 / m))
        rl = xl - m * np.rint(xl * (1.0 / m))
        t = rh * c26 + rl
        assert np.abs(t).max() <= 128 * 128 + 128
        r = t - m * np.rint(t * (1.0 / m))       # the final one-part residue: |t| < 2^50
        ref = np.array([((e % m) + m) % m for e in exact], dtype=np.float64)
        assert np.array_equal(np.mod(r, m), ref), m


def test_release_build_rejects_measurement_overrides():
    """The shipped library is a release build (gp2d_build_info, checked by _native.lib() on load),
    and a GP2D_RELEASE compile with a measurement override (-DGP2D_<NAME>) fails at the
    preprocessor (csrc/common.hpp), so no dev switch reaches libgp2d.so."""
    import subprocess
    from gp2d import _native
    info = _native.lib().gp2d_build_info().decode()
    assert info.startswith("release gfx950") and "oz_pw=49" in info and "oz_pb=45" in info
    src = os.path.join(ROOT, "2d-gp_amd", "csrc", "common.hpp")
    base = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-x", "hip", "-E", "-o", os.devnull, src]
    ok = subprocess.run(base + ["-DGP2D_RELEASE=1"], capture_output=True, text=True)
    assert ok.returncode == 0, ok.stderr[-500:]
    bad = subprocess.run(base + ["-DGP2D_RELEASE=1", "-DGP2D_OZ_PW=50"], capture_output=True, text=True)
    assert bad.returncode != 0 and "not allowed in a GP2D_RELEASE build" in bad.stderr
    lib_src = os.path.join(ROOT, "2d-gp_amd", "csrc", "gp2d.hip")
    norel = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-E", "-o", os.devnull, lib_src],
                           capture_output=True, text=True)
    assert norel.returncode != 0 and "GP2D_RELEASE" in norel.stderr
