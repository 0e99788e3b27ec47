"""Index, grid and input-preparation work of the reference (host side, bit-exact).

These are integer / ordering operations with negligible cost next to the fit and
predict; they run on the host in numpy and must reproduce the reference's
output exactly ("bit-exact index/partition work").
"""
from __future__ import annotations

import numpy as np


def split_indices(n: int, step: int):
    """Training / test split, GP_laser.py:80-83 and krig.py:335-337.

    samples = arange(0, n, step); test = np.array(list(set(arange(n)) − set(samples))).
    The test order is CPython's set iteration order (it is NOT sorted for many n,
    SURVEY.md §0.2); the same set arithmetic on Python ints reproduces it because
    hash(np.int64(k)) == hash(k).
    """
    n = int(n)
    step = int(step)
    if step < 1:
        raise ValueError("step must be >= 1")
    samples = np.arange(0, n, step)
    test = set(range(n)) - set(range(0, n, step))
    return samples, np.array(list(test), dtype=np.int64)


def drifter_split(n_time: int, n_drifters: int, sample_step: int, skip: int):
    """The per-time-step / per-drifter split of krig.kriging (krig.py:300-316).

    Returns (samples, testt, testd): rows of the (time × drifter) arrays used for
    training, and the test time / drifter indices, in the reference's order.
    """
    ss = abs(int(sample_step))
    samples = np.arange(0, n_time, ss)
    if skip > 1:
        testt = np.arange(n_time)
        testd = np.array(list(set(range(n_drifters)) - set(range(0, n_drifters, skip))), dtype=np.int64)
    else:
        testd = np.arange(0, n_drifters)
        if ss > 1:
            testt = np.array(list(set(range(n_time)) - set(range(0, n_time, ss))), dtype=np.int64)
        else:
            testt = samples
    return samples, testt, testd


def valid_mask(*arrays):
    """NaN filter (krig.py:354-369, GP_laser.py:72-76): rows where every array is finite."""
    m = np.ones(np.asarray(arrays[0]).shape, dtype=bool)
    for a in arrays:
        m &= ~np.isnan(np.asarray(a, dtype=np.float64))
    return m


def bound_data(var, varlim, *arrays):
    """krig.boundData (krig.py:79-86): keep drifters whose first-row value of `var`
    lies within [varlim[0], varlim[1]]."""
    il = np.where((var[0, :] >= varlim[0]) & (var[0, :] <= varlim[1]))[0]
    return tuple(a[:, il] for a in arrays)


def laser_grid(xo, yo, xt, yt, dx: float = 0.5, pad: float = 5.0):
    """GP_laser.py:102-109: x = arange(min−pad, max+pad, dx) over obs ∪ test points;
    meshgrid(x, y) flattened row-major, point p = iy·nx + ix."""
    x = np.arange(np.min([np.min(xo), np.min(xt)]) - pad, np.max([np.max(xo), np.max(xt)]) + pad, dx)
    y = np.arange(np.min([np.min(yo), np.min(yt)]) - pad, np.max([np.max(yo), np.max(yt)]) + pad, dx)
    X, Y = np.meshgrid(x, y)
    return x, y, np.reshape(X, [X.size]), np.reshape(Y, [Y.size])


def get_grid(to, yo, xo, dt: float = 0.5, dx: float = 0.5, xL: float = 40, yL: float = 40):
    """krig.getGrid (krig.py:648-678).  Window: if the data span exceeds xL (yL) the
    grid is centred on the mean with width xL (yL), else it covers the data ± dx.
    Flatten order: meshgrid(yg, tg, xg) → T-major, then Y, then X.
    Returns (X (M,3) in T,Y,X order, tg, yg, xg)."""
    if (np.max(xo) - np.min(xo)) > xL:
        xmin = np.mean(xo) - xL / 2
        xmax = np.mean(xo) + xL / 2
    else:
        xmin = np.min(xo) - dx
        xmax = np.max(xo) + dx
    if (np.max(yo) - np.min(yo)) > yL:
        ymin = np.mean(yo) - yL / 2
        ymax = np.mean(yo) + yL / 2
    else:
        ymin = np.min(yo) - dx
        ymax = np.max(yo) + dx
    xg = np.arange(xmin, xmax, dx)
    yg = np.arange(ymin, ymax, dx)
    tg = np.arange(np.min(to), np.max(to), dt)
    Yg, Tg, Xg = np.meshgrid(yg, tg, xg)
    X = np.concatenate([np.reshape(Tg, [Tg.size, 1]), np.reshape(Yg, [Yg.size, 1]),
                        np.reshape(Xg, [Xg.size, 1])], axis=1)
    return X, tg, yg, xg


def synthetic_tracks(n: int, seed: int = 2016, box=(60.0, 45.0), amp: float = 1.0, L: float = 15.0,
                     noise_sd: float = 0.05):
    """Seeded synthetic drifter observations: N points uniform in a
    60×45 km box; (u, v) from the div-free stream function ψ = A·exp(−r²/L²)
    (u = ∂ψ/∂y, v = −∂ψ/∂x, as GP_scripts.generate_2D_gaussian, GP_scripts.py:202-223)
    plus N(0, 0.05²) noise."""
    rng = np.random.default_rng(seed)
    x = rng.uniform(0, box[0], n)
    y = rng.uniform(0, box[1], n)
    x0, y0 = box[0] / 2, box[1] / 2
    psi = amp * np.exp(-((x - x0) ** 2 + (y - y0) ** 2) / L ** 2)
    u = psi * (-2 * (y - y0) / L ** 2)
    v = -psi * (-2 * (x - x0) / L ** 2)
    u = u + rng.normal(0, noise_sd, n)
    v = v + rng.normal(0, noise_sd, n)
    return x, y, u, v


def bbox_grid(x, y, G: int, pad: float = 5.0, Gy: int | None = None):
    """G×Gy uniform grid over the training bounding box ± pad (GP_laser.py:103-106 extents),
    flattened row-major (p = iy·G + ix).  Returns (gx, gy, points (M,2))."""
    Gy = G if Gy is None else Gy
    gx = np.linspace(np.min(x) - pad, np.max(x) + pad, G)
    gy = np.linspace(np.min(y) - pad, np.max(y) + pad, Gy)
    GX, GY = np.meshgrid(gx, gy)
    return gx, gy, np.stack([GX.reshape(-1), GY.reshape(-1)], 1)


def shard_range(m: int, world: int, rank: int, align: int = 64):
    """Contiguous, tile-aligned [lo, hi) shard of m points for `rank` of `world`
    (SURVEY.md §8e).  Concatenating the shards in rank order gives 0..m."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    tiles = (m + align - 1) // align
    per, rem = divmod(tiles, world)
    t0 = rank * per + min(rank, rem)
    t1 = t0 + per + (1 if rank < rem else 0)
    return min(m, t0 * align), min(m, t1 * align)
