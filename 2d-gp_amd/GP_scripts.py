"""The reference's ``GP_scripts`` functional API (GP_scripts.py:1-142), computed by the HIP engine.

Same names, argument meaning and return shapes as the reference, so a caller such as
GP_laser.laser (GP_laser.py:113-136) or GP_plots (GP_plots.py:262-289) runs unchanged with
``import GP_scripts`` resolving here:

  * ``myKernel(xa, xb, r_df, r_cf, alpha=1)``      GP_scripts.py:6-42
  * ``getMean(KS, Ki, y)``                           GP_scripts.py:44-46
  * ``getCov(x1, x2, x1s, x2s, sigma, divFree)``     GP_scripts.py:48-54
  * ``nonDivK(xa, xb, sigma, divFree)``              GP_scripts.py:57-69
  * ``compute_K(x1, x2, sigma, divFree)``            GP_scripts.py:74-95
  * ``compute_Ks(x1, x2, x1s, x2s, sigma, divFree)`` GP_scripts.py:97-123
  * ``sqExp(x1, y1, x2, y2, sigma)``                 GP_scripts.py:125-134
  * ``rbf(x1, x2, l, sigma, noise)``                 GP_scripts.py:136-142

Covariances come from the assembly kernel (gp2d_assemble), products from the FP64 MFMA GEMM
core (gp2d_gemm), the inverse in getCov from the Cholesky factor (gp2d_potrf, gp2d_trtri).
Inputs are numpy arrays (or torch tensors); outputs are numpy arrays, as in the reference.
There is no CPU path: without the HIP engine every function raises NativeLibraryError.

One deliberate difference: the reference inverts with ``np.linalg.inv``, which succeeds on
any non-singular matrix; getCov here factors K and raises ``numpy.linalg.LinAlgError`` when
K is not positive definite (a covariance without noise whose points nearly coincide).
"""
from __future__ import annotations

import numpy as np
import torch

from gp2d import engine as E

_DIVFREE = {0: "scalar", 1: "df", 2: "cf"}


def _np(t):
    return t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)


def _points(a, b):
    return np.stack([np.reshape(np.asarray(a, dtype=np.float64), [-1]),
                     np.reshape(np.asarray(b, dtype=np.float64), [-1])], 1)


def _spec(sigma, divFree):
    if int(divFree) not in _DIVFREE:   # the reference's else-branch: plain SE
        divFree = 0
    return E.KernelSpec(kind=_DIVFREE[int(divFree)], l_df=float(sigma), l_cf=float(sigma))


def myKernel(xa, xb, r_df, r_cf, alpha=1):
    """alpha·K_df(r_df) + (1 − alpha)·K_cf(r_cf) between the rows of xa (Na, 2) and xb (Nb, 2):
    the (2Na, 2Nb) component-major matrix of GP_scripts.py:6-42."""
    xa = np.asarray(xa, dtype=np.float64).reshape(-1, 2)
    xb = np.asarray(xb, dtype=np.float64).reshape(-1, 2)
    if alpha == 1:
        spec = E.KernelSpec(kind="df", l_df=float(r_df))
    elif alpha == 0:
        spec = E.KernelSpec(kind="cf", l_df=float(r_cf), l_cf=float(r_cf))
    else:
        spec = E.KernelSpec(kind="mixed", l_df=float(r_df), l_cf=float(r_cf), ratio=float(alpha))
    return _np(E.assemble(spec, xa, xb))


def getMean(KS, Ki, y):
    """f = KS·(Ki·y), flattened (GP_scripts.py:44-46): two FP64 MFMA products."""
    if not isinstance(y, torch.Tensor):
        y = np.asarray(y, dtype=np.float64)
    Kiy = E.gemm(Ki, y.reshape(-1, 1))
    return np.reshape(_np(E.gemm(KS, Kiy)), [-1])


def getCov(x1, x2, x1s, x2s, sigma=0.2, divFree=1):
    """(ML, Ki, Ks) of GP_scripts.py:48-54: K = compute_K(x1, x2), Ki = K⁻¹,
    Ks = compute_Ks(…), ML = Kss − Ks·Ki·Ksᵀ (the full 2M × 2M posterior covariance).
    ML is formed as Kss − (Ks·Wᵀ)(Ks·Wᵀ)ᵀ with W = L⁻¹ (the same product, symmetric by
    construction)."""
    spec = _spec(sigma, divFree)
    x = _points(x1, x2)
    xs = _points(x1s, x2s)
    K = E.assemble(spec, x)
    Ki, W = E.spd_inverse(K, return_factor=True)
    Ks = E.assemble(spec, xs, x)
    Kss = E.assemble(spec, xs)
    V = E.gemm(Ks, W, transb=True)                    # Ks·Wᵀ, (2M, 2N)
    ML = E.gemm(V, V, transb=True, alpha=-1.0, C=Kss, beta=1.0)
    return _np(ML), _np(Ki), _np(Ks)


def compute_K(x1, x2, sigma, divFree=1):
    """Symmetric (2N, 2N) covariance at the points (x1, x2) (GP_scripts.py:74-95)."""
    return _np(E.assemble(_spec(sigma, divFree), _points(x1, x2)))


def compute_Ks(x1, x2, x1s, x2s, sigma, divFree=1):
    """(2M, 2N) cross-covariance of the M points (x1s, x2s) with the N points (x1, x2)
    (GP_scripts.py:97-123)."""
    return _np(E.assemble(_spec(sigma, divFree), _points(x1s, x2s), _points(x1, x2)))


def nonDivK(xa, xb, sigma, divFree=1):
    """One 2×2 block k(xa, xb) (GP_scripts.py:57-69); a scalar for divFree = 0."""
    K = compute_Ks(np.array([xb[0]]), np.array([xb[1]]), np.array([xa[0]]), np.array([xa[1]]), sigma, divFree)
    if int(divFree) not in (1, 2):
        return K[0, 0]
    return K


def sqExp(x1, y1, x2, y2, sigma):
    """(I, J) scalar SE matrix exp(−|a − b|²/2σ²) (GP_scripts.py:125-134)."""
    a, b = _points(x1, y1), _points(x2, y2)
    K = E.assemble(_spec(sigma, 0), a, b)
    return _np(K[:a.shape[0], :b.shape[0]])


def rbf(x1, x2, l=1, sigma=1, noise=0):  # noqa: E741 (reference name)
    """1-D RBF σ²·exp(−(x1_i − x2_j)²/2l²), plus noise·I when the sizes agree (GP_scripts.py:136-142)."""
    x1 = np.reshape(np.asarray(x1, dtype=np.float64), [-1])
    x2 = np.reshape(np.asarray(x2, dtype=np.float64), [-1])
    spec = E.KernelSpec(family="ard", variances=(float(sigma) ** 2,), lengthscales=((float(l),),))
    K = _np(E.assemble(spec, x1.reshape(-1, 1), x2.reshape(-1, 1)))
    if x1.size == x2.size:
        K = K + np.identity(x1.size) * noise
    return K
