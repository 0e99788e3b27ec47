"""The reference's kernel plugin / operator API, computed by the HIP engine.

Mirrors
  * the GPy ``Kern`` plugin classes of myKernel.py: ``myKernel`` (mixed,
    myKernel.py:12-57), ``nonDivK`` (div-free, :148-180), ``nonRotK`` (curl-free,
    :244-275) — constructor arguments, parameter names, ``K(X, X2)`` and
    ``Kdiag(X)``;
  * the functional API of GP_scripts.py under the module's own names lives in
    ``2d-gp_amd/GP_scripts.py`` (``myKernel``, ``getMean``, ``getCov``, ``nonDivK``,
    ``compute_K``, ``compute_Ks``, ``sqExp``, ``rbf``); the helpers below (``vector_K``,
    ``compute_K``, ``compute_Ks``, ``nonDivK_block``) are kept for existing callers.

GPy itself is not a dependency: the classes expose the same methods and
parameters without the paramz machinery.  Parameters are floats carrying a
``.gradient`` attribute, which ``update_gradients_full`` fills with the EXACT
derivative contraction (HIP kernel gp2d_kernel_grad) — the reference's own
formula is not a derivative of its kernel.
``gradients_X`` raises, as the reference's does (NameError, myKernel.py:123).
Outputs are numpy arrays, as in the reference; ``*_device`` variants return the
torch tensor resident in HBM.
"""
from __future__ import annotations

import numpy as np

from . import engine as E


class Param(float):
    """A float hyperparameter with a GPy-style ``.gradient`` slot."""

    def __new__(cls, value):
        obj = super().__new__(cls, value)
        obj.gradient = 0.0
        return obj


class _VectorKern:
    input_dim = 2
    _grad_index = (0, 1, 2)   # engine.kernel_grad entries for parameter_names()

    def __init__(self, input_dim=2, active_dim=(0, 1), name="kern"):
        assert input_dim == 2, "For this kernel we assume input_dim=2"
        self.active_dims = list(active_dim)
        self.name = name

    def _spec(self) -> E.KernelSpec:
        raise NotImplementedError

    def _cols(self, X):
        X = np.asarray(X, dtype=np.float64)
        if X.ndim == 2 and X.shape[1] > 2:
            X = X[:, self.active_dims]
        return X.reshape(-1, 2)

    def K_device(self, X, X2=None):
        X = self._cols(X)
        return E.assemble(self._spec(), X, None if X2 is None else self._cols(X2))

    def K(self, X, X2=None):
        """(2N, 2M) component-major covariance (myKernel.py:27-53)."""
        return self.K_device(X, X2).cpu().numpy()

    def Kdiag(self, X):
        """k(x,x) for every component: 2N entries (myKernel.py:55-57; the reference's
        X.shape[0]*X.shape[1] equals 2N because input_dim == 2)."""
        n = self._cols(X).shape[0]
        return np.full(2 * n, self._spec().kdiag())

    def update_gradients_full(self, dL_dK, X, X2=None):
        """Set each parameter's .gradient to Σ dL_dK ⊙ ∂K(X, X2)/∂θ (myKernel.py:59-105)."""
        g = E.kernel_grad(self._spec(), self._cols(X), dL_dK, None if X2 is None else self._cols(X2))
        for name, i in zip(self.parameter_names(), self._grad_index):
            p = Param(getattr(self, name))
            p.gradient = float(g[i])
            setattr(self, name, p)

    def update_gradients_diag(self, dL_dKdiag, X):
        """Kdiag depends on the length scales only through 1/ℓ²; the reference leaves this a
        no-op (myKernel.py:107-108), and so does this mirror."""

    def gradients_X(self, dL_dK, X, X2=None):
        raise NotImplementedError("gradients_X is broken in the reference (NameError, myKernel.py:123); "
                                  "not provided")

    @property
    def param_array(self):
        return np.array([getattr(self, p) for p in self.parameter_names()], dtype=np.float64)


class myKernel(_VectorKern):
    """Mixed kernel ratio·K_df(length_df) + (1−ratio)·K_cf(length_cf) (myKernel.py:12-22)."""

    def __init__(self, input_dim=2, active_dim=(0, 1), l_df=1.0, l_cf=1.0, ratio=1.0):
        super().__init__(input_dim, active_dim, "myKern")
        if l_df <= 0 or l_cf <= 0:
            raise ValueError("length scales must be positive")
        if not 0.0 <= ratio <= 1.0:
            raise ValueError("ratio is bounded to [0, 1] (myKernel.py:21)")
        self.length_df = Param(l_df)
        self.length_cf = Param(l_cf)
        self.ratio = Param(ratio)

    def parameter_names(self):
        return ["length_df", "length_cf", "ratio"]

    def _spec(self):
        return E.KernelSpec(kind="mixed", l_df=self.length_df, l_cf=self.length_cf, ratio=self.ratio)


class nonDivK(_VectorKern):
    """Divergence-free SE kernel (myKernel.py:148-180)."""
    _grad_index = (0,)

    def __init__(self, input_dim=2, active_dim=(0, 1), length=1.0):
        super().__init__(input_dim, active_dim, "nonDivK")
        if length <= 0:
            raise ValueError("length must be positive")
        self.length = Param(length)

    def parameter_names(self):
        return ["length"]

    def _spec(self):
        return E.KernelSpec(kind="df", l_df=self.length)


class nonRotK(_VectorKern):
    """Curl-free SE kernel (myKernel.py:244-275)."""
    _grad_index = (1,)

    def __init__(self, input_dim=2, active_dim=(0, 1), l=1.0):  # noqa: E741 (reference name)
        super().__init__(input_dim, active_dim, "nonRotK")
        if l <= 0:
            raise ValueError("length must be positive")
        self.length = Param(l)

    def parameter_names(self):
        return ["length"]

    def _spec(self):
        return E.KernelSpec(kind="cf", l_df=self.length, l_cf=self.length)


# ------------------------------------------------------------------ functional API
_DIVFREE = {0: "scalar", 1: "df", 2: "cf"}


def vector_K(xa, xb, r_df, r_cf, alpha=1.0):
    """GP_scripts.myKernel(xa, xb, r_df, r_cf, alpha) (GP_scripts.py:6-42): (2Na, 2Nb)."""
    if alpha == 1:
        spec = E.KernelSpec(kind="df", l_df=r_df)
    elif alpha == 0:
        spec = E.KernelSpec(kind="cf", l_df=r_cf, l_cf=r_cf)
    else:
        spec = E.KernelSpec(kind="mixed", l_df=r_df, l_cf=r_cf, ratio=alpha)
    return E.assemble(spec, np.asarray(xa).reshape(-1, 2), np.asarray(xb).reshape(-1, 2)).cpu().numpy()


def compute_K(x1, x2, sigma, divFree=1):
    """GP_scripts.compute_K (GP_scripts.py:74-95): symmetric (2N, 2N) for divFree 0/1/2."""
    x = np.stack([np.reshape(x1, [-1]), np.reshape(x2, [-1])], 1)
    spec = E.KernelSpec(kind=_DIVFREE[int(divFree)], l_df=sigma, l_cf=sigma)
    return E.assemble(spec, x).cpu().numpy()


def compute_Ks(x1, x2, x1s, x2s, sigma, divFree=1):
    """GP_scripts.compute_Ks (GP_scripts.py:97-123): (2M, 2N) cross-covariance grid × train."""
    x = np.stack([np.reshape(x1, [-1]), np.reshape(x2, [-1])], 1)
    xs = np.stack([np.reshape(x1s, [-1]), np.reshape(x2s, [-1])], 1)
    spec = E.KernelSpec(kind=_DIVFREE[int(divFree)], l_df=sigma, l_cf=sigma)
    return E.assemble(spec, xs, x).cpu().numpy()


def nonDivK_block(xa, xb, sigma, divFree=1):
    """GP_scripts.nonDivK (GP_scripts.py:57-69): one 2×2 block (scalar for divFree=0)."""
    K = compute_Ks(np.array([xb[0]]), np.array([xb[1]]), np.array([xa[0]]), np.array([xa[1]]), sigma, divFree)
    return K[0, 0] if int(divFree) == 0 else K
