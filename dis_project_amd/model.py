"""``ExactLFM`` — the SIM latent force model surface of wejpurvis/DIS_project
(src/model.py:29-414), backed by the gfx950 kernels in ``liblfm.so``.

Same class, method and argument names and the same return shapes as the reference
(GPJax ``gpx.base.Module`` with constrained parameters):

=====================  ==========================================  ===================
method                 reference                                   device entry point
=====================  ==========================================  ===================
``mean_function(x)``   model.py:124-149 -> [N, 1]                  lfm_mean_function_f64
``kernel(t, t')``      model.py:152-195 -> scalar                  lfm_cross_covariance_f64
``kernel_xx/xf/ff``    model.py:197-312 -> scalar                  lfm_cross_covariance_f64
``h(j, k, t1, t2)``    model.py:315-365                            lfm_h_f64
``gamma(k)``           model.py:367-369 (parameter arithmetic)     —
``cross_covariance``   model.py:372-394 -> [N, M]                  lfm_cross_covariance_f64
``gram(kernel, x)``    model.py:396-414 -> PSD dense operator       lfm_gram_f64
=====================  ==========================================  ===================

Every value is computed on the GPU; nothing here evaluates the kernel on the host.
Parameters are held *constrained* (true_d, true_s, true_b, l, obs_stddev), as the
reference's model is after ``constrain()`` (trainer.py:102-103).
"""

from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import HypArgs, as_f64, dptr, get_context


class DenseOperator:
    """Minimal stand-in for ``cola.PSD(cola.ops.Dense(K))`` (model.py:414): holds the
    dense gram and exposes ``to_dense()`` / ``shape`` / ``+`` with arrays or operators."""

    def __init__(self, mat: np.ndarray, psd: bool = True):
        self.mat = np.asarray(mat, dtype=np.float64)
        self.psd = psd

    @property
    def shape(self):
        return self.mat.shape

    def to_dense(self) -> np.ndarray:
        return self.mat

    def __array__(self, dtype=None):
        return self.mat if dtype is None else self.mat.astype(dtype)

    def __add__(self, other):
        o = other.to_dense() if isinstance(other, DenseOperator) else np.asarray(other)
        return DenseOperator(self.mat + o, self.psd)

    __radd__ = __add__


def identity_like(op, scale: float = 1.0) -> np.ndarray:
    """``cola.ops.I_like(op) * scale`` as a dense array."""
    return np.eye(op.shape[0]) * scale


@dataclass
class ExactLFM:
    """SIMM latent force model (Lawrence et al. 2006), model.py:29-121.

    Defaults follow model.py:64-121: jitter 1e-6 (main.py:41 passes 1e-4),
    obs_stddev 1.0, num_genes 5, D = 0.4, S = 1.0, B = 0.05 per gene, l = 2.5.
    """

    jitter: float = 1e-6
    obs_stddev: float = 1.0
    num_genes: int = 5
    true_d: np.ndarray | None = None
    true_s: np.ndarray | None = None
    true_b: np.ndarray | None = None
    l: float = 2.5
    device: int | None = field(default=None, repr=False)

    def __post_init__(self):
        g = int(self.num_genes)
        if g < 1:
            raise ValueError("num_genes must be >= 1")
        # model.py:99-108
        self.true_d = as_f64([0.4] * g if self.true_d is None else self.true_d).reshape(-1)
        self.true_s = as_f64([1.0] * g if self.true_s is None else self.true_s).reshape(-1)
        self.true_b = as_f64([0.05] * g if self.true_b is None else self.true_b).reshape(-1)
        for name in ("true_d", "true_s", "true_b"):
            if getattr(self, name).size != g:
                raise ValueError(f"{name} must have num_genes={g} entries")

    # ------------------------------------------------------------ plumbing
    @property
    def ctx(self) -> _lib.Context:
        return get_context(self.device)

    def hyp(self) -> HypArgs:
        return HypArgs(self.true_d, self.true_s, self.true_b, self.l, self.obs_stddev, self.jitter)

    def replace(self, **kw) -> "ExactLFM":
        d = dict(jitter=self.jitter, obs_stddev=self.obs_stddev, num_genes=self.num_genes,
                 true_d=self.true_d, true_s=self.true_s, true_b=self.true_b, l=self.l,
                 device=self.device)
        d.update(kw)
        return ExactLFM(**d)

    # ------------------------------------------------------- model surface
    def mean_function(self, x) -> np.ndarray:
        """model.py:124-149 -> [N, 1]."""
        x = as_f64(x).reshape(-1, 3)
        out = np.empty(x.shape[0])
        hp = self.hyp()
        ctx = self.ctx
        ctx.check(ctx.lib.lfm_mean_function_f64(ctx.handle, dptr(x), x.shape[0], hp.ref, dptr(out)))
        return out.reshape(-1, 1)

    def cross_covariance(self, kernel, x, y) -> np.ndarray:
        """model.py:372-394: kernel(x_i, y_j) for all pairs -> [N, M]."""
        self._check_kernel(kernel)
        x = as_f64(x).reshape(-1, 3)
        y = as_f64(y).reshape(-1, 3)
        out = np.empty((x.shape[0], y.shape[0]))
        hp = self.hyp()
        ctx = self.ctx
        ctx.check(ctx.lib.lfm_cross_covariance_f64(ctx.handle, dptr(x), x.shape[0], dptr(y),
                                                   y.shape[0], hp.ref, dptr(out), y.shape[0]))
        return out

    def gram(self, kernel, x) -> DenseOperator:
        """model.py:396-414 -> PSD dense operator over the N x N gram."""
        self._check_kernel(kernel)
        x = as_f64(x).reshape(-1, 3)
        n = x.shape[0]
        out = np.empty((n, n))
        hp = self.hyp()
        ctx = self.ctx
        ctx.check(ctx.lib.lfm_gram_f64(ctx.handle, dptr(x), n, hp.ref, 0.0, _lib.LFM_UPLO_FULL,
                                       dptr(out), n))
        return DenseOperator(out)

    def gram_f32(self, x) -> np.ndarray:
        """fp32 gram (config 4's HBM-bound variant)."""
        x = as_f64(x).reshape(-1, 3)
        n = x.shape[0]
        out = np.empty((n, n), dtype=np.float32)
        hp = self.hyp()
        ctx = self.ctx
        ctx.check(ctx.lib.lfm_gram_f32(ctx.handle, dptr(x), n, hp.ref, 0.0, _lib.LFM_UPLO_FULL,
                                       out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), n))
        return out

    def kernel(self, t, t_prime) -> float:
        """model.py:152-195: flag-switched kxx / kff / kxf / kfx for one pair of rows."""
        a = as_f64(t).reshape(1, 3)
        b = as_f64(t_prime).reshape(1, 3)
        return float(self.cross_covariance(self.kernel, a, b)[0, 0])

    def kernel_xx(self, t, t_prime) -> float:
        """model.py:197-235 (both rows treated as gene rows)."""
        a = as_f64(t).reshape(3).copy()
        b = as_f64(t_prime).reshape(3).copy()
        a[2] = b[2] = 1.0
        return self.kernel(a, b)

    def kernel_xf(self, t, t_prime) -> float:
        """model.py:237-282: the row with flag 0 is the latent-force row."""
        a = as_f64(t).reshape(3).copy()
        b = as_f64(t_prime).reshape(3).copy()
        if a[2] == 0:
            a[2], b[2] = 0.0, 1.0
        else:
            a[2], b[2] = 1.0, 0.0
        return self.kernel(a, b)

    def kernel_ff(self, t, t_prime) -> float:
        """model.py:284-312."""
        a = as_f64(t).reshape(3).copy()
        b = as_f64(t_prime).reshape(3).copy()
        a[2] = b[2] = 0.0
        return self.kernel(a, b)

    def h(self, j, k, t1, t2):
        """model.py:315-365, element-wise over broadcast arguments."""
        j, k, t1, t2 = np.broadcast_arrays(np.asarray(j), np.asarray(k), np.asarray(t1),
                                           np.asarray(t2))
        shape = j.shape
        jj = np.ascontiguousarray(j, dtype=np.int64).reshape(-1)
        kk = np.ascontiguousarray(k, dtype=np.int64).reshape(-1)
        a = as_f64(t1).reshape(-1)
        b = as_f64(t2).reshape(-1)
        out = np.empty(jj.size)
        hp = self.hyp()
        ctx = self.ctx
        p64 = ctypes.POINTER(ctypes.c_int64)
        ctx.check(ctx.lib.lfm_h_f64(ctx.handle, hp.ref, jj.ctypes.data_as(p64),
                                    kk.ctypes.data_as(p64), dptr(a), dptr(b), jj.size, dptr(out)))
        return out.reshape(shape) if shape else float(out[0])

    def gamma(self, k):
        """model.py:367-369: D_k * l / 2."""
        return (self.true_d[k] * self.l) / 2

    # ----------------------------------------------------------- predictors
    def _posterior(self, t, train_data, diag_add):
        from .dataset import dataset_3d

        x, y, variances = dataset_3d(train_data)
        x = as_f64(x).reshape(-1, 3)
        y = as_f64(y).reshape(-1)
        v = as_f64(variances).reshape(-1)
        t = as_f64(t).reshape(-1, 3)
        m = t.shape[0]
        mean = np.empty(m)
        cov = np.empty((m, m))
        hp = self.hyp()
        ctx = self.ctx
        rc = ctx.lib.lfm_posterior_f64(ctx.handle, dptr(x), dptr(y), x.shape[0], dptr(v),
                                       float(diag_add), dptr(t), m, hp.ref, dptr(mean), dptr(cov))
        ctx.check(rc, allow_not_pd=True)
        return mean, cov

    def latent_predict(self, test_inputs, train_data):
        """model.py:420-465: S = K(x,x) + diag(variances) + jitter I (no observation noise);
        mean = m(t) + K(t,x) S^{-1} (y - m(x)); var = diag(diag(K(t,t) + jitter I - K(t,x)
        S^{-1} K(x,t))) + jitter I. One lfm_posterior_f64 call (Schur complement on the
        Cholesky kernels; the reference's explicit cola.inv is the same operator)."""
        from .distributions import GaussianDistribution

        mean, cov = self._posterior(test_inputs, train_data, self.jitter)
        var = np.diag(np.diag(cov) + self.jitter) + np.eye(mean.shape[0]) * self.jitter
        return GaussianDistribution(np.atleast_1d(mean.squeeze()), var, device=self.device)

    def multi_gene_predict(self, test_inputs, train_data):
        """model.py:467-514: S = K(x,x) + diag(variances) + obs_stddev^2 I;
        mean = m(t) + K(t,x) S^{-1} (y - m(x)); var = K(t,t) - K(t,x) S^{-1} K(x,t)
        + jitter I. (The reference's ``t2`` with flags set to 1 is computed and unused.)"""
        from .distributions import GaussianDistribution

        mean, cov = self._posterior(test_inputs, train_data, self.obs_stddev**2)
        var = cov + np.eye(mean.shape[0]) * self.jitter
        return GaussianDistribution(np.atleast_1d(mean.squeeze()), var, device=self.device)

    def _check_kernel(self, kernel):
        # The reference passes ``model.kernel`` (objectives.py:70); any other kernel
        # object is not part of this hot path.
        if kernel is not None and getattr(kernel, "__func__", None) is not ExactLFM.kernel:
            raise TypeError("only ExactLFM.kernel is supported on this path")
