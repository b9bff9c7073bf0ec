"""``GaussianDistribution`` — the part of gpjax 0.8.2 ``gpjax.distributions`` on the
hot path (called at src/objectives.py:76-78): ``log_prob(y)`` of a dense SPD scale,

    log N(y; loc, S) = -1/2 ( n log 2pi + logdet S + (y - loc)^T S^{-1} (y - loc) ),

with logdet and solve through a Cholesky factor, computed by ``lfm_log_prob_f64``.
A scale that is not positive definite gives NaN (JAX semantics).
"""

from __future__ import annotations

import numpy as np

from ._lib import as_f64, dptr, get_context
from .model import DenseOperator


class GaussianDistribution:
    def __init__(self, loc, scale, device: int | None = None):
        self.loc = as_f64(np.atleast_1d(loc)).reshape(-1)
        s = scale.to_dense() if isinstance(scale, DenseOperator) else scale
        self.scale = as_f64(s)
        n = self.loc.shape[0]
        if self.scale.shape != (n, n):
            raise ValueError(f"scale must be {n} x {n}")
        self.device = device

    def mean(self) -> np.ndarray:
        return self.loc

    def log_prob(self, y) -> float:
        y = as_f64(np.atleast_1d(y)).reshape(-1)
        n = self.loc.shape[0]
        if y.shape[0] != n:
            raise ValueError("y has the wrong length")
        out = np.empty(1)
        ctx = get_context(self.device)
        rc = ctx.lib.lfm_log_prob_f64(ctx.handle, dptr(self.loc), dptr(self.scale), n, n,
                                      dptr(y), dptr(out))
        ctx.check(rc, allow_not_pd=True)
        return float(out[0])
