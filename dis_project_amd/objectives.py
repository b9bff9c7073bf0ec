"""``CustomConjMLL`` — src/objectives.py:19-78 of the reference, on the GPU.

``CustomConjMLL(negative=True)(model, Dataset(X, y))`` returns
``constant * log N(y; m(X), K(X, X) + jitter I + obs_stddev^2 I)`` with
``constant = -1`` if ``negative`` else ``+1`` (gpjax 0.8.2 ``AbstractObjective``).
The whole step — mean, gram, Sigma assembly, Cholesky, solve, logdet — is one call
into ``liblfm.so`` (``lfm_mll_f64``); only the fp64 scalar comes back.

Like the reference's JAX path, a Sigma that is not positive definite yields NaN
rather than an exception.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import HypArgs, LfmProblem, as_f64, dptr
from .dataset import Dataset
from .model import ExactLFM


@dataclass
class CustomConjMLL:
    """objectives.py:19-20 (gpx.objectives.AbstractObjective subclass)."""

    negative: bool = False

    @property
    def constant(self) -> float:
        return -1.0 if self.negative else 1.0

    def __call__(self, model: ExactLFM, train_data: Dataset) -> float:
        return self.step(model, train_data)

    def step(self, model: ExactLFM, train_data: Dataset) -> float:
        """objectives.py:21-78."""
        x = as_f64(train_data.X).reshape(-1, 3)
        y = as_f64(train_data.y).reshape(-1)
        if y.shape[0] != x.shape[0]:
            raise ValueError("X and y must have the same number of rows")
        out = np.empty(1)
        hp = model.hyp()
        ctx = model.ctx
        rc = ctx.lib.lfm_mll_f64(ctx.handle, dptr(x), dptr(y), x.shape[0], hp.ref,
                                 int(self.negative), dptr(out))
        ctx.check(rc, allow_not_pd=True)
        return float(out[0])

    def value_and_grad(self, model: ExactLFM, train_data: Dataset):
        """Value and gradient of ``step`` with respect to the constrained parameters —
        what ``jax.value_and_grad(loss)`` differentiates at trainer.py:126 before the
        bijectors' chain rule (trainer.py:103). One call into ``lfm_mll_grad_f64``.

        Returns ``(value, grads)`` with ``grads = {"true_d": [G], "true_s": [G],
        "true_b": [G], "l": float, "obs_stddev": float}`` (``jitter`` is static,
        model.py:64). A Sigma that is not PD gives NaN everywhere, like JAX.
        """
        x = as_f64(train_data.X).reshape(-1, 3)
        y = as_f64(train_data.y).reshape(-1)
        if y.shape[0] != x.shape[0]:
            raise ValueError("X and y must have the same number of rows")
        G = int(model.num_genes)
        val = np.empty(1)
        g = np.empty(3 * G + 2)
        hp = model.hyp()
        ctx = model.ctx
        rc = ctx.lib.lfm_mll_grad_f64(ctx.handle, dptr(x), dptr(y), x.shape[0], hp.ref,
                                      int(self.negative), dptr(val), dptr(g))
        ctx.check(rc, allow_not_pd=True)
        grads = {"true_d": g[:G].copy(), "true_s": g[G:2 * G].copy(),
                 "true_b": g[2 * G:3 * G].copy(), "l": float(g[3 * G]),
                 "obs_stddev": float(g[3 * G + 1])}
        return float(val[0]), grads

    def batch(self, models, datasets) -> np.ndarray:
        """Independent evaluations (restarts / ablations) in one call; NaN where not PD."""
        models = list(models)
        datasets = list(datasets)
        if len(models) != len(datasets):
            raise ValueError("models and datasets must pair up")
        if not models:
            return np.empty(0)
        keep, probs = [], (LfmProblem * len(models))()
        for i, (m, d) in enumerate(zip(models, datasets)):
            x = as_f64(d.X).reshape(-1, 3)
            y = as_f64(d.y).reshape(-1)
            hp = m.hyp()
            keep.append((x, y, hp))
            probs[i].x = dptr(x)
            probs[i].y = dptr(y)
            probs[i].n = x.shape[0]
            probs[i].hyp = hp.struct
        out = np.empty(len(models))
        st = (_lib.c_int * len(models))()
        ctx = models[0].ctx
        rc = ctx.lib.lfm_mll_batch_f64(ctx.handle, len(models), probs, int(self.negative),
                                       dptr(out), st)
        ctx.check(rc, allow_not_pd=True)
        return out
