"""``JaxTrainer`` — src/trainer.py:36-228 of the reference, driving liblfm's MLL gradient.

The reference trains in the unconstrained space of the model's bijectors
(``self.model = model.unconstrain()``, trainer.py:75): each step evaluates
``objective(model.constrain(), batch)`` and its gradient with ``jax.value_and_grad``
(trainer.py:103, 126), applies an optax update (trainer.py:127-128) and, every
``num_steps_per_epoch`` steps (step 0 included), runs ``after_epoch_jax`` on the
*unconstrained* model (trainer.py:210-215). After the scan the model is constrained and
``after_epoch_jax`` runs once more on the constrained values (trainer.py:220-224).

Here ``objective.value_and_grad(model, data)`` (``CustomConjMLL.value_and_grad``: one
``lfm_mll_grad_f64`` call on the GPU) returns the gradient with respect to the constrained
parameters; the bijectors' chain rule is applied on the host:
    true_d, true_s, true_b, obs_stddev: tfb.Softplus  (model.py:66, 79, 86, 93)
    l:                                  tfb.Sigmoid(low=0.5, high=3.5)  (model.py:111)
``adam`` restates optax.adam (b1 0.9, b2 0.999, eps 1e-8, eps_root 0; main.py:45 uses
learning rate 0.01).

``BatchTrainer`` runs JaxTrainer.fit for many independent problems at once — the reference's
ablation / replicate training runs (notebook.py:33-75, one JaxTrainer per problem; main.py:59)
— with every step on the GPU: ``lfm_batch_fit_f64`` steps each problem's Adam loop inside one
kernel launch (one workgroup per problem), with the same constrain / chain rule / adam /
after_epoch arithmetic as this module's host loop.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Sequence

import numpy as np

from .dataset import Dataset
from .model import ExactLFM

PARAMS = ("true_d", "true_s", "true_b", "l", "obs_stddev")
L_LOW, L_HIGH = 0.5, 3.5


def softplus(x):
    return np.logaddexp(0.0, np.asarray(x, np.float64))


def softplus_inverse(y):
    y = np.asarray(y, np.float64)
    return y + np.log(-np.expm1(-y))


def sigmoid(x):
    x = np.asarray(x, np.float64)
    return np.where(x >= 0, 1.0 / (1.0 + np.exp(-np.abs(x))),
                    np.exp(-np.abs(x)) / (1.0 + np.exp(-np.abs(x))))


def l_forward(x):
    """tfb.Sigmoid(low, high): low + (high - low) sigmoid(x)."""
    return L_LOW + (L_HIGH - L_LOW) * sigmoid(x)


def l_inverse(y):
    u = (np.asarray(y, np.float64) - L_LOW) / (L_HIGH - L_LOW)
    return np.log(u) - np.log1p(-u)


def unconstrain(model: ExactLFM) -> dict:
    """gpjax Module.unconstrain(): parameter leaves through the bijectors' inverses."""
    return {"true_d": softplus_inverse(model.true_d), "true_s": softplus_inverse(model.true_s),
            "true_b": softplus_inverse(model.true_b), "l": float(l_inverse(model.l)),
            "obs_stddev": float(softplus_inverse(model.obs_stddev))}


def constrain(raw: dict, like: ExactLFM) -> ExactLFM:
    """gpjax Module.constrain(): static fields (jitter, num_genes) come from `like`."""
    return like.replace(true_d=softplus(raw["true_d"]), true_s=softplus(raw["true_s"]),
                        true_b=softplus(raw["true_b"]), l=float(l_forward(raw["l"])),
                        obs_stddev=float(softplus(raw["obs_stddev"])))


def chain_rule(raw: dict, g: dict) -> dict:
    """d loss / d raw = d loss / d constrained * bijector'(raw)."""
    s_l = sigmoid(raw["l"])
    return {"true_d": g["true_d"] * sigmoid(raw["true_d"]),
            "true_s": g["true_s"] * sigmoid(raw["true_s"]),
            "true_b": g["true_b"] * sigmoid(raw["true_b"]),
            "l": float(g["l"] * (L_HIGH - L_LOW) * s_l * (1.0 - s_l)),
            "obs_stddev": float(g["obs_stddev"] * sigmoid(raw["obs_stddev"]))}


@dataclass
class AdamState:
    count: int
    mu: dict
    nu: dict


@dataclass
class adam:  # noqa: N801 — optax.adam(learning_rate) spelling
    """optax.adam: scale_by_adam(b1, b2, eps, eps_root) then scale(-learning_rate)."""

    learning_rate: float
    b1: float = 0.9
    b2: float = 0.999
    eps: float = 1e-8
    eps_root: float = 0.0

    def init(self, params: dict) -> AdamState:
        z = {k: np.zeros_like(np.asarray(v, np.float64)) for k, v in params.items()}
        return AdamState(0, z, {k: v.copy() for k, v in z.items()})

    def update(self, grads: dict, state: AdamState, params: Any = None):
        count = state.count + 1
        mu = {k: self.b1 * state.mu[k] + (1 - self.b1) * np.asarray(g) for k, g in grads.items()}
        nu = {k: self.b2 * state.nu[k] + (1 - self.b2) * np.square(np.asarray(g))
              for k, g in grads.items()}
        c1 = 1 - self.b1**count
        c2 = 1 - self.b2**count
        # optax's order: scale_by_adam's mu_hat / (sqrt(nu_hat + eps_root) + eps), then
        # scale(-learning_rate) multiplies
        upd = {k: -self.learning_rate * ((mu[k] / c1) / (np.sqrt(nu[k] / c2 + self.eps_root)
                                                          + self.eps)) for k in grads}
        return upd, AdamState(count, mu, nu)


def apply_updates(params: dict, updates: dict) -> dict:
    out = {}
    for k, v in params.items():
        nv = np.asarray(v, np.float64) + updates[k]
        out[k] = float(nv) if np.ndim(nv) == 0 else nv
    return out


@dataclass
class JaxTrainer:
    """trainer.py:36-228. `objective` must offer ``value_and_grad(model, data)``."""

    model: ExactLFM
    objective: Any
    training_data: Dataset
    optim: adam
    key: Any = None
    num_iters: int = 150
    track_parameters: Any = None
    history: Any = field(default_factory=list)

    def __post_init__(self):
        self._like = self.model
        self.raw = unconstrain(self.model)  # trainer.py:75
        self.track_parameters = ({k: [] for k in self.track_parameters}
                                 if self.track_parameters else None)

    def loss_and_grad(self, raw: dict, batch: Dataset):
        """trainer.py:103 + 126: objective(model.constrain(), batch) and d/d raw."""
        value, g = self.objective.value_and_grad(constrain(raw, self._like), batch)
        return value, chain_rule(raw, g)

    def step(self, carry, key=None, step_count=0):
        """trainer.py:105-132."""
        raw, opt_state = carry
        loss_val, grad = self.loss_and_grad(raw, self.training_data)
        updates, opt_state = self.optim.update(grad, opt_state, raw)
        raw = apply_updates(raw, updates)
        return (raw, opt_state), loss_val

    @staticmethod
    def after_epoch(params: dict, fix_params: bool) -> dict:
        """trainer.py:134-160 (index 3: p21's sensitivity 1.0 and decay 0.8)."""
        if not fix_params:
            return params
        out = dict(params)
        out["true_s"] = np.array(params["true_s"], np.float64).copy()
        out["true_d"] = np.array(params["true_d"], np.float64).copy()
        # JAX drops an out-of-bounds .at[3].set(...) (G <= 3): nothing changes then
        if out["true_s"].size > 3:
            out["true_s"][3] = 1.0
        if out["true_d"].size > 3:
            out["true_d"][3] = 0.8
        return out

    def fit(self, fix_params: bool = True, num_steps_per_epoch: int = 1000):
        """trainer.py:162-228."""
        state = self.optim.init(self.raw)
        raw = self.raw
        history = []
        for step_count in range(self.num_iters):
            (raw, state), loss_val = self.step((raw, state), None, step_count)
            if step_count % num_steps_per_epoch == 0:
                raw = self.after_epoch(raw, fix_params)  # on the unconstrained model
            history.append(loss_val)
        model = constrain(raw, self._like)
        if fix_params:
            c = self.after_epoch({"true_s": model.true_s, "true_d": model.true_d}, True)
            model = model.replace(true_s=c["true_s"], true_d=c["true_d"])
        self.model = model
        self.raw = raw
        self.history = np.asarray(history)
        if self.track_parameters:
            return self.model, self.history, self.track_parameters
        return self.model, self.history


def pack_raw(raws: Sequence[dict], jitters: Sequence[float]) -> np.ndarray:
    """Unconstrained parameters of P problems in lfm_batch's packed layout: raw true_d, true_s,
    true_b of each problem in order, then raw l, raw obs_stddev and the (static, constrained)
    jitter of each."""
    vec = [np.concatenate([np.asarray(r["true_d"], np.float64), np.asarray(r["true_s"], np.float64),
                           np.asarray(r["true_b"], np.float64)]) for r in raws]
    sc = [[float(r["l"]), float(r["obs_stddev"]), float(j)] for r, j in zip(raws, jitters)]
    return np.concatenate(vec + [np.asarray(sc, np.float64).reshape(-1)])


def unpack_raw(packed: np.ndarray, genes: Sequence[int]) -> list:
    """pack_raw's inverse (the jitter slots dropped)."""
    out, off = [], 0
    nvec = 3 * int(sum(genes))
    for p, G in enumerate(genes):
        v = packed[off:off + 3 * G]
        sc = packed[nvec + 3 * p: nvec + 3 * p + 3]
        out.append({"true_d": v[:G].copy(), "true_s": v[G:2 * G].copy(), "true_b": v[2 * G:].copy(),
                    "l": float(sc[0]), "obs_stddev": float(sc[1])})
        off += 3 * G
    return out


@dataclass
class BatchTrainer:
    """``JaxTrainer`` (trainer.py:36-228) over P independent (model, dataset) problems at once:
    ``fit`` runs every problem's ``num_iters`` training steps on the GPU in ONE launch
    (``lfm_batch_fit_f64``: one workgroup per problem, its Adam loop inside the kernel, no host
    round trip between steps; n <= 127 per problem). Per problem the semantics are JaxTrainer's:
    training in the bijectors' unconstrained space (trainer.py:75), the objective's value and
    gradient at the constrained model (trainer.py:103, 126), ``optim`` (an ``adam``) on the
    unconstrained leaves (trainer.py:127-128), ``after_epoch`` on the unconstrained model every
    ``num_steps_per_epoch`` steps (step 0 included, trainer.py:205-210), then the constrained
    model with ``after_epoch`` once more (trainer.py:218-222). ``objective`` is a
    ``CustomConjMLL`` (its ``negative``). The datasets are registered in HBM once
    (farm.BatchEvaluator); ``close()`` releases them."""

    models: Sequence[ExactLFM]
    objective: Any
    training_data: Sequence[Dataset]
    optim: adam
    key: Any = None
    num_iters: int = 150
    ctx: Any = None
    history: Any = None

    def __post_init__(self):
        from . import _lib
        from .farm import BatchEvaluator

        self.models = list(self.models)
        self.training_data = list(self.training_data)
        if len(self.models) != len(self.training_data):
            raise ValueError("one model per dataset")
        self._like = list(self.models)
        self.raws = [unconstrain(m) for m in self.models]  # trainer.py:75
        self.ctx = self.ctx or _lib.get_context()
        self._ev = BatchEvaluator(self.ctx, self.training_data, bool(self.objective.negative))

    def fit(self, fix_params: bool = True, num_steps_per_epoch: int = 1000):
        """trainer.py:162-228 for every problem; returns (models, histories [P, num_iters])."""
        from . import _lib

        genes = [int(m.num_genes) for m in self._like]
        batch = self._ev.registered(genes)
        raw = pack_raw(self.raws, [m.jitter for m in self._like])
        mu, nu = np.zeros_like(raw), np.zeros_like(raw)
        hist = np.empty((self.num_iters, len(genes)))
        st = np.zeros(len(genes), np.int32)
        o = self.optim
        opt = _lib.LfmAdam(o.learning_rate, o.b1, o.b2, o.eps, o.eps_root,
                           int(num_steps_per_epoch), int(bool(fix_params)))
        rc = self.ctx.lib.lfm_batch_fit_f64(self.ctx.handle, batch, _lib.ctypes.byref(opt),
                                            int(bool(self.objective.negative)), 0, self.num_iters,
                                            _lib.dptr(raw), _lib.dptr(mu), _lib.dptr(nu),
                                            _lib.dptr(hist), _lib.dptr(st))
        self.ctx.check(rc, allow_not_pd=True)
        self.status = st
        self.raws = unpack_raw(raw, genes)
        out = []
        for r, like in zip(self.raws, self._like):
            m = constrain(r, like)
            if fix_params:  # trainer.py:218-222, on the constrained model
                c = JaxTrainer.after_epoch({"true_s": m.true_s, "true_d": m.true_d}, True)
                m = m.replace(true_s=c["true_s"], true_d=c["true_d"])
            out.append(m)
        self.models = out
        self.history = hist.T.copy()
        return self.models, self.history

    def close(self):
        self._ev.close()


def fit_records(raws: Sequence[dict], hist: np.ndarray, gmax: int) -> np.ndarray:
    """Each problem's fit result as one fixed-length fp64 record (FarmTrainer's exchange):
    raw true_d / true_s / true_b (G each, NaN-padded to gmax), raw l, raw obs_stddev, then the
    loss history. hist: [P, iters]."""
    hist = np.asarray(hist, np.float64)
    rec = np.full((len(raws), 3 * gmax + 2 + hist.shape[1]), np.nan)
    for q, r in enumerate(raws):
        G = np.asarray(r["true_d"]).size
        for k, key in enumerate(("true_d", "true_s", "true_b")):
            rec[q, k * gmax: k * gmax + G] = r[key]
        rec[q, 3 * gmax] = r["l"]
        rec[q, 3 * gmax + 1] = r["obs_stddev"]
        rec[q, 3 * gmax + 2:] = hist[q]
    return rec


def unfit_records(rec: np.ndarray, genes: Sequence[int], gmax: int):
    """fit_records' inverse: (raws, hist [P, iters])."""
    raws = []
    for q, G in enumerate(genes):
        r = rec[q]
        raws.append({"true_d": r[:G].copy(), "true_s": r[gmax:gmax + G].copy(),
                     "true_b": r[2 * gmax:2 * gmax + G].copy(), "l": float(r[3 * gmax]),
                     "obs_stddev": float(r[3 * gmax + 1])})
    return raws, np.ascontiguousarray(rec[:, 3 * gmax + 2:])


class FarmTrainer:
    """``JaxTrainer.fit`` of P independent problems farmed over W ranks (one process per GPU;
    the reference runs one JaxTrainer.fit per ablation problem, notebook.py:58-75 over
    trainer.py:162-228): rank r fits its static block ``farm.partition(P, W, r)`` in ONE
    ``lfm_batch_fit_f64`` launch (a BatchTrainer over the block), then ONE all-gather exchanges
    every problem's final raw parameters and loss history as NaN-padded fixed-length records
    (``Farm.run_records``, ``fit_records``). Every rank ends with every problem's fitted model
    and history — the bits of a one-rank BatchTrainer.fit of all P (each problem's fit is one
    workgroup's, whatever else shares its launch). ``fit`` always starts from the models given
    here (a fresh JaxTrainer per problem). ``block_fit(indices, fix_params, spe) -> (raws,
    hist)`` replaces the GPU block (the CPU tests drive the exchange with the C++ port)."""

    def __init__(self, models, objective, training_data, optim: adam, farm, num_iters: int = 150,
                 ctx: Any = None, block_fit=None):
        self.models = list(models)
        self.training_data = list(training_data)
        if len(self.models) != len(self.training_data):
            raise ValueError("one model per dataset")
        self.objective, self.optim, self.farm = objective, optim, farm
        self.num_iters, self.ctx = int(num_iters), ctx
        self.genes = [int(m.num_genes) for m in self.models]
        self.gmax = max(self.genes)
        self._raw0 = [unconstrain(m) for m in self.models]
        self._block_fit = block_fit or self._gpu_block
        self._bt = None
        self.raws, self.history = None, None

    def _gpu_block(self, idx, fix_params, spe):
        if self._bt is None:
            self._bt = BatchTrainer([self.models[i] for i in idx], self.objective,
                                    [self.training_data[i] for i in idx], self.optim,
                                    num_iters=self.num_iters, ctx=self.ctx)
        self._bt.raws = [self._raw0[i] for i in idx]
        _, hist = self._bt.fit(fix_params=fix_params, num_steps_per_epoch=spe)
        return self._bt.raws, hist

    def fit(self, fix_params: bool = True, num_steps_per_epoch: int = 1000):
        """trainer.py:162-228 for every problem, farmed; returns (models, histories [P, iters])
        on every rank."""
        def block(idx):
            raws, hist = self._block_fit(list(idx), fix_params, num_steps_per_epoch)
            return fit_records(raws, hist, self.gmax)

        rec = self.farm.run_records(len(self.models), 3 * self.gmax + 2 + self.num_iters, block)
        self.raws, self.history = unfit_records(rec, self.genes, self.gmax)
        out = []
        for r, like in zip(self.raws, self.models):
            m = constrain(r, like)
            if fix_params:  # trainer.py:218-222, on the constrained model
                c = JaxTrainer.after_epoch({"true_s": m.true_s, "true_d": m.true_d}, True)
                m = m.replace(true_s=c["true_s"], true_d=c["true_d"])
            out.append(m)
        return out, self.history

    def close(self):
        if self._bt is not None:
            self._bt.close()
            self._bt = None
