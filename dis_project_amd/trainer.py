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
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any

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
        upd = {k: -self.learning_rate * (mu[k] / c1) / (np.sqrt(nu[k] / c2 + self.eps_root)
                                                         + self.eps) for k in grads}
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
        out["true_s"][3] = 1.0
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
