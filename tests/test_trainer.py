"""Host logic of the training loop (trainer.py:36-228 mirror): bijectors, their chain rule,
optax.adam, the after-epoch quirk. The objective injected here is the CPU oracle
(test-only); tests/test_gpu_grad.py runs the same loop on liblfm's gradient."""

import numpy as np
import pytest

from dis_project_amd import ExactLFM, trainer as TR
from dis_project_amd.dataset import Dataset
from oracle import lfm_oracle as O
from tests.conftest import load_golden


class OracleObjective:
    def __init__(self, negative=True):
        self.negative = negative

    def value_and_grad(self, model, data):
        g = O.mll_grad(data.X, data.y, model.true_d, model.true_s, model.true_b, model.l,
                       model.obs_stddev, model.jitter, self.negative)
        return g["value"], {"true_d": g["d"], "true_s": g["s"], "true_b": g["b"],
                            "l": g["l"], "obs_stddev": g["obs_stddev"]}


def c1():
    g = load_golden("c1_p53_n35")
    return ExactLFM(jitter=1e-4, num_genes=5), Dataset(g["x"], g["y"].reshape(-1, 1))


def test_bijector_round_trip():
    m = ExactLFM(num_genes=3, true_d=[0.2, 0.9, 3.0], true_s=[1e-3, 1.0, 7.0],
                 true_b=[0.05, 0.5, 2.0], l=0.7, obs_stddev=0.3)
    back = TR.constrain(TR.unconstrain(m), m)
    for k in ("true_d", "true_s", "true_b"):
        np.testing.assert_allclose(getattr(back, k), getattr(m, k), rtol=1e-12)
    assert back.l == pytest.approx(0.7, rel=1e-12)
    assert back.obs_stddev == pytest.approx(0.3, rel=1e-12)
    assert TR.l_forward(0.0) == pytest.approx(2.0)  # midpoint of (0.5, 3.5)


def test_chain_rule_matches_finite_differences():
    model, data = c1()
    model = model.replace(true_d=[0.3, 0.5, 0.4, 0.8, 0.6], l=1.9, obs_stddev=0.8)
    obj = OracleObjective(negative=True)
    t = TR.JaxTrainer(model, obj, data, TR.adam(0.01), num_iters=1)
    raw = t.raw
    _, g = t.loss_and_grad(raw, data)

    def f(r):
        return obj.value_and_grad(TR.constrain(r, model), data)[0]

    h = 1e-6
    for k in ("true_d", "true_s", "true_b"):
        for i in range(5):
            rp = {kk: np.array(v, copy=True) for kk, v in raw.items()}
            rm = {kk: np.array(v, copy=True) for kk, v in raw.items()}
            rp[k][i] += h
            rm[k][i] -= h
            assert g[k][i] == pytest.approx((f(rp) - f(rm)) / (2 * h), rel=1e-5, abs=1e-7)
    for k in ("l", "obs_stddev"):
        rp, rm = dict(raw), dict(raw)
        rp[k] = raw[k] + h
        rm[k] = raw[k] - h
        assert g[k] == pytest.approx((f(rp) - f(rm)) / (2 * h), rel=1e-5, abs=1e-7)


def test_adam_matches_optax_formula():
    opt = TR.adam(0.01)
    p = {"a": np.array([1.0, -2.0]), "b": 0.5}
    st = opt.init(p)
    g1 = {"a": np.array([0.3, -0.1]), "b": 2.0}
    g2 = {"a": np.array([-0.2, 0.4]), "b": -1.0}
    u1, st = opt.update(g1, st)
    # first step: mu_hat = g, nu_hat = g^2 -> update = -lr g / (|g| + eps)
    np.testing.assert_allclose(u1["a"], -0.01 * np.sign(g1["a"]) * np.abs(g1["a"]) /
                               (np.abs(g1["a"]) + 1e-8), rtol=1e-12)
    u2, st = opt.update(g2, st)
    mu = 0.9 * (0.1 * g1["a"]) + 0.1 * g2["a"]
    nu = 0.999 * (0.001 * g1["a"] ** 2) + 0.001 * g2["a"] ** 2
    ref = -0.01 * (mu / (1 - 0.81)) / (np.sqrt(nu / (1 - 0.999**2)) + 1e-8)
    np.testing.assert_allclose(u2["a"], ref, rtol=1e-12)
    assert st.count == 2


def test_fit_loop_and_after_epoch_quirk():
    model, data = c1()
    t = TR.JaxTrainer(model, OracleObjective(True), data, TR.adam(0.01), num_iters=4)
    out_model, hist = t.fit(fix_params=True, num_steps_per_epoch=1000)
    assert hist.shape == (4,)
    assert np.all(np.isfinite(hist))
    assert hist[-1] < hist[0]  # Adam on -MLL descends from the reference init
    # trainer.py:220-224: the constrained model gets p21's values at the end
    assert out_model.true_s[3] == 1.0 and out_model.true_d[3] == 0.8
    # trainer.py:210-215: at step 0 the *unconstrained* leaves were set to 1.0 / 0.8 and then
    # moved by three Adam steps of size <= lr each
    assert abs(t.raw["true_s"][3] - 1.0) <= 3 * 0.01 + 1e-12
    assert abs(t.raw["true_d"][3] - 0.8) <= 3 * 0.01 + 1e-12
    no_fix = TR.JaxTrainer(model, OracleObjective(True), data, TR.adam(0.01), num_iters=2,
                           track_parameters=["s"])
    m2, h2, tracked = no_fix.fit(fix_params=False)
    assert tracked == {"s": []}
    assert h2[0] == pytest.approx(hist[0], rel=1e-14)
