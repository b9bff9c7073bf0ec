"""GPU parity of the MLL gradient (lfm_mll_grad_f64: bordered factorisation + W-weighted
kernel-derivative reduction) against the oracle's complex-step gradient.

Tolerance per component: |g - g_ref| <= 1e-8 * scale + 1e-10 * |g_ref|, where scale is the
oracle's sum of |terms| (1/2 sum |W||dSigma| + |a||dm|): the gradient is a sum of O(n^2)
signed terms, so a relative bar on a component that cancels to ~0 would be meaningless.
The value itself is held to 1e-9 relative (fp64 end to end)."""

import numpy as np
import pytest

from oracle import lfm_oracle as O
from tests.conftest import load_golden

pytestmark = pytest.mark.gpu

KEYS = (("d", "true_d"), ("s", "true_s"), ("b", "true_b"), ("l", "l"),
        ("obs_stddev", "obs_stddev"))


@pytest.fixture(scope="module")
def lfm():
    import dis_project_amd as m
    from dis_project_amd import _lib

    assert _lib.device_count() >= 1, "no HIP device visible"
    return m


def model_of(lfm, D, S, B, l, sd, jit):
    return lfm.ExactLFM(jitter=float(jit), obs_stddev=float(sd), num_genes=len(D), true_d=D,
                        true_s=S, true_b=B, l=float(l))


def check(got_val, got, ref_val, ref_grad, ref_scale, sign=1.0):
    assert got_val == pytest.approx(sign * ref_val, rel=1e-9)
    for ok, gk in KEYS:
        g = np.atleast_1d(got[gk])
        r = sign * np.atleast_1d(ref_grad[ok])
        sc = np.atleast_1d(ref_scale[ok])
        err = np.abs(g - r)
        bound = 1e-8 * sc + 1e-10 * np.abs(r)
        assert np.all(err <= bound), (gk, g, r, err / np.maximum(sc, 1e-300))


@pytest.mark.parametrize("name", ["c1_p53_n35", "grid_n64", "p53_3rep_n105", "scattered_n200",
                                  "mixed_mll_n48", "grid_n512", "kat_zero_times_n32"])
@pytest.mark.parametrize("negative", [False, True])
def test_grad_vs_golden(lfm, name, negative):
    g = load_golden(name)
    m = model_of(lfm, g["D"], g["S"], g["B"], g["l"], g["obs_stddev"], g["jitter"])
    data = lfm.Dataset(g["x"], g["y"].reshape(-1, 1))
    val, gr = lfm.CustomConjMLL(negative=negative).value_and_grad(m, data)
    ref = {k: g["grad_" + k] for k, _ in KEYS}
    sc = {k: g["gscale_" + k] for k, _ in KEYS}
    check(val, gr, float(g["mll"]), ref, sc, -1.0 if negative else 1.0)
    # the value agrees with the MLL-only path
    assert val == pytest.approx(lfm.CustomConjMLL(negative=negative)(m, data), rel=1e-11)


@pytest.mark.parametrize("G,T", [(2, 64), (4, 32), (3, 43), (4, 96)])
def test_grad_block_edges(lfm, G, T):
    """n = 128 (Mp = 256), 128, 129 (ragged), 384: bordered windows at block boundaries."""
    rng = np.random.default_rng(G * 1000 + T)
    D = rng.uniform(0.2, 1.0, G); S = rng.uniform(0.5, 1.5, G); B = rng.uniform(0.01, 0.1, G)
    t = np.linspace(0, 12, T)
    x = np.stack((np.tile(t, G), np.repeat(np.arange(G), T), np.ones(G * T)), -1)
    y = np.repeat(B / D, T) + 0.5 * rng.standard_normal(G * T)
    ref = O.mll_grad(x, y, D, S, B, 2.2, 0.9, 1e-4, negative=True)
    m = model_of(lfm, D, S, B, 2.2, 0.9, 1e-4)
    val, gr = lfm.CustomConjMLL(negative=True).value_and_grad(m, lfm.Dataset(x, y))
    check(val, gr, ref["value"], ref, {k: ref["scale_" + k] for k, _ in KEYS})


def test_grad_not_pd_is_nan(lfm):
    g = load_golden("grid_n64")
    m = model_of(lfm, g["D"], g["S"], g["B"], g["l"], 1e-9, -5.0)  # Sigma = K - 5 I
    val, gr = lfm.CustomConjMLL(negative=True).value_and_grad(m, lfm.Dataset(g["x"], g["y"]))
    assert np.isnan(val)
    assert all(np.all(np.isnan(np.atleast_1d(gr[k]))) for _, k in KEYS)


def test_trainer_on_gpu_matches_oracle_loop(lfm):
    """Ten steps of JaxTrainer.fit (Adam 0.01, -MLL) on C1: the GPU gradient and the
    oracle gradient drive the same host loop to the same history."""
    from dis_project_amd import trainer as TR
    from tests.test_trainer import OracleObjective

    g = load_golden("c1_p53_n35")
    data = lfm.Dataset(g["x"], g["y"].reshape(-1, 1))
    model = lfm.ExactLFM(jitter=1e-4, num_genes=5)
    t_gpu = TR.JaxTrainer(model, lfm.CustomConjMLL(negative=True), data, TR.adam(0.01),
                          num_iters=10)
    m_gpu, h_gpu = t_gpu.fit(num_steps_per_epoch=1000)
    t_cpu = TR.JaxTrainer(model, OracleObjective(True), data, TR.adam(0.01), num_iters=10)
    m_cpu, h_cpu = t_cpu.fit(num_steps_per_epoch=1000)
    np.testing.assert_allclose(h_gpu, h_cpu, rtol=1e-9)
    for k in ("true_d", "true_s", "true_b"):
        np.testing.assert_allclose(getattr(m_gpu, k), getattr(m_cpu, k), rtol=1e-8)
    assert m_gpu.l == pytest.approx(m_cpu.l, rel=1e-8)


@pytest.mark.slow
def test_grad_n1024_vs_oracle(lfm):
    rng = np.random.default_rng(1024)
    G, T = 8, 128
    D = rng.uniform(0.2, 1.0, G); S = rng.uniform(0.5, 1.5, G); B = rng.uniform(0.01, 0.1, G)
    t = np.linspace(0, 12, T)
    x = np.stack((np.tile(t, G), np.repeat(np.arange(G), T), np.ones(G * T)), -1)
    y = np.repeat(B / D, T) + 0.5 * rng.standard_normal(G * T)
    ref = O.mll_grad(x, y, D, S, B, 2.5, 1.0, 1e-4, negative=True)
    m = model_of(lfm, D, S, B, 2.5, 1.0, 1e-4)
    val, gr = lfm.CustomConjMLL(negative=True).value_and_grad(m, lfm.Dataset(x, y))
    check(val, gr, ref["value"], ref, {k: ref["scale_" + k] for k, _ in KEYS})


@pytest.mark.parametrize("env", [{"LFM_SCHED": "1"}, {"LFM_SCHED": "3"},
                                 {"LFM_SCHED": "3", "LFM_W4_MIN": "1024"},
                                 {"LFM_SCHED": "3", "LFM_W4_MIN": "1024", "LFM_S3_EVENTS": "1"},
                                 {"LFM_SCHED": "3", "LFM_GRAD_DIRECT": "1"}])
def test_grad_schedules_vs_oracle(lfm, env, monkeypatch):
    """N = 1024 (4 genes x 256): the bordered inverse through schedule 1 and through schedule
    3's sliding Mp-row window (w = 1 steps; w = 4 super-panels with LFM_W4_MIN=1024; its
    event-ordered profiling mode), each against the oracle's complex-step gradient; the
    gradient reduction through the grid-table kernel (the default on this layout) and through
    the per-pair dual-number kernel (LFM_GRAD_DIRECT=1)."""
    from dis_project_amd import _lib

    for k, v in env.items():
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(4256)
    G, T = 4, 256
    D = rng.uniform(0.2, 1.0, G); S = rng.uniform(0.5, 1.5, G); B = rng.uniform(0.01, 0.1, G)
    t = np.linspace(0, 12, T)
    x = np.stack((np.tile(t, G), np.repeat(np.arange(G), T), np.ones(G * T)), -1)
    y = np.repeat(B / D, T) + 0.5 * rng.standard_normal(G * T)
    ref = O.mll_grad(x, y, D, S, B, 2.3, 0.8, 1e-4, negative=True)
    m = model_of(lfm, D, S, B, 2.3, 0.8, 1e-4)
    ctx = _lib.Context(0)  # schedule knobs are read when a context is created
    try:
        val = np.empty(1)
        gv = np.empty(3 * G + 2)
        hp = m.hyp()
        ctx.check(ctx.lib.lfm_mll_grad_f64(ctx.handle, _lib.dptr(np.ascontiguousarray(x)),
                                           _lib.dptr(y), x.shape[0], hp.ref, 1, _lib.dptr(val),
                                           _lib.dptr(gv)))
    finally:
        ctx.close()
    gr = {"true_d": gv[:G], "true_s": gv[G:2 * G], "true_b": gv[2 * G:3 * G], "l": gv[3 * G],
          "obs_stddev": gv[3 * G + 1]}
    check(float(val[0]), gr, ref["value"], ref, {k: ref["scale_" + k] for k, _ in KEYS})


def test_grad_n16384_schedule3_matches_schedule1(lfm, monkeypatch):
    """C2 at full size (N = 16384): the schedule-3 bordered inverse (the default) and the
    schedule-1 one, and the grid-table gradient kernel (the default) and the per-pair
    dual-number one, give the same value (1e-11) and gradient (1e-9 of the largest component)."""
    from dis_project_amd import _lib, configs

    work = configs.c2()
    x = np.ascontiguousarray(work.data.X)
    y = np.ascontiguousarray(work.data.y.reshape(-1))
    G = work.model.num_genes
    out = {}
    for sched, direct in (("3", "0"), ("1", "0"), ("3", "1")):
        monkeypatch.setenv("LFM_SCHED", sched)
        monkeypatch.setenv("LFM_GRAD_DIRECT", direct)
        ctx = _lib.Context(0)
        try:
            val, gv = np.empty(1), np.empty(3 * G + 2)
            ctx.check(ctx.lib.lfm_mll_grad_f64(ctx.handle, _lib.dptr(x), _lib.dptr(y), x.shape[0],
                                               work.model.hyp().ref, 1, _lib.dptr(val),
                                               _lib.dptr(gv)))
            out[sched + direct] = (float(val[0]), gv.copy())
        finally:
            ctx.close()
    (v3, g3), (v1, g1), (vd, gd) = out["30"], out["10"], out["31"]
    assert v3 == pytest.approx(v1, rel=1e-11)
    assert vd == pytest.approx(v3, rel=1e-11)
    assert np.all(np.isfinite(g3))
    scale = np.max(np.abs(gd))
    assert np.max(np.abs(g3 - g1)) <= 1e-9 * scale, np.max(np.abs(g3 - g1))
    assert np.max(np.abs(g3 - gd)) <= 1e-9 * scale, np.max(np.abs(g3 - gd))
