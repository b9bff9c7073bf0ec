"""The batched small-N gradient and the on-device fit (VERDICT r04
item 3): ``lfm_batch_mll_grad_f64`` (every problem's value and gradient in one launch) and
``lfm_batch_fit_f64`` / ``trainer.BatchTrainer`` (JaxTrainer.fit of every problem, each
problem's Adam loop inside one kernel) — the reference's actual ablation / p53 workflow
(notebook.py:55-75, main.py:45-59: 150 steps of adam(0.01) on CustomConjMLL(negative=True)).

Oracles: oracle.mll_grad (complex-step derivatives of the reference kernel, explicit inverse)
per component within 1e-8 x the magnitude of its summed terms (as tests/test_gpu_grad.py); the
training trajectories of 15 + 2 oracle-driven JaxTrainer loops (tests/golden/fit_*.npz,
tests/golden/make_golden_fit.py)."""

import os

import numpy as np
import pytest

from dis_project_amd import farm
from oracle import lfm_oracle as O

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
KEYS = (("true_d", "d"), ("true_s", "s"), ("true_b", "b"), ("l", "l"),
        ("obs_stddev", "obs_stddev"))


def _check_grads(vals, grads, models, datasets, negative):
    for v, g, m, d in zip(vals, grads, models, datasets):
        ref = O.mll_grad(d.X, d.y, m.true_d, m.true_s, m.true_b, m.l, m.obs_stddev, m.jitter,
                         negative)
        assert abs(v - ref["value"]) <= 1e-9 * abs(ref["value"]), (v, ref["value"])
        for k, rk in KEYS:
            got, want = np.asarray(g[k]), np.asarray(ref[rk])
            tol = 1e-8 * np.maximum(np.asarray(ref["scale_" + rk]), 1e-300)
            assert np.all(np.abs(got - want) <= tol), (k, got, want, tol)


def _problems(kind, seed=21):
    """Small problems off the dataset_3d grid path: scattered times, a latent row, shuffled
    rows, mixed flags (the per-pair dual-number reduction)."""
    from dis_project_amd.dataset import Dataset, grid_inputs
    from dis_project_amd.model import ExactLFM

    rng = np.random.default_rng(seed)
    models, datasets = [], []
    for kk, (G, T) in enumerate(((4, 7), (3, 9), (5, 7), (2, 16), (1, 20), (6, 5))):
        D, S, B = rng.uniform(0.2, 1.0, G), rng.uniform(0.5, 1.5, G), rng.uniform(0.01, 0.1, G)
        x = grid_inputs(G, T).copy()
        if kind == "scattered":
            if kk % 3 == 0:
                x[:, 0] = rng.uniform(0.0, 12.0, G * T)
            elif kk % 3 == 1:
                x[[2, 7], 2] = 0.0  # latent rows: kernel_xf / kernel_ff pairs
            else:
                x = x[rng.permutation(G * T)]
        y = np.repeat(B / D, T) + 0.5 * rng.standard_normal(G * T)
        models.append(ExactLFM(jitter=1e-4, num_genes=G, true_d=D, true_s=S, true_b=B,
                               l=float(rng.uniform(1.0, 3.4)),
                               obs_stddev=float(rng.uniform(0.3, 1.2))))
        datasets.append(Dataset(np.ascontiguousarray(x), y))
    return models, datasets


@pytest.mark.parametrize("negative", [True, False])
def test_batch_grad_c5_and_c1_vs_oracle(negative):
    """The C5 problems and C1 in one launch: every value within 1e-9 of the oracle and within
    1e-12 of lfm_batch_mll_f64's (the same Sigma; the gradient's one-wave path factors by the
    sweep operator, the MLL kernel by Cholesky), every gradient component within 1e-8 of its
    summed terms' magnitude; a second call gives the same bits."""
    from dis_project_amd import _lib, configs

    models, datasets = farm.workload("c5")
    c1 = configs.c1_p53()
    models, datasets = models + [c1.model], datasets + [c1.data]
    ev = farm.BatchEvaluator(_lib.get_context(), datasets, negative=negative)
    try:
        vals, grads = ev.value_and_grad(models)
        np.testing.assert_allclose(vals, ev(models), rtol=1e-12, atol=0)
        _check_grads(vals, grads, models, datasets, negative)
        vals2, grads2 = ev.value_and_grad(models)
        np.testing.assert_array_equal(vals2, vals)
        for a, b in zip(grads, grads2):
            for k, _ in KEYS:
                np.testing.assert_array_equal(a[k], b[k])
    finally:
        ev.close()


@pytest.mark.parametrize("kind", ["grid", "scattered"])
def test_batch_grad_layouts_vs_oracle(kind):
    """Grid-layout problems of other shapes (the derivative tables, one wave per gene-block
    pair) and problems off the grid (scattered times, latent rows, shuffled rows: the per-pair
    dual-number kernel), n = 15 ... 36, one launch."""
    from dis_project_amd import _lib

    models, datasets = _problems(kind)
    ev = farm.BatchEvaluator(_lib.get_context(), datasets, negative=True)
    try:
        vals, grads = ev.value_and_grad(models)
        _check_grads(vals, grads, models, datasets, True)
    finally:
        ev.close()


def test_batch_grad_memory_path_and_not_pd(monkeypatch):
    """More than 16 problems (the problem table and hyperparameters read from memory, not the
    kernel arguments): the same bits as the argument path; a non-PD problem is NaN with its
    status, the others unaffected; n = 128 is refused (n <= 127)."""
    from dis_project_amd import _lib
    from dis_project_amd.dataset import Dataset, grid_inputs

    models, datasets = farm.workload("c5")
    ctx = _lib.get_context()
    ev = farm.BatchEvaluator(ctx, datasets, negative=True)
    try:
        v16, g16 = ev.value_and_grad(models)
    finally:
        ev.close()
    big = farm.BatchEvaluator(ctx, datasets * 2, negative=True)
    try:
        bad = list(models * 2)
        v32, g32 = big.value_and_grad(bad)
        np.testing.assert_array_equal(v32, np.concatenate([v16, v16]))
        for a, b in zip(g32, g16 + g16):
            for k, _ in KEYS:
                np.testing.assert_array_equal(a[k], b[k])
        bad[20] = bad[20].replace(jitter=-50.0, obs_stddev=0.0)
        v, g = big.value_and_grad(bad)
        assert np.isnan(v[20]) and big.status[20] != 0
        assert np.all(np.isnan(g[20]["true_d"])) and np.isnan(g[20]["l"])
        mask = np.arange(len(bad)) != 20
        np.testing.assert_array_equal(v[mask], v32[mask])
    finally:
        big.close()
    wide = farm.BatchEvaluator(ctx, [Dataset(grid_inputs(4, 32), np.zeros(128))], negative=True)
    try:
        from dis_project_amd.model import ExactLFM

        with pytest.raises(_lib.LfmError) as ei:
            wide.value_and_grad([ExactLFM(jitter=1e-4, num_genes=4)])
        assert ei.value.code == _lib.LFM_E_ARG
    finally:
        wide.close()


def test_batch_grad_two_wave_problems_vs_oracle():
    """Problems past one wave (64 < n + 1 <= 128: the sweep on four waves, one barrier a step):
    the notebook's pooled replicates (N = 105, 84), a shuffled-row N = 96 problem and N = 127,
    in one launch with a small C5 problem (the four-wave sweep and the one-wave one):
    values within 1e-12 of lfm_batch_mll_f64's (whose factor is Cholesky), gradients within
    1e-8 of the oracle's summed terms."""
    from dis_project_amd import _lib, configs
    from dis_project_amd.dataset import Dataset, grid_inputs
    from dis_project_amd.model import ExactLFM

    ws = configs.notebook_pooled()
    models, datasets = [w.model for w in ws[:3]], [w.data for w in ws[:3]]
    rng = np.random.default_rng(96)
    for G, T, shuffle in ((4, 24, True), (1, 127, True)):
        D, S, B = rng.uniform(0.2, 1.0, G), rng.uniform(0.5, 1.5, G), rng.uniform(0.01, 0.1, G)
        x = grid_inputs(G, T)
        if shuffle:
            x = x[rng.permutation(G * T)]
        y = np.repeat(B / D, T) + 0.5 * rng.standard_normal(G * T)
        models.append(ExactLFM(jitter=1e-4, num_genes=G, true_d=D, true_s=S, true_b=B, l=2.1))
        datasets.append(Dataset(np.ascontiguousarray(x), y))
    c5m, c5d = farm.workload("c5")
    models.append(c5m[0])
    datasets.append(c5d[0])
    ev = farm.BatchEvaluator(_lib.get_context(), datasets, negative=True)
    try:
        vals, grads = ev.value_and_grad(models)
        np.testing.assert_allclose(vals, ev(models), rtol=1e-12, atol=0)
        _check_grads(vals, grads, models, datasets, True)
    finally:
        ev.close()


@pytest.mark.parametrize("case", ["fit_c5", "fit_c1", "fit_c1_epoch", "fit_pooled"])
def test_batch_fit_matches_oracle_jaxtrainer(case, golden):
    """JaxTrainer.fit on the device (one launch: 150 Adam steps per problem inside the kernel)
    against the oracle-driven host JaxTrainer loops (tests/golden/make_golden_fit.py): the C5
    ablation fit (15 problems, fix_params=False), main.py's C1 fit (fix_params=True), the same
    with after_epoch every 50 steps, and the notebook's pooled data (N = 105 and 84: two waves). Loss histories within 1e-9 relative, final
    unconstrained and constrained parameters within 1e-9 (relative, absolute below 1)."""
    from dis_project_amd import _lib, configs
    from dis_project_amd import trainer as TR
    from dis_project_amd.objectives import CustomConjMLL

    ref = golden(case)
    if case == "fit_c5":
        models, datasets = farm.workload("c5")
    elif case == "fit_pooled":
        ws = configs.notebook_pooled()
        models, datasets = [w.model for w in ws], [w.data for w in ws]
    else:
        c1 = configs.c1_p53()
        models, datasets = [c1.model], [c1.data]
    bt = TR.BatchTrainer(models, CustomConjMLL(negative=True), datasets, TR.adam(0.01),
                         num_iters=int(ref["iters"]), ctx=_lib.get_context())
    try:
        np.testing.assert_array_equal(
            TR.pack_raw(bt.raws, [m.jitter for m in models]), ref["raw0"])
        out, hist = bt.fit(fix_params=bool(ref["fix_params"]),
                           num_steps_per_epoch=int(ref["spe"]))
        assert not np.any(bt.status)
        np.testing.assert_allclose(hist, ref["hist"], rtol=1e-9, atol=0)
        raw1 = TR.pack_raw(bt.raws, [m.jitter for m in models])
        np.testing.assert_allclose(raw1, ref["raw1"], rtol=1e-9, atol=1e-9)
        final = np.concatenate([np.concatenate([m.true_d, m.true_s, m.true_b, [m.l, m.obs_stddev]])
                                for m in out])
        np.testing.assert_allclose(final, ref["final"], rtol=1e-9, atol=1e-9)
        if ref["fix_params"]:
            assert all(m.true_s[3] == 1.0 and m.true_d[3] == 0.8 for m in out)
    finally:
        bt.close()


def _first_divergence(ha, hist, snaps, fit, raw0, models, datasets):
    """The failure report of a fit-kernel vs host-loop mismatch: the first
    step s1 whose loss differs; at step s0 = s1 - 1 both paths had the same parameters, so the
    step s0 gradient / update of one of them was wrong. Names the path: the host loop's batch
    gradient at s0 against oracle.mll_grad, and each path's raw parameters after s1 steps against
    the Adam step driven by the oracle's gradient."""
    from dis_project_amd import trainer as TR

    bad = np.abs(hist - ha) > 1e-12 * np.abs(ha)
    s1 = int(np.argmax(bad.any(axis=1)))
    p = int(np.argmax(bad[s1]))
    genes = [m.num_genes for m in models]
    if s1 == 0:
        cur = snaps[0][2][p]
        ref = O.mll_grad(datasets[p].X, datasets[p].y, cur.true_d, cur.true_s, cur.true_b,
                         cur.l, cur.obs_stddev, cur.jitter, True)["value"]
        return (f"step 0 problem {p}: fit kernel {ha[0, p]!r}, host loop {hist[0, p]!r}, "
                f"oracle {ref!r}")
    s0 = s1 - 1
    raws0, states0, cur0, grads0 = snaps[s0]
    m, d = cur0[p], datasets[p]
    ref = O.mll_grad(d.X, d.y, m.true_d, m.true_s, m.true_b, m.l, m.obs_stddev, m.jitter, True)
    host_err = max(float(np.max(np.abs(np.asarray(grads0[p][k]) - ref[rk]) /
                                np.maximum(np.asarray(ref["scale_" + rk]), 1e-300)))
                   for k, rk in KEYS)
    g = TR.chain_rule(raws0[p], {k: ref[rk] for k, rk in KEYS})
    upd, _ = TR.adam(0.01).update(g, states0[p], raws0[p])
    want = TR.apply_updates(raws0[p], upd)
    if s0 % 30 == 0:
        want = TR.JaxTrainer.after_epoch(want, True)
    kraw = raw0.copy()
    fit(kraw, np.zeros_like(kraw), np.zeros_like(kraw), 0, s1)
    kern = TR.unpack_raw(kraw, genes)[p]
    host = snaps[s1][0][p]

    def dev(r):
        return max(float(np.max(np.abs(np.asarray(r[k]) - np.asarray(want[k])))) for k in want)

    return (f"first divergence at step {s1}, problem {p}: the host loop's batch gradient at step "
            f"{s0} is {host_err:.3g} x its 1e-8 tolerance from oracle.mll_grad (> 1e-8: the "
            f"gradient path is wrong); raw parameters after {s1} steps vs the oracle-driven Adam "
            f"step: fit kernel {dev(kern):.3g}, host loop {dev(host):.3g} (the larger names the "
            f"wrong path)")


def test_batch_fit_resumes_and_matches_the_batch_gradient_loop():
    """Two fit calls of 40 steps (step0 carries Adam's count and the epoch phase) give the bits
    of one call of 80; and the in-kernel loop equals a host loop driven by
    lfm_batch_mll_grad_f64 (the same gradient kernel, numpy's Adam) to 1e-12. On a mismatch the
    failure names the path that left the oracle at the first diverging step (_first_divergence)."""
    from dis_project_amd import _lib
    from dis_project_amd import trainer as TR

    ctx = _lib.get_context()
    models, datasets = farm.workload("c5")
    models, datasets = models[:5], datasets[:5]
    ev = farm.BatchEvaluator(ctx, datasets, negative=True)
    try:
        genes = [m.num_genes for m in models]
        batch = ev.registered(genes)
        raw0 = TR.pack_raw([TR.unconstrain(m) for m in models], [m.jitter for m in models])
        opt = _lib.LfmAdam(0.01, 0.9, 0.999, 1e-8, 0.0, 30, 1)

        def fit(raw, mu, nu, step0, k):
            hist = np.empty((k, len(models)))
            ctx.check(ctx.lib.lfm_batch_fit_f64(ctx.handle, batch, _lib.ctypes.byref(opt), 1,
                                                step0, k, _lib.dptr(raw), _lib.dptr(mu),
                                                _lib.dptr(nu), _lib.dptr(hist), None))
            return hist

        a = raw0.copy(); ma = np.zeros_like(a); na = np.zeros_like(a)
        ha = fit(a, ma, na, 0, 80)
        b = raw0.copy(); mb = np.zeros_like(b); nb = np.zeros_like(b)
        hb = np.concatenate([fit(b, mb, nb, 0, 40), fit(b, mb, nb, 40, 40)])
        np.testing.assert_array_equal(ha, hb)
        np.testing.assert_array_equal(a, b)
        # the host loop: the batch gradient + trainer.py's chain rule / adam / after_epoch, with
        # each step's state kept for the failure report
        trainers = [TR.JaxTrainer(m, None, d, TR.adam(0.01), num_iters=80)
                    for m, d in zip(models, datasets)]
        raws = [t.raw for t in trainers]
        states = [TR.adam(0.01).init(r) for r in raws]
        hist, snaps = [], []
        for s in range(80):
            cur = [TR.constrain(r, m) for r, m in zip(raws, models)]
            vals, grads = ev.value_and_grad(cur)
            hist.append(vals)
            snaps.append((list(raws), list(states), cur, grads))
            for p in range(len(models)):
                g = TR.chain_rule(raws[p], grads[p])
                upd, states[p] = TR.adam(0.01).update(g, states[p], raws[p])
                raws[p] = TR.apply_updates(raws[p], upd)
                if s % 30 == 0:
                    raws[p] = TR.JaxTrainer.after_epoch(raws[p], True)
        snaps.append((list(raws), list(states), None, None))
        hist = np.asarray(hist)
        if not np.all(np.abs(hist - ha) <= 1e-12 * np.abs(ha)):
            pytest.fail(_first_divergence(ha, hist, snaps, fit, raw0, models, datasets))
        np.testing.assert_allclose(TR.pack_raw(raws, [m.jitter for m in models]), a,
                                   rtol=1e-12, atol=1e-12)
    finally:
        ev.close()


def test_batch_fit_past_256_parameters_vs_cpu_port():
    """A fit whose 3G + 2 parameters exceed the workgroup's 256 threads (G = 85 genes, one row
    each, off the time grid: the four-wave sweep; the largest G whose fit map fits 160 KB of LDS):
    every parameter is updated (the update was one thread per parameter, so
    obs_stddev, parameter 256, stayed frozen), against oracle/lfm_cpu.cpp's JaxTrainer.fit (the
    C++ port) over 4 steps — histories within 1e-9, final raw parameters within 1e-9."""
    from dis_project_amd import _lib
    from dis_project_amd import trainer as TR
    from dis_project_amd.dataset import Dataset
    from dis_project_amd.model import ExactLFM
    from dis_project_amd.objectives import CustomConjMLL
    from oracle import lfm_cpu

    G = 85
    rng = np.random.default_rng(85)
    x = np.stack((rng.uniform(0.0, 12.0, G), np.arange(G, dtype=np.float64), np.ones(G)), -1)
    D, S, B = rng.uniform(0.2, 1.0, G), rng.uniform(0.5, 1.5, G), rng.uniform(0.01, 0.1, G)
    y = B / D + 0.5 * rng.standard_normal(G)
    model = ExactLFM(jitter=1e-4, num_genes=G, true_d=D, true_s=S, true_b=B, l=2.0)
    data = Dataset(np.ascontiguousarray(x), y)
    iters = 4
    bt = TR.BatchTrainer([model], CustomConjMLL(negative=True), [data], TR.adam(0.01),
                         num_iters=iters,
                         ctx=_lib.get_context())
    try:
        raw0 = TR.pack_raw(bt.raws, [model.jitter])
        _, hist = bt.fit(fix_params=False, num_steps_per_epoch=1000)
        assert not np.any(bt.status)
        raw1 = TR.pack_raw(bt.raws, [model.jitter])
    finally:
        bt.close()
    r = np.concatenate([raw0[:3 * G], raw0[3 * G:3 * G + 3]])
    h, _ = lfm_cpu.fit(data.X, data.y, G, r, iters, lr=0.01, spe=1000, fix=False, negative=True)
    np.testing.assert_allclose(np.asarray(hist).reshape(-1), h, rtol=1e-9, atol=0)
    # every parameter moved, obs_stddev (index 3G + 1 > 255) included
    assert np.all(raw1[:3 * G + 2] != raw0[:3 * G + 2])
    np.testing.assert_allclose(raw1[:3 * G + 2], r[:3 * G + 2], rtol=1e-9, atol=1e-9)
