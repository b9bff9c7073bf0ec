"""Full-size parity (N = 16384, BASELINE.json configs[1] and two configs[2] restarts) against
golden values the CPU oracle computed in the container (tests/golden/make_golden_full.py):
the schedule-3 path exactly as bench.py runs it (w = 4 super-panels, light w = 1 chains), and
the structured fp64 gram on 16 sampled full rows.

Tolerances: MLL 1e-9 relative (north_star: 1e-5) for the C2 base point and restart 0; gram
entries 16 eps M, M the magnitude of the reference formula's intermediate terms
(oracle.gram_error_scale). Restart 1 is ill-conditioned (logdet -7.1e4, quad
7.6e6): there the oracle's own gram rounding (the reference formula cancels to ~eps M) moves
the MLL by ~5e-7 relative, so it is held to the north_star 1e-5 against the oracle, and the
factorisation alone to 1e-9 against scipy's Cholesky of the device's own Sigma."""

import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "full_n16384.npz")
MLL_RTOL = 1e-9


@pytest.fixture(scope="module")
def full():
    if not os.path.exists(GOLDEN):
        pytest.fail("tests/golden/full_n16384.npz missing: run tests/golden/make_golden_full.py")
    return np.load(GOLDEN)


@pytest.fixture(scope="module")
def c2_dev():
    """C2 inputs resident on the device (as bench.py holds them)."""
    from dis_project_amd import _lib, configs

    ctx = _lib.get_context(0)
    work = configs.c2()
    x = np.ascontiguousarray(work.data.X)
    y = np.ascontiguousarray(work.data.y.reshape(-1))
    dx, dy = _lib.c_void_p(), _lib.c_void_p()
    ctx.check(ctx.lib.lfm_dev_alloc(ctx.handle, x.nbytes, _lib.ctypes.byref(dx)))
    ctx.check(ctx.lib.lfm_dev_alloc(ctx.handle, y.nbytes, _lib.ctypes.byref(dy)))
    ctx.check(ctx.lib.lfm_memcpy_h2d(ctx.handle, dx, x.ctypes.data, x.nbytes))
    ctx.check(ctx.lib.lfm_memcpy_h2d(ctx.handle, dy, y.ctypes.data, y.nbytes))
    yield ctx, work, dx, dy
    ctx.lib.lfm_dev_free(ctx.handle, dx)
    ctx.lib.lfm_dev_free(ctx.handle, dy)


@pytest.mark.parametrize("tag,rtol", [("c2", MLL_RTOL), ("c3_r0", MLL_RTOL), ("c3_r1", 1e-5)])
def test_mll_n16384_vs_golden(full, c2_dev, tag, rtol):
    from dis_project_amd import _lib, configs

    ctx, work, dx, dy = c2_dev
    model = work.model if tag == "c2" else configs.c3_restarts(work, 2)[int(tag[-1])]
    hp = model.hyp()
    out = np.empty(1)
    for _ in range(2):  # the second call reuses the workspace and the device counters
        ctx.check(ctx.lib.lfm_mll_f64_dev(ctx.handle, dx, dy, work.n, hp.ref, 0, _lib.dptr(out)))
        ref = float(full[f"{tag}_mll"])
        assert abs(out[0] - ref) <= rtol * abs(ref), (tag, out[0], ref)


def test_mll_n16384_ill_conditioned_factorisation(c2_dev):
    """Restart 1: the device MLL equals the scipy (LAPACK) log-density of the device's own
    Sigma = gram + (jitter + sigma^2) I to 1e-9 — the Cholesky / solve / logdet path is exact to
    fp64 rounding here too; the 5e-7 gap to the oracle is the gram inputs' conditioning."""
    import math

    import scipy.linalg

    from dis_project_amd import _lib, configs

    ctx, work, dx, dy = c2_dev
    model = configs.c3_restarts(work, 2)[1]
    hp = model.hyp()
    n = work.n
    out = np.empty(1)
    ctx.check(ctx.lib.lfm_mll_f64_dev(ctx.handle, dx, dy, n, hp.ref, 0, _lib.dptr(out)))
    sig = np.empty((n, n))
    dK = _lib.c_void_p()
    ctx.check(ctx.lib.lfm_dev_alloc(ctx.handle, n * n * 8, _lib.ctypes.byref(dK)))
    try:
        ctx.check(ctx.lib.lfm_gram_f64_dev(ctx.handle, dx, n, hp.ref,
                                           model.jitter + model.obs_stddev ** 2, 1, dK, n))
        ctx.check(ctx.lib.lfm_memcpy_d2h(ctx.handle, sig.ctypes.data, dK, n * n * 8))
    finally:
        ctx.lib.lfm_dev_free(ctx.handle, dK)
    x = np.ascontiguousarray(work.data.X)
    y = np.ascontiguousarray(work.data.y.reshape(-1))
    from oracle import lfm_oracle as O

    r = y - O.mean_function(x, model.true_d, model.true_b, model.num_genes).reshape(-1)
    c, _ = scipy.linalg.cho_factor(sig, lower=True, overwrite_a=True, check_finite=False)
    z = scipy.linalg.solve_triangular(c, r, lower=True, check_finite=False)
    ref = -0.5 * (n * math.log(2 * math.pi) + 2.0 * np.sum(np.log(np.diag(c))) + z @ z)
    assert abs(out[0] - ref) <= MLL_RTOL * abs(ref), (out[0], ref)


def test_gram_rows_n16384_vs_golden(full, c2_dev):
    from dis_project_amd import _lib

    ctx, work, dx, _ = c2_dev
    n = work.n
    dK = _lib.c_void_p()
    ctx.check(ctx.lib.lfm_dev_alloc(ctx.handle, n * n * 8, _lib.ctypes.byref(dK)))
    try:
        hp = work.model.hyp()
        ctx.check(ctx.lib.lfm_gram_f64_dev(ctx.handle, dx, n, hp.ref, 0.0, 0, dK, n))
        rows = full["c2_rows"]
        got = np.empty((rows.size, n))
        for i, r in enumerate(rows):
            ctx.check(ctx.lib.lfm_memcpy_d2h(ctx.handle, got[i].ctypes.data,
                                             _lib.c_void_p(dK.value + int(r) * n * 8), n * 8))
    finally:
        ctx.lib.lfm_dev_free(ctx.handle, dK)
    ref, scale = full["c2_krows"], full["c2_kscale"]
    err = np.abs(got - ref)
    tol = 16 * np.finfo(np.float64).eps * scale
    assert np.all(err <= tol), (err / tol).max()


def test_dataset_handle_matches_per_call_path(c2_dev):
    """lfm_mll_f64_data (layout analysed once per dataset) returns exactly what
    lfm_mll_f64_dev returns, for two hyperparameter sets and for a small (fused-kernel) n."""
    from dis_project_amd import _lib, configs

    ctx, work, dx, dy = c2_dev
    lib, h = ctx.lib, ctx.handle
    data = _lib.c_void_p()
    ctx.check(lib.lfm_data_create(h, dx, dy, work.n, _lib.ctypes.byref(data)))
    try:
        for model in (work.model, configs.c3_restarts(work, 1)[0]):
            hp = model.hyp()
            a, b = np.empty(1), np.empty(1)
            ctx.check(lib.lfm_mll_f64_dev(h, dx, dy, work.n, hp.ref, 1, _lib.dptr(a)))
            ctx.check(lib.lfm_mll_f64_data(h, data, hp.ref, 1, _lib.dptr(b)))
            assert a[0] == b[0], (a[0], b[0])
    finally:
        lib.lfm_data_destroy(data)
    small = configs.c1_p53()
    x = np.ascontiguousarray(small.data.X)
    y = np.ascontiguousarray(small.data.y.reshape(-1))
    sx, sy = _lib.c_void_p(), _lib.c_void_p()
    ctx.check(lib.lfm_dev_alloc(h, x.nbytes, _lib.ctypes.byref(sx)))
    ctx.check(lib.lfm_dev_alloc(h, y.nbytes, _lib.ctypes.byref(sy)))
    try:
        ctx.check(lib.lfm_memcpy_h2d(h, sx, x.ctypes.data, x.nbytes))
        ctx.check(lib.lfm_memcpy_h2d(h, sy, y.ctypes.data, y.nbytes))
        ctx.check(lib.lfm_data_create(h, sx, sy, x.shape[0], _lib.ctypes.byref(data)))
        hp = small.model.hyp()
        a, b = np.empty(1), np.empty(1)
        ctx.check(lib.lfm_mll_f64(h, _lib.dptr(x), _lib.dptr(y), x.shape[0], hp.ref, 1, _lib.dptr(a)))
        ctx.check(lib.lfm_mll_f64_data(h, data, hp.ref, 1, _lib.dptr(b)))
        lib.lfm_data_destroy(data)
        assert a[0] == b[0], (a[0], b[0])
    finally:
        lib.lfm_dev_free(h, sx)
        lib.lfm_dev_free(h, sy)


@pytest.mark.parametrize("env", [{"LFM_SCHED": "1"}, {"LFM_SCHED": "3", "LFM_S3_EVENTS": "1"}])
def test_mll_n16384_other_schedules_vs_golden(full, env, monkeypatch):
    """The full-size C2 MLL through schedule 1 (potrf / trsm / SYRK launches) and schedule 3
    in its event-ordered profiling mode — each against the golden value at 1e-9."""
    from dis_project_amd import _lib, configs

    for k, v in env.items():
        monkeypatch.setenv(k, v)
    work = configs.c2()
    x = np.ascontiguousarray(work.data.X)
    y = np.ascontiguousarray(work.data.y.reshape(-1))
    ctx = _lib.Context(0)  # knobs are read when a context is created
    try:
        out = np.empty(1)
        hp = work.model.hyp()
        ctx.check(ctx.lib.lfm_mll_f64(ctx.handle, _lib.dptr(x), _lib.dptr(y), x.shape[0], hp.ref,
                                      0, _lib.dptr(out)))
        ref = float(full["c2_mll"])
        assert abs(out[0] - ref) <= MLL_RTOL * abs(ref), (env, out[0], ref)
    finally:
        ctx.close()


@pytest.mark.parametrize("G,T", [(10, 256), (64, 256)])
def test_serialised_schedule3_is_bit_identical(monkeypatch, G, T):
    """LFM_S3_EVENTS=2 (the timed schedule's own launches ordered by events, the mode the PMC
    passes count) gives the default schedule 3's MLL bit for bit: N = 2560 and the C2 size."""
    from dis_project_amd import _lib, configs

    work = configs.grid_workload("serial", G, T, seed_params=7, seed_y=8)
    x = np.ascontiguousarray(work.data.X)
    y = np.ascontiguousarray(work.data.y.reshape(-1))
    hp = work.model.hyp()
    vals = []
    for mode in ("0", "2"):
        monkeypatch.setenv("LFM_SCHED", "3")
        monkeypatch.setenv("LFM_S3_EVENTS", mode)
        ctx = _lib.Context(0)  # read when the context is created
        try:
            out = np.empty(1)
            ctx.check(ctx.lib.lfm_mll_f64(ctx.handle, _lib.dptr(x), _lib.dptr(y), x.shape[0],
                                          hp.ref, 0, _lib.dptr(out)))
            assert ctx.fallbacks == 0
            vals.append(out[0])
        finally:
            ctx.close()
    assert vals[0] == vals[1], vals


@pytest.mark.parametrize("G,T", [(4, 256), (64, 256)])
def test_fused_gram_is_bit_identical(monkeypatch, G, T):
    """The gram fused into the first trailing update (the schedule-3 default on an aligned grid
    layout: the first step's update units generate their Sigma tiles from the tables) gives the
    same MLL, bit for bit, as the separate gram kernel (LFM_GRAM_FUSE=0); N = 1024 and the
    N = 16384 bench workload. The gradient's bordered factorisation fuses too (1e-12)."""
    from dis_project_amd import _lib, configs

    work = configs.grid_workload("fuse", G, T, seed_params=2, seed_y=3)
    x = np.ascontiguousarray(work.data.X)
    y = np.ascontiguousarray(work.data.y.reshape(-1))
    out = {}
    for fuse in ("1", "0"):
        monkeypatch.setenv("LFM_GRAM_FUSE", fuse)
        ctx = _lib.Context(0)  # read at context creation
        try:
            v = np.empty(1)
            ctx.check(ctx.lib.lfm_mll_f64(ctx.handle, _lib.dptr(x), _lib.dptr(y), x.shape[0],
                                          work.model.hyp().ref, 0, _lib.dptr(v)))
            gv, val = np.empty(3 * G + 2), np.empty(1)
            ctx.check(ctx.lib.lfm_mll_grad_f64(ctx.handle, _lib.dptr(x), _lib.dptr(y), x.shape[0],
                                               work.model.hyp().ref, 1, _lib.dptr(val),
                                               _lib.dptr(gv)))
            out[fuse] = (float(v[0]), float(val[0]), gv.copy())
        finally:
            ctx.close()
    (m1, g1v, g1), (m0, g0v, g0) = out["1"], out["0"]
    assert np.isfinite(m1)
    assert m1 == m0
    assert g1v == pytest.approx(g0v, rel=1e-12)
    assert np.max(np.abs(g1 - g0)) <= 1e-12 * np.max(np.abs(g0))


def test_fused_gram_replicated_shuffled_genes(monkeypatch):
    """The fused gram's per-tile gene lookup (block genes through detect_grid): 2 replicates of
    4 genes in a shuffled order, 256 timepoints each (N = 2048), fused vs unfused bit-identical
    and within 1e-9 of the oracle."""
    from dis_project_amd import _lib
    from oracle import lfm_oracle as O

    rng = np.random.default_rng(2048)
    G, T = 4, 256
    order = [2, 0, 3, 1, 2, 0, 3, 1]
    t = np.linspace(0, 12, T)
    x = np.concatenate([np.stack((t, np.full(T, g, float), np.ones(T)), -1) for g in order])
    D = rng.uniform(0.2, 1.0, G); S = rng.uniform(0.5, 1.5, G); B = rng.uniform(0.01, 0.1, G)
    y = (B / D)[np.array(order).repeat(T)] + 0.5 * rng.standard_normal(x.shape[0])
    hyp = _lib.HypArgs(D, S, B, 2.2, 0.9, 1e-4)
    out = {}
    for fuse in ("1", "0"):
        monkeypatch.setenv("LFM_GRAM_FUSE", fuse)
        ctx = _lib.Context(0)
        try:
            v = np.empty(1)
            ctx.check(ctx.lib.lfm_mll_f64(ctx.handle, _lib.dptr(np.ascontiguousarray(x)),
                                          _lib.dptr(y), x.shape[0], hyp.ref, 0, _lib.dptr(v)))
            out[fuse] = float(v[0])
        finally:
            ctx.close()
    assert out["1"] == out["0"]
    ref = O.mll(x, y, D, S, B, 2.2, 0.9, 1e-4, negative=False)
    assert abs(out["1"] - ref) <= MLL_RTOL * abs(ref), (out["1"], ref)


def test_side_cu_helper_is_bit_identical_and_flops_conserved(c2_dev, monkeypatch):
    """The side-CU helper (schedule 3, LFM_HELPER, the default: the tail of long steps'
    trailing updates runs on the 32 chain CUs between chains) changes where units run, not
    what they compute: the N = 16384 MLL is bit-identical with it off, and the algorithmic
    flops the profiler books to the main step launches plus the helper launches equal the
    main launches' alone without it (the host's mirror of the unit enumeration prices the
    helper's share exactly)."""
    from dis_project_amd import _lib

    _, work, dx, dy = c2_dev
    res = {}
    for on in ("1", "0"):
        monkeypatch.setenv("LFM_HELPER", on)
        ctx = _lib.Context(0)  # knobs are read when a context is created
        try:
            v = np.empty(1)
            ctx.check(ctx.lib.lfm_mll_f64_dev(ctx.handle, dx, dy, work.n, work.model.hyp().ref, 0,
                                              _lib.dptr(v)))  # warm
            ctx.profile_reset()
            ctx.profile(True)
            ctx.check(ctx.lib.lfm_mll_f64_dev(ctx.handle, dx, dy, work.n, work.model.hyp().ref, 0,
                                              _lib.dptr(v)))
            ctx.profile(False)
            st = ctx.profile_read()
        finally:
            ctx.close()
        res[on] = (float(v[0]), st.get("syrk", {}).get("flops", 0.0),
                   st.get("syrk_side", {}).get("flops", 0.0),
                   st.get("syrk_side", {}).get("launches", 0))
    (m1, f1, h1, n1), (m0, f0, h0, n0) = res["1"], res["0"]
    assert np.isfinite(m1) and m1 == m0
    assert n1 > 0 and n0 == 0 and h0 == 0.0
    assert f1 + h1 == pytest.approx(f0, rel=1e-12)


def test_side_cu_helper_gradient_bit_identical(monkeypatch):
    """The bordered factorisation of value_and_grad (trainer.py:126) with and without the
    side-CU helper at N = 16384: the same value bit for bit; the gradient to 1e-12 of its
    largest component (its reduction accumulates per-workgroup partial sums with atomics, so
    it is not bit-reproducible from run to run in any case)."""
    from dis_project_amd import _lib, configs

    work = configs.c2()
    x = np.ascontiguousarray(work.data.X)
    y = np.ascontiguousarray(work.data.y.reshape(-1))
    G = work.model.num_genes
    out = {}
    for on in ("1", "0"):
        monkeypatch.setenv("LFM_HELPER", on)
        ctx = _lib.Context(0)  # knobs are read when a context is created
        try:
            gv, val = np.empty(3 * G + 2), np.empty(1)
            ctx.check(ctx.lib.lfm_mll_grad_f64(ctx.handle, _lib.dptr(x), _lib.dptr(y), x.shape[0],
                                               work.model.hyp().ref, 1, _lib.dptr(val),
                                               _lib.dptr(gv)))
        finally:
            ctx.close()
        out[on] = (float(val[0]), gv.copy())
    assert np.isfinite(out["1"][0]) and out["1"][0] == out["0"][0]
    g1, g0 = out["1"][1], out["0"][1]
    assert np.max(np.abs(g1 - g0)) <= 1e-12 * np.max(np.abs(g0))


@pytest.mark.parametrize("G,T", [(16, 256), (10, 200)])
def test_side_cu_helper_forced_on_every_step(monkeypatch, G, T):
    """The side-CU helper forced onto every eligible step (LFM_HELPER_MIN=0, LFM_HELPER_TC=0:
    half of each step's rest triangle on the side CUs, including the w = 2 and w = 1 steps
    where the chain is critical) at N = 4096 (aligned grid, fused gram) and N = 2000 (padded,
    unaligned): slower, but the MLL is bit-identical to the helper off."""
    from dis_project_amd import _lib, configs

    work = configs.grid_workload("helper", G, T, seed_params=2, seed_y=3)
    x = np.ascontiguousarray(work.data.X)
    y = np.ascontiguousarray(work.data.y.reshape(-1))
    out = {}
    for env in ({"LFM_HELPER": "0"},
                {"LFM_HELPER": "1", "LFM_HELPER_MIN": "0", "LFM_HELPER_TC": "0"}):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        ctx = _lib.Context(0)  # knobs are read when a context is created
        try:
            v = np.empty(1)
            ctx.profile_reset()
            ctx.profile(True)
            ctx.check(ctx.lib.lfm_mll_f64(ctx.handle, _lib.dptr(x), _lib.dptr(y), x.shape[0],
                                          work.model.hyp().ref, 0, _lib.dptr(v)))
            ctx.profile(False)
            helpers = ctx.profile_read().get("syrk_side", {}).get("launches", 0)
        finally:
            ctx.close()
        out[env["LFM_HELPER"]] = (float(v[0]), helpers)
    assert out["0"][1] == 0 and out["1"][1] > 0  # the forced run used helper launches
    assert np.isfinite(out["1"][0]) and out["1"][0] == out["0"][0]




def _multi(ctx, data, models, negative=0):
    from dis_project_amd import _lib

    hps = [m.hyp() for m in models]
    arr = (_lib.LfmHyp * len(hps))(*[hp.struct for hp in hps])
    out = np.empty(len(models))
    st = np.full(len(models), -7, np.int32)
    rc = ctx.lib.lfm_mll_multi_f64(ctx.handle, data, len(hps), arr, negative, _lib.dptr(out),
                                   _lib.dptr(st))
    return rc, out, st


@pytest.mark.parametrize("knobs", [{}, {"LFM_OVL_AT": "16384"}, {"LFM_OVERLAP": "0"}])
def test_restart_pipeline_bit_identical(full, c2_dev, monkeypatch, knobs):
    """C3's restart pipeline (lfm_mll_multi_f64: set k + 1's prologue — its gram tables and
    region, chain(0), X_0, chain(1), step 0 — on the overlap stream under set k's tail, the rest
    after set k's launches on the partitioned pair): six N = 16384 restarts, one of them not PD
    (NaN, its status, the others unaffected), bit-identical to one lfm_mll_f64_data call each;
    restarts 0 / 1 against the goldens. Tail start at the default 6144 rows, at 16384 (the next
    set's prologue from the first launch on) and the pipeline off (LFM_OVERLAP=0)."""
    from dis_project_amd import _lib, configs

    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    _, work, dx, dy = c2_dev
    ctx = _lib.Context(0)  # the knobs are read at context creation
    data = _lib.c_void_p()
    try:
        ctx.check(ctx.lib.lfm_data_create(ctx.handle, dx, dy, work.n, _lib.ctypes.byref(data)))
        models = configs.c3_restarts(work, 6)
        models[3] = models[3].replace(jitter=-50.0, obs_stddev=0.0)
        rc, got, st = _multi(ctx, data, models)
        assert rc == _lib.LFM_E_NOT_PD and st[3] == _lib.LFM_E_NOT_PD and np.isnan(got[3])
        assert np.all(st[[0, 1, 2, 4, 5]] == 0)
        one = np.empty(1)
        for k, m in enumerate(models):
            rc1 = ctx.lib.lfm_mll_f64_data(ctx.handle, data, m.hyp().ref, 0, _lib.dptr(one))
            if k == 3:
                assert rc1 == _lib.LFM_E_NOT_PD
                continue
            ctx.check(rc1)
            assert got[k] == one[0], (k, got[k], one[0])
        for k, rtol in ((0, MLL_RTOL), (1, 1e-5)):
            ref = float(full[f"c3_r{k}_mll"])
            assert abs(got[k] - ref) <= rtol * abs(ref), (k, got[k], ref)
        # a second call reuses the workspaces; the same bits
        rc2, got2, _ = _multi(ctx, data, models)
        assert rc2 == _lib.LFM_E_NOT_PD
        np.testing.assert_array_equal(got2, got)
        assert ctx.fallbacks == 0
    finally:
        if data:
            ctx.lib.lfm_data_destroy(data)
        ctx.close()


def test_restart_pipeline_small_and_grid_sizes():
    """The pipeline on an aligned grid (G = 16, T = 256: N = 4096, the fused gram) and off it
    (G = 8, T = 100: N = 800, the separate gram fill), four sets each, bit-identical to one call
    per set; a schedule change on the context drops the pipeline's workspaces (they borrow its
    stream pair) and the next call rebuilds them."""
    from dis_project_amd import _lib, configs

    ctx = _lib.get_context(0)
    for G, T in ((16, 256), (8, 100)):
        work = configs.grid_workload(f"pipe_{G}x{T}", G, T, seed_params=7, seed_y=8)
        x = np.ascontiguousarray(work.data.X)
        y = np.ascontiguousarray(work.data.y.reshape(-1))
        dx, dy, data = _lib.c_void_p(), _lib.c_void_p(), _lib.c_void_p()
        ctx.check(ctx.lib.lfm_dev_alloc(ctx.handle, x.nbytes, _lib.ctypes.byref(dx)))
        ctx.check(ctx.lib.lfm_dev_alloc(ctx.handle, y.nbytes, _lib.ctypes.byref(dy)))
        try:
            ctx.check(ctx.lib.lfm_memcpy_h2d(ctx.handle, dx, x.ctypes.data, x.nbytes))
            ctx.check(ctx.lib.lfm_memcpy_h2d(ctx.handle, dy, y.ctypes.data, y.nbytes))
            ctx.check(ctx.lib.lfm_data_create(ctx.handle, dx, dy, work.n, _lib.ctypes.byref(data)))
            models = configs.c3_restarts(work, 4)
            for rep in range(2):
                rc, got, st = _multi(ctx, data, models, negative=1)
                assert rc in (0, _lib.LFM_E_NOT_PD) and np.sum(st == 0) >= 2, (rc, st)
                one = np.empty(1)
                for k, m in enumerate(models):
                    rc1 = ctx.lib.lfm_mll_f64_data(ctx.handle, data, m.hyp().ref, 1,
                                                   _lib.dptr(one))
                    assert rc1 == st[k], (G, T, k, rc1, st[k])
                    if rc1 == 0:
                        assert got[k] == one[0], (G, T, k, got[k], one[0])
                if rep == 0:
                    ctx.schedule = 1
                    ctx.schedule = 3
        finally:
            if data:
                ctx.lib.lfm_data_destroy(data)
            ctx.lib.lfm_dev_free(ctx.handle, dx)
            ctx.lib.lfm_dev_free(ctx.handle, dy)
