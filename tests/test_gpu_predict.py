"""GPU parity of the posterior predictors (model.py:420-514) — lfm_posterior_f64, a Schur
complement on the Cholesky kernels — against the oracle (explicit inverse / Cholesky solve).
Tolerance: |d| <= 1e-9 * max|ref| + 1e-12 (fp64, Sigma well conditioned: obs noise or the
data variances on its diagonal)."""

import numpy as np
import pytest

from oracle import lfm_oracle as O
from tests.conftest import load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lfm():
    import dis_project_amd as m
    from dis_project_amd import _lib

    assert _lib.device_count() >= 1, "no HIP device visible"
    return m


def close(a, b, rtol=1e-9):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape
    assert np.max(np.abs(a - b)) <= rtol * np.max(np.abs(b)) + 1e-12


@pytest.mark.parametrize("tag", ["rep0", "all"])
def test_predictors_vs_golden(lfm, tag):
    from dis_project_amd import dataset as ds

    g = load_golden(f"predict_p53_{tag}")
    data = ds.SyntheticP53Data(replicate=0 if tag == "rep0" else None, seed=5)
    x, y, v = ds.dataset_3d(data)
    np.testing.assert_array_equal(x, g["x"])
    np.testing.assert_array_equal(y.reshape(-1), g["y"])
    m = lfm.ExactLFM(jitter=float(g["jitter"]), obs_stddev=float(g["obs_stddev"]), num_genes=5,
                     true_d=g["D"], true_s=g["S"], true_b=g["B"], l=float(g["l"]))
    lat = m.latent_predict(g["t_lat"], data)
    close(lat.loc, g["lat_mean"])
    close(lat.scale, g["lat_var"])
    gene = m.multi_gene_predict(g["t_gene"], data)
    close(gene.loc, g["gene_mean"])
    close(gene.scale, g["gene_var"])


@pytest.mark.parametrize("n_genes,T,m", [(4, 250, 300), (3, 43, 129)])
def test_posterior_schur_sizes(lfm, n_genes, T, m):
    """n = 1000 (several block columns, Np = 1024) and ragged n = 129 with m = 129 test rows:
    the raw C-ABI posterior against the oracle's Cholesky solve."""
    from dis_project_amd import _lib

    rng = np.random.default_rng(T)
    D = rng.uniform(0.2, 1.0, n_genes); S = rng.uniform(0.5, 1.5, n_genes)
    B = rng.uniform(0.01, 0.1, n_genes)
    n = n_genes * T
    x = np.stack((rng.uniform(0, 12, n), rng.integers(0, n_genes, n).astype(float),
                  np.ones(n)), -1)
    y = rng.normal(0.4, 0.5, n)
    v = rng.uniform(0.01, 0.05, n)
    mm = m - m % n_genes
    t = np.stack((rng.uniform(0, 13, mm), rng.integers(-1, n_genes + 1, mm).astype(float),
                  rng.integers(0, 2, mm).astype(float)), -1)
    ref_m, ref_v = O.multi_gene_predict(x, y, v, t, D, S, B, 1.8, 0.7, 0.0)
    hyp = _lib.HypArgs(D, S, B, 1.8, 0.7, 1e-4)
    mean = np.empty(mm)
    cov = np.empty((mm, mm))
    ctx = _lib.get_context()
    ctx.check(ctx.lib.lfm_posterior_f64(ctx.handle, _lib.dptr(x), _lib.dptr(y), n, _lib.dptr(v),
                                        0.49, _lib.dptr(t), mm, hyp.ref, _lib.dptr(mean),
                                        _lib.dptr(cov)))
    close(mean, ref_m)
    close(cov, ref_v)
    np.testing.assert_array_equal(cov, cov.T)


def test_posterior_not_pd_nan(lfm):
    from dis_project_amd import _lib

    g = load_golden("grid_n64")
    t = g["x"][:8]
    hyp = _lib.HypArgs(g["D"], g["S"], g["B"], float(g["l"]), 1.0, 1e-4)
    mean = np.empty(8)
    cov = np.empty((8, 8))
    ctx = _lib.get_context()
    rc = ctx.lib.lfm_posterior_f64(ctx.handle, _lib.dptr(g["x"]), _lib.dptr(g["y"]), 64, None,
                                   -50.0, _lib.dptr(t), 8, hyp.ref, _lib.dptr(mean),
                                   _lib.dptr(cov))
    assert rc == _lib.LFM_E_NOT_PD
    assert np.all(np.isnan(mean)) and np.all(np.isnan(cov))
