"""CPU oracle for the SIM latent-force-model MLL hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module, and only as the checker / the timed CPU baseline. The
product path (``dis_project_amd``) never imports it and has no CPU fallback.

What it restates (wejpurvis/DIS_project @ 2024-08-07):
  * ``h``           src/model.py:315-365
  * ``gamma``       src/model.py:367-369
  * ``kernel_xx``   src/model.py:197-235
  * ``kernel_xf``   src/model.py:237-282
  * ``kernel_ff``   src/model.py:284-312 (divides by 2*l, kept)
  * ``kernel``      src/model.py:152-195 (flag switches: all four branches are
                    evaluated and multiplied by their integer switch, as the
                    reference does under vmap)
  * ``cross_covariance`` / ``gram``  src/model.py:372-414
  * ``mean_function``                src/model.py:124-149 (block position, not x[:,1])
  * ``mll``         src/objectives.py:21-78 -> gpjax 0.8.2 GaussianDistribution.log_prob:
                    -1/2 (n log 2pi + logdet S + r^T S^{-1} r), logdet and solve through
                    a Cholesky factor (cola Cholesky -> LAPACK potrf); a failed
                    factorisation yields NaN (JAX semantics).
  * ``dataset_3d``  src/dataset.py:358-399 (row layout of x / y)

PARITY STATUS: **parity unpinned** by the reference itself. The reference is pure
JAX/GPJax (jax 0.4.28, gpjax 0.8.2, cola-ml 0.0.5 pinned in environment.yml); none
of them is installed in this image (ModuleNotFoundError, not a permission denial)
and the reference ships no tests, fixtures or golden vectors.
This restatement is instead pinned by:
  * known-answer tests derived from the reference formulas (t = 0 rows vanish;
    all-zero times give a diagonal Sigma with a closed-form log-density; exact
    symmetry of kxx);
  * 50-digit mpmath evaluation of ``h`` (``h_mpmath``);
  * a scalar pure-Python restatement (``kernel_scalar``) that shares no code with
    the vectorised one;
  * an independent cross-read of the GPyTorch twin's ``h``
    (src/gpytorch_alfi/model_alfi.py:343-378), which agrees term by term.
"""

from __future__ import annotations

import math

import numpy as np
import scipy.linalg
import scipy.special

SQRT_PI = math.sqrt(math.pi)
LOG_2PI = math.log(2.0 * math.pi)


# ------------------------------------------------------------------ indices
def gene_index(g, G):
    """int(x[1]) with JAX gather semantics: truncate, wrap negatives, clamp."""
    g = np.trunc(np.asarray(g, dtype=np.float64))
    g = np.where(g < 0, g + G, g)
    g = np.where(np.isnan(g), 0, g)
    return np.clip(g, 0, G - 1).astype(np.int64)


def flag_int(f):
    f = np.trunc(np.asarray(f, dtype=np.float64))
    return np.where(np.isnan(f), 0, f).astype(np.int64)


# --------------------------------------------------------------- kernel math
def gamma(D, l, k):
    """model.py:367-369."""
    return (D[k] * l) / 2


def h(D, l, j, k, t1, t2):
    """model.py:315-365, vectorised over broadcastable j, k, t1, t2."""
    t_dist = t2 - t1
    gk = gamma(D, l, k)
    multiplier = np.exp(gk**2) / (D[j] + D[k])
    first_multiplier = np.exp(-D[k] * t_dist)
    first_erf_terms = scipy.special.erf((t_dist / l) - gk) + scipy.special.erf(t1 / l + gk)
    second_multiplier = np.exp(-(D[k] * t2 + D[j] * t1))
    second_erf_terms = scipy.special.erf((t2 / l) - gk) + scipy.special.erf(gk)
    return multiplier * (first_multiplier * first_erf_terms - second_multiplier * second_erf_terms)


def kernel_xx(D, S, l, ta, ja, tb, jb):
    """model.py:197-235; ja / jb are clamped integer gene indices."""
    mult = S[ja] * S[jb] * l * SQRT_PI * 0.5
    return mult * (h(D, l, jb, ja, tb, ta) + h(D, l, ja, jb, ta, tb))


def kernel_xf(D, S, l, ta, ga, fa, tb, gb):
    """model.py:237-282: the row whose flag (as float) is 0 is the latent row."""
    a_lat = fa == 0
    t_gene = np.where(a_lat, tb, ta)
    g_gene = np.where(a_lat, gb, ga)
    t_lat = np.where(a_lat, ta, tb)
    j = gene_index(g_gene, D.shape[0])
    t_dist = t_gene - t_lat
    gj = gamma(D, l, j)
    first_term = 0.5 * l * SQRT_PI * S[j]
    first_expon_term = np.exp(gj**2)
    second_expon_term = np.exp(-D[j] * t_dist)
    erf_terms = scipy.special.erf((t_dist / l) - gj) + scipy.special.erf(t_lat / l + gj)
    return first_term * first_expon_term * second_expon_term * erf_terms


def kernel_ff(l, ta, tb):
    """model.py:284-312."""
    sq_dist = np.square(ta - tb)
    sq_dist = sq_dist / (2 * l)
    return np.exp(-sq_dist)


def kernel_pairs(xa, xb, D, S, l):
    """model.py:152-195 over broadcast rows xa[..., 3], xb[..., 3]."""
    G = D.shape[0]
    ta, ga, fa = xa[..., 0], xa[..., 1], xa[..., 2]
    tb, gb, fb = xb[..., 0], xb[..., 1], xb[..., 2]
    f1, f2 = flag_int(fa), flag_int(fb)
    kxx_switch = f1 * f2
    kff_switch = (1 - f1) * (1 - f2)
    kxf_switch = f1 * (1 - f2)
    kxf_t_switch = (1 - f1) * f2
    with np.errstate(over="ignore", invalid="ignore"):
        return (
            kxx_switch * kernel_xx(D, S, l, ta, gene_index(ga, G), tb, gene_index(gb, G))
            + kff_switch * kernel_ff(l, ta, tb)
            + kxf_switch * kernel_xf(D, S, l, ta, ga, fa, tb, gb)
            + kxf_t_switch * kernel_xf(D, S, l, tb, gb, fb, ta, ga)
        )


def cross_covariance(x, y, D, S, l, chunk=256):
    """model.py:372-394 (vmap over rows of x, then rows of y), row-chunked."""
    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64)
    # complex D / S / l propagate (complex-step derivatives in mll_grad)
    dt = np.result_type(np.asarray(D).dtype, np.asarray(S).dtype, np.asarray(l).dtype, np.float64)
    out = np.empty((x.shape[0], y.shape[0]), dtype=dt)
    for i0 in range(0, x.shape[0], chunk):
        xa = x[i0:i0 + chunk, None, :]
        out[i0:i0 + chunk] = kernel_pairs(xa, y[None, :, :], D, S, l)
    return out


def gram_error_scale(x, y, D, S, l, chunk=256):
    """Per-element magnitude M of the intermediate terms of kernel() in the reference's
    evaluation order: for gene/gene pairs S_j S_k l sqrt(pi)/2 times, for each h,
    multiplier * (first_multiplier (|erf a| + |erf b|) + second_multiplier (|erf c| + |erf d|)).
    An fp64 evaluation of the reference formula is accurate to ~eps * M, not eps * |K|
    (the erf sums cancel and are then scaled by e^{gamma^2 - D delta}); tests compare two
    evaluations with an absolute tolerance proportional to M."""
    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64)
    G = D.shape[0]
    erf = scipy.special.erf

    def habs(j, k, t1, t2):
        td = t2 - t1
        gk = gamma(D, l, k)
        mult = np.exp(gk**2) / (D[j] + D[k])
        a = np.exp(-D[k] * td) * (np.abs(erf(td / l - gk)) + np.abs(erf(t1 / l + gk)))
        b = np.exp(-(D[k] * t2 + D[j] * t1)) * (np.abs(erf(t2 / l - gk)) + np.abs(erf(gk)))
        return mult * (a + b)

    out = np.empty((x.shape[0], y.shape[0]))
    for i0 in range(0, x.shape[0], chunk):
        xa = x[i0:i0 + chunk, None, :]
        yb = y[None, :, :]
        ta, tb = xa[..., 0], yb[..., 0]
        ja, jb = gene_index(xa[..., 1], G), gene_index(yb[..., 1], G)
        with np.errstate(over="ignore", invalid="ignore"):
            mxx = (S[ja] * S[jb] * l * SQRT_PI * 0.5) * (habs(jb, ja, tb, ta) + habs(ja, jb, ta, tb))
            kv = np.abs(kernel_pairs(xa, yb, D, S, l))
        both = (flag_int(xa[..., 2]) * flag_int(yb[..., 2])) != 0
        out[i0:i0 + chunk] = np.where(both, np.maximum(mxx, kv), kv + 1.0)
    return out


def gram(x, D, S, l):
    """model.py:396-414 (the dense matrix behind cola.PSD(Dense(.)))."""
    return cross_covariance(x, x, D, S, l)


def mean_function(x, D, B, num_genes):
    """model.py:124-149: block position i // (N // G), times int(flag)."""
    x = np.asarray(x, np.float64)
    f = flag_int(x[:, 2:])
    block_size = x.shape[0] // num_genes
    mean = (B / D).reshape(-1, 1)
    mean = np.repeat(mean, block_size, axis=0).reshape(-1, 1)
    return mean * f


# ----------------------------------------------------------------------- MLL
def log_prob(loc, Sigma, y):
    """gpjax 0.8.2 GaussianDistribution.log_prob with a Cholesky-backed PSD scale."""
    n = loc.shape[-1]
    diff = y - loc
    try:
        c = scipy.linalg.cho_factor(Sigma, lower=True, check_finite=False)
    except (np.linalg.LinAlgError, scipy.linalg.LinAlgError):
        return float("nan")
    L = np.tril(c[0])
    d = np.diag(L)
    if not np.all(np.isfinite(d)) or np.any(d <= 0):
        return float("nan")
    logdet = 2.0 * np.sum(np.log(d))
    quad = diff @ scipy.linalg.cho_solve(c, diff, check_finite=False)
    return float(-0.5 * (n * LOG_2PI + logdet + quad))


def sigma(x, D, S, l, obs_stddev, jitter):
    """objectives.py:66-73: Sigma = (K + jitter I) + obs_stddev^2 I."""
    n = x.shape[0]
    K = gram(x, D, S, l)
    K = K + np.eye(n) * jitter
    return K + np.eye(n) * (obs_stddev**2)


def mll(x, y, D, S, B, l, obs_stddev, jitter, negative=False):
    """CustomConjMLL(negative).step (objectives.py:21-78)."""
    D = np.asarray(D, np.float64)
    S = np.asarray(S, np.float64)
    B = np.asarray(B, np.float64)
    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64).reshape(-1)
    mx = mean_function(x, D, B, D.shape[0]).reshape(-1)
    Sig = sigma(x, D, S, l, obs_stddev, jitter)
    constant = -1.0 if negative else 1.0
    return constant * log_prob(mx, Sig, y)


def mll_grad(x, y, D, S, B, l, obs_stddev, jitter, negative=False, step=1e-30):
    """Value and gradient of CustomConjMLL(negative).step with respect to the constrained
    parameters (true_d, true_s, true_b, l, obs_stddev): the quantity
    jax.value_and_grad(loss) differentiates before the bijectors' chain rule
    (trainer.py:103, 126; jitter is a static field, model.py:64).

        d log N / d theta = 1/2 tr((a a^T - Sigma^{-1}) dSigma/dtheta) + a^T dm/dtheta,
        a = Sigma^{-1} (y - m),  dSigma/d obs_stddev = 2 obs_stddev I.

    dK/dtheta of the reference kernel (model.py:152-369) is taken by complex step
    (imag K(theta + i h) / h, exact to rounding: every operation of the kernel is analytic
    and scipy's erf accepts complex arguments); dm/dtheta of mean_function
    (model.py:124-149, block position i // (n // G)) is analytic.

    Returns a dict: value, d, s, b (arrays [G]), l, obs_stddev, and the magnitudes
    scale_{d,s,b,l,obs_stddev} of the summed terms (1/2 sum |W| |dSigma| + |a| |dm|) that
    the tests scale their tolerance by.
    """
    D = np.asarray(D, np.float64)
    S = np.asarray(S, np.float64)
    B = np.asarray(B, np.float64)
    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64).reshape(-1)
    n, G = x.shape[0], D.shape[0]
    sign = -1.0 if negative else 1.0
    nanres = dict(value=float("nan"), d=np.full(G, np.nan), s=np.full(G, np.nan),
                  b=np.full(G, np.nan), l=float("nan"), obs_stddev=float("nan"))
    mx = mean_function(x, D, B, G).reshape(-1)
    Sig = sigma(x, D, S, l, obs_stddev, jitter)
    try:
        c = scipy.linalg.cho_factor(Sig, lower=True, check_finite=False)
    except (np.linalg.LinAlgError, scipy.linalg.LinAlgError):
        return nanres
    dg = np.diag(np.tril(c[0]))
    if not np.all(np.isfinite(dg)) or np.any(dg <= 0):
        return nanres
    r = y - mx
    a = scipy.linalg.cho_solve(c, r, check_finite=False)
    Sinv = scipy.linalg.cho_solve(c, np.eye(n), check_finite=False)
    W = np.outer(a, a) - Sinv
    value = -0.5 * (n * LOG_2PI + 2.0 * np.sum(np.log(dg)) + r @ a)

    def dgram(Dc, Sc, lc):
        return np.imag(gram(x, Dc, Sc, lc)) / step

    def contract(dK):
        return 0.5 * np.sum(W * dK), 0.5 * np.sum(np.abs(W) * np.abs(dK))

    out = dict(value=sign * value)
    gd, gs, sd_, ss_ = np.zeros(G), np.zeros(G), np.zeros(G), np.zeros(G)
    for g in range(G):
        e = np.zeros(G, complex)
        e[g] = 1j * step
        gd[g], sd_[g] = contract(dgram(D + e, S, l))
        gs[g], ss_[g] = contract(dgram(D, S + e, l))
    gl, sl = contract(dgram(D, S, l + 1j * step))
    # mean: m_i = (B/D)[i // bs] * flag_i
    bs = n // G
    f = flag_int(x[:, 2])
    af = np.bincount(np.arange(n) // bs, weights=a * f, minlength=G)[:G]
    aabs = np.bincount(np.arange(n) // bs, weights=np.abs(a * f), minlength=G)[:G]
    gb = af / D
    gd_mean = -B / D**2 * af
    out["d"] = sign * (gd + gd_mean)
    out["s"] = sign * gs
    out["b"] = sign * gb
    out["l"] = sign * gl
    out["obs_stddev"] = sign * obs_stddev * np.trace(W)
    out["scale_d"] = sd_ + np.abs(B / D**2) * aabs
    out["scale_s"] = ss_
    out["scale_b"] = aabs / np.abs(D)
    out["scale_l"] = sl
    out["scale_obs_stddev"] = abs(obs_stddev) * np.sum(np.abs(np.diag(W)))
    return out


# ------------------------------------------------------------- Barenco loader
def barenco_transform(log_expr, se):
    """dataset.py:268-313 element by element: rows DDB2, BIK, DR5, p21, SESN1, p53; columns
    replicate-major (r, t). Returns gene_expressions / gene_variances [3, 5, 7] and
    p53_expressions / p53_variances [3, 1, 7]."""
    log_expr = np.asarray(log_expr, np.float64)
    var = np.asarray(se, np.float64) ** 2
    out_e = np.empty((3, 6, 7))
    out_v = np.empty((3, 6, 7))
    for g in range(6):
        full = [math.exp(log_expr[g, c] + var[g, c] / 2) for c in range(21)]
        vfull = [(math.exp(var[g, c]) - 1) * math.exp(2 * log_expr[g, c] + var[g, c])
                 for c in range(21)]
        first = full[:7]
        mean = sum(first) / 7
        scale = math.sqrt(sum((f - mean) ** 2 for f in first) / 6)  # ddof = 1, replicate 1
        for r in range(3):
            for t in range(7):
                out_e[r, g, t] = full[7 * r + t] / scale
                out_v[r, g, t] = vfull[7 * r + t] / scale**2
    return {"gene_expressions": out_e[:, :5], "gene_variances": out_v[:, :5],
            "p53_expressions": out_e[:, 5:], "p53_variances": out_v[:, 5:]}


# ---------------------------------------------------------------- predictors
def latent_predict(x, y, variances, t, D, S, B, l, jitter):
    """model.py:420-465 (cola.inv -> an explicit inverse here too).
    Returns (mean [m], var [m, m] diagonal)."""
    D, S, B = (np.asarray(v, np.float64) for v in (D, S, B))
    y = np.asarray(y, np.float64).reshape(-1, 1)
    G = D.shape[0]
    mean_x = mean_function(x, D, B, G)
    mean_t = mean_function(t, D, B, G)
    Kxx = gram(x, D, S, l) + np.diag(np.asarray(variances, np.float64).reshape(-1))
    Kxx = Kxx + np.eye(Kxx.shape[0]) * jitter
    K_inv = np.linalg.inv(Kxx)
    Kxf = cross_covariance(x, t, D, S, l)
    KfxKxx = Kxf.T @ K_inv
    mean = mean_t + KfxKxx @ (y - mean_x)
    Kff = gram(t, D, S, l) + np.eye(t.shape[0]) * jitter
    var = Kff - KfxKxx @ Kxf
    var = np.diag(np.diag(var)) + np.eye(t.shape[0]) * jitter
    return np.atleast_1d(mean.squeeze()), var


def multi_gene_predict(x, y, variances, t, D, S, B, l, obs_stddev, jitter):
    """model.py:467-514 (cola.solve on a PSD operator -> Cholesky solve).
    Returns (mean [m], var [m, m])."""
    D, S, B = (np.asarray(v, np.float64) for v in (D, S, B))
    y = np.asarray(y, np.float64).reshape(-1, 1)
    G = D.shape[0]
    mean_x = mean_function(x, D, B, G)
    Kxx = gram(x, D, S, l)
    Sigma = Kxx + np.diag(np.asarray(variances, np.float64).reshape(-1))
    Sigma = Sigma + np.eye(Sigma.shape[0]) * obs_stddev**2
    mean_t = mean_function(t, D, B, G)
    Ktt = gram(t, D, S, l)
    Kxt = cross_covariance(x, t, D, S, l)
    c = scipy.linalg.cho_factor(Sigma, lower=True)
    Sigma_inv_Kxt = scipy.linalg.cho_solve(c, Kxt)
    mean = mean_t + Sigma_inv_Kxt.T @ (y - mean_x)
    var = Ktt - Kxt.T @ Sigma_inv_Kxt + np.eye(t.shape[0]) * jitter
    return np.atleast_1d(mean.squeeze()), var


# -------------------------------------------------- scalar restatement (math)
def h_scalar(D, l, j, k, t1, t2):
    t_dist = t2 - t1
    gk = D[k] * l / 2
    mult = math.exp(gk * gk) / (D[j] + D[k])
    a = math.exp(-D[k] * t_dist) * (math.erf(t_dist / l - gk) + math.erf(t1 / l + gk))
    b = math.exp(-(D[k] * t2 + D[j] * t1)) * (math.erf(t2 / l - gk) + math.erf(gk))
    return mult * (a - b)


def kernel_scalar(xa, xb, D, S, l):
    """Pure-Python loop restatement of model.py:152-312 for one pair of rows."""
    G = len(D)

    def gi(g):
        g = math.trunc(g)
        if g < 0:
            g += G
        return int(min(max(g, 0), G - 1))

    f1, f2 = math.trunc(xa[2]), math.trunc(xb[2])
    val = 0.0
    if f1 * f2:
        j, k = gi(xa[1]), gi(xb[1])
        mult = S[j] * S[k] * l * SQRT_PI * 0.5
        val += f1 * f2 * mult * (h_scalar(D, l, k, j, xb[0], xa[0]) + h_scalar(D, l, j, k, xa[0], xb[0]))
    if (1 - f1) * (1 - f2):
        val += (1 - f1) * (1 - f2) * math.exp(-((xa[0] - xb[0]) ** 2) / (2 * l))
    for sw, ra, rb in ((f1 * (1 - f2), xa, xb), ((1 - f1) * f2, xb, xa)):
        if sw:
            gene, lat = (rb, ra) if ra[2] == 0 else (ra, rb)
            j = gi(gene[1])
            td = gene[0] - lat[0]
            gj = D[j] * l / 2
            val += sw * (0.5 * l * SQRT_PI * S[j] * math.exp(gj * gj) * math.exp(-D[j] * td)
                         * (math.erf(td / l - gj) + math.erf(lat[0] / l + gj)))
    return val


def h_mpmath(D, l, j, k, t1, t2, dps=50):
    """50-digit evaluation of model.py:315-365 (pins the fp64 restatements)."""
    import mpmath

    with mpmath.workdps(dps):
        Dj, Dk, L = mpmath.mpf(D[j]), mpmath.mpf(D[k]), mpmath.mpf(l)
        T1, T2 = mpmath.mpf(t1), mpmath.mpf(t2)
        gk = Dk * L / 2
        td = T2 - T1
        mult = mpmath.exp(gk**2) / (Dj + Dk)
        a = mpmath.exp(-Dk * td) * (mpmath.erf(td / L - gk) + mpmath.erf(T1 / L + gk))
        b = mpmath.exp(-(Dk * T2 + Dj * T1)) * (mpmath.erf(T2 / L - gk) + mpmath.erf(gk))
        return float(mult * (a - b))


# --------------------------------------------------------------- data layout
def dataset_3d(gene_expressions, timepoints):
    """src/dataset.py:358-399 for expressions shaped (R, G, T): rows r*G*T + g*T + tau."""
    R, G, T = gene_expressions.shape
    time_points_repeated = np.tile(np.asarray(timepoints, np.float64), R * G)
    gene_indices = np.tile(np.repeat(np.arange(G), T), R)
    ones = np.ones(G * T * R, dtype=np.int64)
    x = np.stack((time_points_repeated, gene_indices, ones), axis=-1).astype(np.float64)
    y = np.asarray(gene_expressions, np.float64).reshape(-1, 1)
    return x, y
