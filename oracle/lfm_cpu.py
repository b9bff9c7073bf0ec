"""ctypes binding of oracle/liblfm_cpu.so — TEST INFRASTRUCTURE ONLY.

The C++ / OpenMP CPU restatement of the reference's MLL path (oracle/lfm_cpu.cpp): the
full-size parity check of the GPU path and bench.py's timed ``cpu_baseline``. Only
``tests/``, ``__graft_entry__`` and ``bench.py``'s ``cpu_baseline`` leg import it; the product
package never does. Build: ``make -C oracle`` (``__graft_entry__.build()`` runs it).
"""

from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_double, c_int, c_int64

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liblfm_cpu.so")
_dp = POINTER(c_double)
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FileNotFoundError(f"{LIB_PATH} missing: run `make -C oracle`")
        lib = ctypes.CDLL(LIB_PATH)
        lib.lfm_cpu_gram.restype = c_int
        lib.lfm_cpu_gram.argtypes = [_dp, c_int64, c_int64, _dp, _dp, c_double, c_double, _dp,
                                     c_int64, c_int]
        lib.lfm_cpu_gram_rows_f32.restype = c_int
        lib.lfm_cpu_gram_rows_f32.argtypes = [_dp, c_int64, c_int64, _dp, _dp, c_double,
                                              c_double, POINTER(c_int64), c_int64,
                                              POINTER(ctypes.c_float), c_int]
        lib.lfm_cpu_potrf.restype = c_int64
        lib.lfm_cpu_potrf.argtypes = [_dp, c_int64, c_int64, c_int]
        lib.lfm_cpu_mll.restype = c_double
        lib.lfm_cpu_mll.argtypes = [_dp, _dp, c_int64, c_int64, _dp, _dp, _dp, c_double, c_double,
                                    c_double, c_int, c_int, _dp, _dp]
        lib.lfm_cpu_mll_grad.restype = c_double
        lib.lfm_cpu_mll_grad.argtypes = [_dp, _dp, c_int64, c_int64, _dp, _dp, _dp, c_double,
                                         c_double, c_double, c_int, _dp]
        lib.lfm_cpu_fit.restype = c_int
        lib.lfm_cpu_fit.argtypes = [_dp, _dp, c_int64, c_int64, _dp, c_int64, c_double, c_double,
                                    c_double, c_double, c_double, c_int64, c_int, c_int, _dp]
        vp = ctypes.c_void_p
        lib.lfm_cpu_mll_batch.restype = c_int
        lib.lfm_cpu_mll_batch.argtypes = [c_int64, vp, vp, vp, vp, _dp, c_int, c_int, c_int64,
                                          _dp]
        lib.lfm_cpu_fit_batch.restype = c_int
        lib.lfm_cpu_fit_batch.argtypes = [c_int64, vp, vp, vp, vp, vp, c_int64, c_double,
                                          c_double, c_double, c_double, c_double, c_int64, c_int,
                                          c_int, c_int, _dp]
        _lib = lib
    return _lib


def _f64(a):
    return np.ascontiguousarray(np.asarray(a, np.float64))


def _p(a):
    return a.ctypes.data_as(_dp)


def mll(x, y, D, S, B, l, obs_stddev, jitter, negative=False, threads=0, work=None):
    """CustomConjMLL(negative).step on the CPU. Returns (value, info) with info = dict(mll,
    logdet, quad, t_gram, t_chol, t_solve, fail, threads). `work`: optional n x n float64
    scratch (reused across calls)."""
    lib = load()
    x, y, D, S, B = (_f64(v) for v in (x, y, D, S, B))
    x = x.reshape(-1, 3)
    n = x.shape[0]
    info = np.zeros(8)
    wp = None
    if work is not None:
        assert work.dtype == np.float64 and work.size >= n * n and work.flags.c_contiguous
        wp = _p(work)
    v = lib.lfm_cpu_mll(_p(x), _p(y.reshape(-1)), n, D.size, _p(D), _p(S), _p(B), float(l),
                        float(obs_stddev), float(jitter), int(bool(negative)), int(threads), wp,
                        _p(info))
    keys = ["mll", "logdet", "quad", "t_gram", "t_chol", "t_solve", "fail", "threads"]
    return float(v), dict(zip(keys, info.tolist()))


def gram_lower(x, D, S, l, diag_add=0.0, threads=0):
    """Lower triangle of K(x, x) + diag_add I (upper part zero)."""
    lib = load()
    x, D, S = (_f64(v) for v in (x, D, S))
    x = x.reshape(-1, 3)
    n = x.shape[0]
    K = np.zeros((n, n))
    rc = lib.lfm_cpu_gram(_p(x), n, D.size, _p(D), _p(S), float(l), float(diag_add), _p(K), n,
                          int(threads))
    if rc:
        raise ValueError("lfm_cpu_gram: bad arguments")
    return K


def gram_rows_f32(x, D, S, l, rows, diag_add=0.0, threads=0):
    """Rows `rows` of the lower triangle of K(x, x) + diag_add I in fp64 arithmetic, stored as
    float32 [len(rows), n] (entries above the diagonal zero)."""
    lib = load()
    x, D, S = (_f64(v) for v in (x, D, S))
    x = x.reshape(-1, 3)
    n = x.shape[0]
    rows = np.ascontiguousarray(np.asarray(rows, np.int64))
    out = np.zeros((rows.size, n), np.float32)
    rc = lib.lfm_cpu_gram_rows_f32(_p(x), n, D.size, _p(D), _p(S), float(l), float(diag_add),
                                   rows.ctypes.data_as(POINTER(c_int64)), rows.size,
                                   out.ctypes.data_as(POINTER(ctypes.c_float)), int(threads))
    if rc:
        raise ValueError("lfm_cpu_gram_rows_f32: bad arguments")
    return out


def potrf(A, threads=0):
    """In-place lower Cholesky of a C-contiguous float64 square array; returns the failing
    pivot or -1."""
    lib = load()
    assert A.dtype == np.float64 and A.flags.c_contiguous and A.shape[0] == A.shape[1]
    return int(lib.lfm_cpu_potrf(_p(A), A.shape[0], A.shape[0], int(threads)))


def mll_grad(x, y, D, S, B, l, obs_stddev, jitter, negative=False):
    """Value and gradient (constrained parameters) of CustomConjMLL(negative).step on one core:
    (value, grad[3G + 2] = dD dS dB, dl, d obs_stddev)."""
    lib = load()
    x, y, D, S, B = (_f64(v) for v in (x, y, D, S, B))
    x = x.reshape(-1, 3)
    g = np.empty(3 * D.size + 2)
    v = lib.lfm_cpu_mll_grad(_p(x), _p(y.reshape(-1)), x.shape[0], D.size, _p(D), _p(S), _p(B),
                             float(l), float(obs_stddev), float(jitter), int(bool(negative)), _p(g))
    return float(v), g


def fit(x, y, G, raw, iters, lr=0.01, b1=0.9, b2=0.999, eps=1e-8, eps_root=0.0, spe=1000,
        fix=False, negative=True):
    """JaxTrainer.fit of one problem on one core: raw [3G + 3] (d s b, l, obs_stddev, jitter;
    unconstrained, the jitter static) is updated in place. Returns (history[iters], failures)."""
    lib = load()
    x, y = _f64(x).reshape(-1, 3), _f64(y).reshape(-1)
    assert raw.dtype == np.float64 and raw.flags.c_contiguous and raw.size == 3 * G + 3
    hist = np.empty(int(iters))
    bad = lib.lfm_cpu_fit(_p(x), _p(y), x.shape[0], int(G), _p(raw), int(iters), lr, b1, b2, eps,
                          eps_root, int(spe), int(bool(fix)), int(bool(negative)), _p(hist))
    return hist, int(bad)

def _ptrs(arrs):
    return (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])


def mll_batch(xs, ys, genes, hyp, negative=False, threads=0, reps=1):
    """Every problem's CustomConjMLL(negative).step, one problem per OpenMP thread at a time
    (threads = 0: all allowed); hyp in lfm_batch_mll_f64's packed layout; reps > 1 evaluates
    the P problems reps times over in the same parallel loop (a timing sample). Returns [P]."""
    lib = load()
    xs = [_f64(x).reshape(-1, 3) for x in xs]
    ys = [_f64(y).reshape(-1) for y in ys]
    ns = np.array([x.shape[0] for x in xs], np.int64)
    gs = np.array(genes, np.int64)
    hyp = _f64(hyp)
    out = np.empty(len(xs))
    rc = lib.lfm_cpu_mll_batch(len(xs), _ptrs(xs), _ptrs(ys), ns.ctypes.data, gs.ctypes.data,
                               _p(hyp), int(bool(negative)), int(threads), int(reps), _p(out))
    if rc:
        raise ValueError("lfm_cpu_mll_batch: bad arguments")
    return out


def fit_batch(xs, ys, genes, raws, iters, lr=0.01, b1=0.9, b2=0.999, eps=1e-8, eps_root=0.0,
              spe=1000, fix=False, negative=True, threads=0):
    """fit() of every problem, one problem per OpenMP thread at a time; raws: per problem a
    [3G + 3] float64 array, updated in place. Returns (history [P, iters], failures)."""
    lib = load()
    xs = [_f64(x).reshape(-1, 3) for x in xs]
    ys = [_f64(y).reshape(-1) for y in ys]
    ns = np.array([x.shape[0] for x in xs], np.int64)
    gs = np.array(genes, np.int64)
    for r, g in zip(raws, genes):
        assert r.dtype == np.float64 and r.flags.c_contiguous and r.size == 3 * g + 3
    hist = np.empty((len(xs), int(iters)))
    bad = lib.lfm_cpu_fit_batch(len(xs), _ptrs(xs), _ptrs(ys), ns.ctypes.data, gs.ctypes.data,
                                _ptrs(raws), int(iters), lr, b1, b2, eps, eps_root, int(spe),
                                int(bool(fix)), int(bool(negative)), int(threads), _p(hist))
    return hist, int(bad)
