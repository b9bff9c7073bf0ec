"""Interleaved A/B timing of per-call settings (env variables read by chol_factor_solve on
every call) in one context at N = 16384: rounds of [variant 0, variant 1, ...], so thermal /
power drift over the run hits every variant alike. Usage:
    python scripts/ab.py "LFM_W4_MIN=6144" "LFM_W4_MIN=5120 LFM_W2_MIN=4096" ...
Prints one line per variant: median / min ms per evaluation over the rounds, MLL."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from dis_project_amd import _lib, configs  # noqa: E402

rounds = int(os.environ.get("AB_ROUNDS", "8"))
reps = int(os.environ.get("AB_REPS", "2"))
variants = [dict(kv.split("=", 1) for kv in v.split()) for v in sys.argv[1:]] or [{}]
work = configs.grid_workload("ab", 64, 256, seed_params=2, seed_y=3)
x = np.ascontiguousarray(work.data.X)
y = np.ascontiguousarray(work.data.y.reshape(-1))
ctx = _lib.Context(0)
lib, h = ctx.lib, ctx.handle
dx, dy = _lib.c_void_p(), _lib.c_void_p()
ctx.check(lib.lfm_dev_alloc(h, x.nbytes, _lib.ctypes.byref(dx)))
ctx.check(lib.lfm_dev_alloc(h, y.nbytes, _lib.ctypes.byref(dy)))
ctx.check(lib.lfm_memcpy_h2d(h, dx, x.ctypes.data, x.nbytes))
ctx.check(lib.lfm_memcpy_h2d(h, dy, y.ctypes.data, y.nbytes))
hp = work.model.hyp()
out = np.empty(1)
base = {k: os.environ.get(k) for v in variants for k in v}
ts = [[] for _ in variants]
mll = [None] * len(variants)


def run(v):
    for k in base:
        if k in v:
            os.environ[k] = v[k]
        elif base[k] is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = base[k]
    ctx.check(lib.lfm_mll_f64_dev(h, dx, dy, x.shape[0], hp.ref, 0, _lib.dptr(out)))  # warm
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ctx.check(lib.lfm_mll_f64_dev(h, dx, dy, x.shape[0], hp.ref, 0, _lib.dptr(out)))
        t.append((time.perf_counter() - t0) * 1e3)
    return t


for r in range(rounds):
    for i, v in enumerate(variants):
        ts[i] += run(v)
        mll[i] = float(out[0])
    print(f"round {r}", " ".join(f"{np.median(t[-reps:]):.3f}" for t in ts), flush=True)
for i, v in enumerate(variants):
    print(f"{' '.join(sys.argv[1 + i].split()) if i < len(sys.argv) - 1 else 'default':45s} "
          f"median {np.median(ts[i]):.3f} min {min(ts[i]):.3f} mll {mll[i]!r}", flush=True)
ctx.close()
