"""Interleaved A/B timing of context-creation settings (LFM_SIDE_CUS, LFM_SIDE_STRIDE, ...):
one context per variant, created up front, evaluated in rounds [v0, v1, ...] at N = 16384.
    python scripts/ab_ctx.py "LFM_SIDE_CUS=32" "LFM_SIDE_CUS=16" ..."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from dis_project_amd import _lib, configs  # noqa: E402

rounds = int(os.environ.get("AB_ROUNDS", "6"))
reps = int(os.environ.get("AB_REPS", "2"))
specs = sys.argv[1:] or [""]
work = configs.grid_workload("ab", 64, 256, seed_params=2, seed_y=3)
x = np.ascontiguousarray(work.data.X)
y = np.ascontiguousarray(work.data.y.reshape(-1))
hp = work.model.hyp()
ctxs = []
for spec in specs:
    kv = dict(s.split("=", 1) for s in spec.split())
    old = {k: os.environ.get(k) for k in kv}
    os.environ.update(kv)
    ctx = _lib.Context(0)
    for k, v in old.items():
        if v is None:
            os.environ.pop(k)
        else:
            os.environ[k] = v
    lib, h = ctx.lib, ctx.handle
    dx, dy = _lib.c_void_p(), _lib.c_void_p()
    ctx.check(lib.lfm_dev_alloc(h, x.nbytes, _lib.ctypes.byref(dx)))
    ctx.check(lib.lfm_dev_alloc(h, y.nbytes, _lib.ctypes.byref(dy)))
    ctx.check(lib.lfm_memcpy_h2d(h, dx, x.ctypes.data, x.nbytes))
    ctx.check(lib.lfm_memcpy_h2d(h, dy, y.ctypes.data, y.nbytes))
    ctxs.append((ctx, dx, dy))
out = np.empty(1)
ts = [[] for _ in specs]
mll = [None] * len(specs)
for r in range(rounds):
    for i, (ctx, dx, dy) in enumerate(ctxs):
        lib, h = ctx.lib, ctx.handle
        ctx.check(lib.lfm_mll_f64_dev(h, dx, dy, x.shape[0], hp.ref, 0, _lib.dptr(out)))
        for _ in range(reps):
            t0 = time.perf_counter()
            ctx.check(lib.lfm_mll_f64_dev(h, dx, dy, x.shape[0], hp.ref, 0, _lib.dptr(out)))
            ts[i].append((time.perf_counter() - t0) * 1e3)
        mll[i] = float(out[0])
    print(f"round {r}", " ".join(f"{np.median(t[-reps:]):.3f}" for t in ts), flush=True)
for i, spec in enumerate(specs):
    print(f"{spec or 'default':45s} median {np.median(ts[i]):.3f} min {min(ts[i]):.3f} "
          f"mll {mll[i]!r}", flush=True)
