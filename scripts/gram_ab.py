"""Gram fill variants (env read per call), interleaved: kernel time from the library's event
profile, fp64 at N = 16384 (C2) and fp32 at N = 65536 (C4), lower triangle, device output.
    python scripts/gram_ab.py ["K=V ..." ...]   (no argument: the library as built)
PAD=<elements> is the script's own: the fill's leading dimension becomes N + PAD. ISO=<us>
(also the script's own): each timed fill follows a device sync and a host sleep of that many
microseconds, as bench.py's steps do (fill, 4-byte read-back, Python) instead of back to back.
MEMSET=1 times lfm_memset_dev over the fill's byte count instead (contiguous; wall time).
LFM_GRAM_AB=<mode> selects a store-shape variant in a library built with -DLFM_GRAM_AB.
Round 3 A/B-ed its rows-per-tile / nontemporal / 16-B store variants this way (profiles/
r03_ab_gram_*); those knobs were removed with the variants, so the gram has no per-call knob now."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from dis_project_amd import _lib, configs  # noqa: E402

variants = [dict(kv.split("=", 1) for kv in v.split()) for v in sys.argv[1:]] or [{}]
maxpad = max(int(v.get("PAD", 0)) for v in variants)
ctx = _lib.get_context(0)
lib, h = ctx.lib, ctx.handle
cases = []
for w, esz, fn in ((configs.c2(), 8, lib.lfm_gram_f64_dev), (configs.c4(), 4, lib.lfm_gram_f32_dev)):
    x = np.ascontiguousarray(w.data.X)
    n = x.shape[0]
    dx, dk = _lib.c_void_p(), _lib.c_void_p()
    ctx.check(lib.lfm_dev_alloc(h, x.nbytes, _lib.ctypes.byref(dx)))
    ctx.check(lib.lfm_memcpy_h2d(h, dx, x.ctypes.data, x.nbytes))
    ctx.check(lib.lfm_dev_alloc(h, n * (n + maxpad) * esz, _lib.ctypes.byref(dk)))
    cases.append((w.name, n, esz, fn, dx, dk, w.model.hyp()))
# bit-identity of every variant against the first: sampled rows of each fill (lower part)
ref_rows = {}
for vi, v in enumerate(variants):
    for k in {kk for vv in variants for kk in vv}:
        os.environ.pop(k, None)
    os.environ.update(v)
    if v.get("MEMSET"):
        continue
    for name, n, esz, fn, dx, dk, hp in cases:
        ld = n + int(v.get("PAD", 0))
        ctx.check(lib.lfm_memset_dev(h, dk, 0, n * ld * esz))
        ctx.check(fn(h, dx, n, hp.ref, 0.0, _lib.LFM_UPLO_LOWER, dk, ld))
        rows = list(range(0, n, n // 61)) + [n - 1]
        buf = np.empty(n, dtype=np.float64 if esz == 8 else np.float32)
        got = []
        for r in rows:
            ctx.check(lib.lfm_memcpy_d2h(h, buf.ctypes.data, _lib.c_void_p(dk.value + r * ld * esz),
                                         (r + 1) * esz))
            got.append(buf[: r + 1].copy())
        if vi == 0:
            ref_rows[name] = got
        else:
            same = all(np.array_equal(a.view(np.uint8), b.view(np.uint8))
                       for a, b in zip(got, ref_rows[name]))
            print(f"{sys.argv[1 + vi]:18s} {name:28s} sampled rows bit-identical to variant 0: {same}",
                  flush=True)
for k in {kk for vv in variants for kk in vv}:
    os.environ.pop(k, None)
res = {}
for rnd in range(4):
    for vi, v in enumerate(variants):
        for k in {kk for vv in variants for kk in vv}:
            os.environ.pop(k, None)
        os.environ.update(v)
        for name, n, esz, fn, dx, dk, hp in cases:
            ld = n + int(v.get("PAD", 0))
            if v.get("MEMSET"):
                # the runtime's fill of the same byte count, contiguous (wall time of 5, synced)
                nb = esz * n * (n + 1) // 2
                ctx.check(lib.lfm_memset_dev(h, dk, 0, nb))
                ctx.check(lib.lfm_ctx_synchronize(h))
                t0 = time.perf_counter()
                for _ in range(5):
                    ctx.check(lib.lfm_memset_dev(h, dk, 0, nb))
                ctx.check(lib.lfm_ctx_synchronize(h))
                res.setdefault((vi, name), []).append((time.perf_counter() - t0) / 5 * 1e3)
                continue
            ctx.check(fn(h, dx, n, hp.ref, 0.0, _lib.LFM_UPLO_LOWER, dk, ld))
            ctx.profile(True, classes=["gram_grid"])
            ctx.profile_reset()
            iso = float(v.get("ISO", 0)) * 1e-6
            for _ in range(5):
                if iso:
                    ctx.check(lib.lfm_ctx_synchronize(h))
                    time.sleep(iso)
                ctx.check(fn(h, dx, n, hp.ref, 0.0, _lib.LFM_UPLO_LOWER, dk, ld))
            st = ctx.profile_read()["gram_grid"]
            ctx.profile(False)
            ms = st["total_ms"] / st["launches"]
            res.setdefault((vi, name), []).append(ms)
for (vi, name), t in sorted(res.items()):
    n = [c[1] for c in cases if c[0] == name][0]
    esz = [c[2] for c in cases if c[0] == name][0]
    ms = float(np.median(t))
    print(f"{sys.argv[1 + vi] if len(sys.argv) > 1 else 'default':18s} {name:28s} {ms:.4f} ms "
          f"{esz * n * (n + 1) / 2 / (ms * 1e-3) / 1e9:.0f} GB/s")
