"""C3 random restarts on ONE GPU: sequential evaluations in one context vs two contexts in two
host threads evaluating concurrently (each context's factor chain on its own 32 CUs, both bulk
streams on the remaining 192), so one evaluation's chain-bound tail overlaps the other's bulk.

    GPU_MAX_HW_QUEUES=8 python scripts/c3_pipe.py [count]

Prints evals/s for both modes and checks that both return the same MLL values."""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from dis_project_amd import _lib, configs  # noqa: E402

count = int(sys.argv[1]) if len(sys.argv) > 1 else 16
base = configs.c2()
restarts = configs.c3_restarts(base, count)
x = np.ascontiguousarray(base.data.X)
y = np.ascontiguousarray(base.data.y.reshape(-1))
n = x.shape[0]


def make(env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        ctx = _lib.Context(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v
    lib, h = ctx.lib, ctx.handle
    dx, dy, data = _lib.c_void_p(), _lib.c_void_p(), _lib.c_void_p()
    ctx.check(lib.lfm_dev_alloc(h, x.nbytes, _lib.ctypes.byref(dx)))
    ctx.check(lib.lfm_dev_alloc(h, y.nbytes, _lib.ctypes.byref(dy)))
    ctx.check(lib.lfm_memcpy_h2d(h, dx, x.ctypes.data, x.nbytes))
    ctx.check(lib.lfm_memcpy_h2d(h, dy, y.ctypes.data, y.nbytes))
    ctx.check(lib.lfm_data_create(h, dx, dy, n, _lib.ctypes.byref(data)))
    return ctx, data


def run(ctx, data, idx, out):
    o = np.empty(1)
    for i in idx:
        hp = restarts[i].hyp()
        ctx.check(ctx.lib.lfm_mll_f64_data(ctx.handle, data, hp.ref, 0, _lib.dptr(o)),
                  allow_not_pd=True)
        out[i] = o[0]


single = make({})
pair = [make({"LFM_SIDE_FIRST": "0", "LFM_MAIN_SKIP": "64"}),
        make({"LFM_SIDE_FIRST": "32", "LFM_MAIN_SKIP": "64"})]
print("contexts:", flush=True)
res = {}
for rnd in range(3):
    out1 = np.empty(count)
    run(*single, [0, 1], out1)  # warm
    t0 = time.perf_counter()
    run(*single, range(count), out1)
    t1 = time.perf_counter() - t0
    out2 = np.empty(count)
    run(*pair[0], [0], out2)
    run(*pair[1], [1], out2)
    t0 = time.perf_counter()
    th = [threading.Thread(target=run, args=(*pair[k], range(k, count, 2), out2)) for k in (0, 1)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    t2 = time.perf_counter() - t0
    same = np.allclose(out1, out2, rtol=1e-12, equal_nan=True)
    print(f"round {rnd}: sequential {count / t1:.2f} evals/s ({t1 / count * 1e3:.2f} ms/eval), "
          f"two contexts {count / t2:.2f} evals/s ({t2 / count * 1e3:.2f} ms/eval), same={same}",
          flush=True)
