"""One process, one GPU: RCCL farm communicator (1 rank) + schedule-3 MLL evaluations at
N = 16384 in the same context, as every rank of `bench.py --gpus N` runs them. Checks that the
streams RCCL creates do not stall the CU-partitioned stream pair (prints ms per evaluation)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from dis_project_amd import _lib, configs  # noqa: E402

work = configs.grid_workload("farm_s3", 64, 256, seed_params=2, seed_y=3)
x = np.ascontiguousarray(work.data.X)
y = np.ascontiguousarray(work.data.y.reshape(-1))
ctx = _lib.Context(0)
lib, h = ctx.lib, ctx.handle
if os.environ.get("FARM", "1") == "1":
    uid = (_lib.ctypes.c_ubyte * 128)()
    ctx.check(lib.lfm_farm_unique_id(h, uid))
    ctx.check(lib.lfm_farm_init(h, uid, 1, 0))
    print("farm initialised", flush=True)
dx, dy = _lib.c_void_p(), _lib.c_void_p()
ctx.check(lib.lfm_dev_alloc(h, x.nbytes, _lib.ctypes.byref(dx)))
ctx.check(lib.lfm_dev_alloc(h, y.nbytes, _lib.ctypes.byref(dy)))
ctx.check(lib.lfm_memcpy_h2d(h, dx, x.ctypes.data, x.nbytes))
ctx.check(lib.lfm_memcpy_h2d(h, dy, y.ctypes.data, y.nbytes))
hp = work.model.hyp()
out = np.empty(1)
got = np.empty(1)
for it in range(4):
    t0 = time.perf_counter()
    ctx.check(lib.lfm_mll_f64_dev(h, dx, dy, x.shape[0], hp.ref, 0, _lib.dptr(out)))
    ms = (time.perf_counter() - t0) * 1e3
    if os.environ.get("FARM", "1") == "1":
        ctx.check(lib.lfm_farm_allgather_f64(h, _lib.dptr(out), 1, _lib.dptr(got)))
    print(f"eval {it}: {ms:.2f} ms mll {out[0]!r}", flush=True)
if os.environ.get("FARM", "1") == "1":
    lib.lfm_farm_destroy(h)
ctx.close()
print("ok", flush=True)
