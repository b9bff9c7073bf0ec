"""Phase timings of the schedule-3 factor chain at N = 16384 (device s_memrealtime stamps).
Per super-panel step: P0 (pending update + identity), grid sync, and per block column c the
diagonal factor, its inverse and the panel-solve sync (us)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from dis_project_amd import _lib, configs  # noqa: E402

work = configs.grid_workload("stamps", 64, 256, seed_params=2, seed_y=3)
x = np.ascontiguousarray(work.data.X)
y = np.ascontiguousarray(work.data.y.reshape(-1))
ctx = _lib.Context(0)
lib, h = ctx.lib, ctx.handle
dx, dy = _lib.c_void_p(), _lib.c_void_p()
ctx.check(lib.lfm_dev_alloc(h, x.nbytes, ctypes.byref(dx)))
ctx.check(lib.lfm_dev_alloc(h, y.nbytes, ctypes.byref(dy)))
ctx.check(lib.lfm_memcpy_h2d(h, dx, x.ctypes.data, x.nbytes))
ctx.check(lib.lfm_memcpy_h2d(h, dy, y.ctypes.data, y.nbytes))
out = np.empty(1)
hp = work.model.hyp()
for _ in range(3):
    ctx.check(lib.lfm_mll_f64_dev(h, dx, dy, x.shape[0], hp.ref, 0, _lib.dptr(out)))
ctx.check(ctx.diag.lfm_debug_stamps(h, 1, None, 0))
ctx.check(lib.lfm_mll_f64_dev(h, dx, dy, x.shape[0], hp.ref, 0, _lib.dptr(out)))
buf = (ctypes.c_ulonglong * (256 * 24))()
ctx.check(ctx.diag.lfm_debug_stamps(h, 0, buf, 256 * 24))
st = np.frombuffer(buf, dtype=np.uint64)[:256 * 16].reshape(256, 16).astype(np.int64)
for s in range(256):
    row = st[s]
    if row[0] == 0:
        break
    t = {p: (row[p] - row[0]) * 0.01 for p in range(16) if row[p]}
    print(s, " ".join(f"{p}:{v:.1f}" for p, v in t.items()))
done = [st[s][15] for s in range(256) if st[s][0]]
per = np.diff(np.array(done, dtype=np.int64)) * 0.01
print("period (us) between chain completions:", " ".join(f"{v:.0f}" for v in per))
