"""Time one N=16384 MLL evaluation under look-ahead settings (env read at context creation).
Prints one JSON line per setting: median / min ms per evaluation and the MLL value."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from dis_project_amd import _lib, configs  # noqa: E402

G = int(os.environ.get("SWEEP_G", "64"))
T = int(os.environ.get("SWEEP_T", "256"))
work = configs.grid_workload("sweep", G, T, seed_params=2, seed_y=3)
x = np.ascontiguousarray(work.data.X)
y = np.ascontiguousarray(work.data.y.reshape(-1))
# setting = lookahead,side_cus[,w4_min,w2_min[,w8_min[,serial_below]]]
settings = [("1", "0"), ("0", "0"), ("1", "8"), ("1", "16"), ("1", "32")]
if len(sys.argv) > 1:
    settings = [tuple(s.split(",")) for s in sys.argv[1:]]
for st in settings:
    la, cus = st[0], st[1]
    os.environ["LFM_LOOKAHEAD"], os.environ["LFM_SIDE_CUS"] = la, cus
    if len(st) > 2:
        os.environ["LFM_W4_MIN"], os.environ["LFM_W2_MIN"] = st[2], st[3]
    os.environ["LFM_W8_MIN"] = st[4] if len(st) > 4 else "1073741824"
    os.environ["LFM_SERIAL_BELOW"] = st[5] if len(st) > 5 else "0"
    ctx = _lib.Context(0)
    lib, h = ctx.lib, ctx.handle
    dx, dy = _lib.c_void_p(), _lib.c_void_p()
    ctx.check(lib.lfm_dev_alloc(h, x.nbytes, _lib.ctypes.byref(dx)))
    ctx.check(lib.lfm_dev_alloc(h, y.nbytes, _lib.ctypes.byref(dy)))
    ctx.check(lib.lfm_memcpy_h2d(h, dx, x.ctypes.data, x.nbytes))
    ctx.check(lib.lfm_memcpy_h2d(h, dy, y.ctypes.data, y.nbytes))
    hp = work.model.hyp()
    out = np.empty(1)
    ts = []
    for it in range(6):
        t0 = time.perf_counter()
        ctx.check(lib.lfm_mll_f64_dev(h, dx, dy, x.shape[0], hp.ref, 0, _lib.dptr(out)))
        ts.append((time.perf_counter() - t0) * 1e3)
    ctx.profile(True)
    ctx.profile_reset()
    ctx.check(lib.lfm_mll_f64_dev(h, dx, dy, x.shape[0], hp.ref, 0, _lib.dptr(out)))
    st = {k: round(v["total_ms"], 3) for k, v in ctx.profile_read().items() if v["launches"]}
    ctx.profile(False)
    print(json.dumps({"lookahead": la, "side_cus": cus, "w4_min": os.environ.get("LFM_W4_MIN"),
                      "w2_min": os.environ.get("LFM_W2_MIN"),
                      "w8_min": os.environ.get("LFM_W8_MIN"),
                      "serial_below": os.environ.get("LFM_SERIAL_BELOW"), "n": int(x.shape[0]),
                      "ms_median": float(np.median(ts[1:])), "ms_min": float(min(ts[1:])),
                      "mll": float(out[0]), "kernel_ms_sum": st}), flush=True)
    lib.lfm_dev_free(h, dx)
    lib.lfm_dev_free(h, dy)
    ctx.close()
