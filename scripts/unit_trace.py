"""Per-workgroup trace of one schedule-3 MLL evaluation (lfm_debug_trace, include/lfm_diag.h):
every step-kernel and side-CU-helper workgroup's entry / exit time (100 MHz), the CU it ran on
and its role / unit. Written raw to an .npz for scripts/unit_trace_report.py.

    python scripts/unit_trace.py out.npz [--genes G] [--grad]
"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from dis_project_amd import _lib, configs  # noqa: E402


def main():
    out_path = sys.argv[1]
    G = int(sys.argv[sys.argv.index("--genes") + 1]) if "--genes" in sys.argv else 64
    grad = "--grad" in sys.argv
    work = configs.c2(G)
    n = work.n
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
    gv = np.empty(3 * work.model.num_genes + 2)
    hp = work.model.hyp()

    def run():
        if grad:
            ctx.check(lib.lfm_mll_grad_f64(h, _lib.dptr(x), _lib.dptr(y), n, hp.ref, 1,
                                           _lib.dptr(out), _lib.dptr(gv)))
        else:
            ctx.check(lib.lfm_mll_f64_dev(h, dx, dy, n, hp.ref, 0, _lib.dptr(out)))

    for _ in range(3):
        run()
    t0 = time.perf_counter()
    for _ in range(5):
        run()
    plain_ms = (time.perf_counter() - t0) / 5 * 1e3
    ref = float(out[0])
    cap = 4 << 20
    ctx.check(ctx.diag.lfm_debug_trace(h, cap, None, 0, None))
    t0 = time.perf_counter()
    run()
    traced_ms = (time.perf_counter() - t0) * 1e3
    nw = ctypes.c_int64()
    buf = np.zeros(4 * cap, dtype=np.uint64)
    ctx.check(ctx.diag.lfm_debug_trace(h, 0, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)),
                                       cap, ctypes.byref(nw)))
    rec = buf[: 4 * nw.value].reshape(-1, 4)
    print(f"N={n}: plain {plain_ms:.2f} ms, traced {traced_ms:.2f} ms, {nw.value} workgroups, "
          f"MLL {'identical' if float(out[0]) == ref else 'DIFFERS'}")
    np.savez_compressed(out_path, rec=rec, n=n, plain_ms=plain_ms, traced_ms=traced_ms,
                        grad=grad)


if __name__ == "__main__":
    main()
