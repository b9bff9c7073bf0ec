"""Per-step timeline of the schedule-3 factorisation at N = 16384 from device stamps
(lfm_debug_stamps, 100 MHz s_memrealtime; include/lfm_diag.h): for each main-stream step
launch s (step s's trailing update + the tall solve of super-panel s + 1) the launch span,
the update units' span and rate, how long the tall units' last wait ran past the update
(the chain-bound exposure), and the chain (s + 1)'s own span.

    python scripts/step_timeline.py [--json out.json] [--grad] [--genes G]

--grad times value_and_grad's bordered factorisation (2Mp x 2Mp, every step updating the
sliding Mp-row window) instead of the MLL's. --genes G: the G x 256 grid (N = 256 G) instead
of C2's 64 genes (its first steps then have the shape of C2's tail steps).
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from dis_project_amd import _lib, configs  # noqa: E402

NB = 128
SLOTS = 4 * 224  # resident step-kernel workgroups: 4 per main-stream CU (32 side CUs)
TALL_SPLIT = 2  # tall units per 64-row x 128-column block of X (lfm_chol.hip LFM_TALL_SPLIT)


def plan(n, bordered=False):
    """Schedule 3's step plan (lfm_chol.hip chol_factor_solve, default LFM_W4_MIN/W2_MIN)."""
    Mp = (n + 1 + NB - 1) // NB * NB
    nblk = Mp // NB if bordered else (n + NB - 1) // NB
    w4 = int(os.environ.get("LFM_W4_MIN", 6144))
    w2 = int(os.environ.get("LFM_W2_MIN", 5120))
    steps, k = [], 0
    while k < nblk:
        m = Mp + NB if bordered else Mp - k * NB
        # the bulk width (lfm_chol.hip chol_factor_solve): 5, its first super-panel 4 (MLL)
        wb = 4 if bordered or len(steps) == 1 else 5
        w = wb if (m >= w4 and k + wb <= nblk) else 4 if (m >= w4 and k + 4 <= nblk) else \
            2 if (m >= w2 and k + 2 <= nblk) else 1
        if k == 0:
            w = 1
        steps.append((k, w))
        k += w
    return steps


def main():
    grad = "--grad" in sys.argv
    G = int(sys.argv[sys.argv.index("--genes") + 1]) if "--genes" in sys.argv else 64
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
    import time

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
    ctx.check(ctx.diag.lfm_debug_stamps(h, 1, None, 0))
    t0 = time.perf_counter()
    run()
    stamped_ms = (time.perf_counter() - t0) * 1e3
    buf = (ctypes.c_ulonglong * (256 * 24))()
    ctx.check(ctx.diag.lfm_debug_stamps(h, 0, buf, 256 * 24))
    allst = np.frombuffer(buf, dtype=np.uint64)
    ch = allst[: 256 * 16].reshape(256, 16).astype(np.int64)
    sp = allst[256 * 16:].reshape(256, 8).copy()
    steps = plan(n, grad)
    S = len(steps)
    Mp = (n + 1 + NB - 1) // NB * NB
    first = ~sp[:, 0]  # earliest unit start (stored as the max of the bitwise NOT)
    t_ref = int(min(int(ch[0][0]), int(first[0])))
    us = lambda t: (int(t) - t_ref) * 0.01  # noqa: E731
    rows = []
    tot_exposed = 0.0
    print(f"N={n}: {S} steps, plain {plain_ms:.2f} ms/eval, stamped {stamped_ms:.2f} ms")
    print(" s  w  m_tr   launch[us]  update[us] TF/s  exposed[us] chain(s+1)[us] clock[MHz] "
          "rest unit[us]")
    for s in range(S - 1):
        k, w = steps[s]
        K1 = (k + w) * NB
        m = Mp if grad else n - K1
        wn = steps[s + 1][1]
        d = min(wn * NB, m)
        alg = 2.0 * w * NB * (m * (m + 1) / 2 + (0 if grad else m) - d * (d + 1) / 2)
        st0, upd_end, wait_end, end = int(first[s]), int(sp[s][1]), int(sp[s][2]), int(sp[s][3])
        launch = (end - st0) * 0.01
        upd = (upd_end - st0) * 0.01 if upd_end else 0.0
        exposed = max(0.0, (wait_end - upd_end) * 0.01) if wait_end and upd_end else 0.0
        tot_exposed += exposed
        c = ch[s + 1]
        chain = (c[15] - c[0]) * 0.01 if c[0] and c[15] else float("nan")
        tf = alg / (upd * 1e-6) / 1e12 if upd > 0 else 0.0
        mhz = float(sp[s][4]) / float(sp[s][5]) * 100.0 if sp[s][5] else 0.0
        T = (m + NB - 1) // NB if not grad else Mp // NB
        nr = (T - wn) * (T - wn + 1)  # rest units (lfm_chol.hip update_args)
        unit_us = float(sp[s][5]) * 0.01 / nr if nr > 0 else 0.0
        na = 2 * wn * (T - wn)  # ahead units
        # tall units of this launch (X_{s+1}): rows below the next diagonal block, identity
        # padding rows (past n) skipped
        K1n = K1 + wn * NB
        rows_t = (Mp if not grad else 2 * Mp) - K1n
        nt_all = rows_t // 64 * wn
        nt = (nt_all if grad else ((n + 1 - K1n + 63) // 64) * wn) * TALL_SPLIT
        tall_us = float(sp[s][6]) * 0.01 / nt if nt > 0 else 0.0
        ahead_us = float(sp[s][7]) * 0.01 / na if na > 0 else 0.0
        # slot occupancy over the launch: summed unit time / (slots x launch span)
        busy = (float(sp[s][5]) + float(sp[s][6]) + float(sp[s][7])) * 0.01
        occ = busy / (SLOTS * launch) if launch > 0 else 0.0
        rows.append(dict(s=s, w=w, m=m, start_us=us(st0), launch_us=launch, update_us=upd,
                         update_tflops=tf, exposed_us=exposed, chain_next_us=chain,
                         chain_next_start_us=us(c[0]) if c[0] else None,
                         chain_next_done_us=us(c[15]) if c[15] else None, update_clock_mhz=mhz,
                         rest_unit_us=unit_us, tall_unit_us=tall_us, ahead_unit_us=ahead_us,
                         tall_units=nt, slot_occupancy=occ))
        print(f"{s:2d} {w:2d} {m:6d} {launch:10.1f} {upd:10.1f} {tf:5.1f} {exposed:10.1f} {chain:10.1f} "
              f"{mhz:7.0f} {unit_us:7.2f} tall {tall_us:6.2f} x{nt} ahead {ahead_us:6.2f} "
              f"occ {occ:.3f}")
    end_all = max(int(v) for v in sp[: S - 1, 3])
    print(f"span first unit -> last unit: {(end_all - int(first[0])) * 0.01:.1f} us; "
          f"chain-bound exposure (tall units waiting past the update) {tot_exposed:.1f} us")
    if "--json" in sys.argv:
        json.dump({"n": n, "grad": grad, "plain_ms": plain_ms, "stamped_ms": stamped_ms,
                   "exposed_us": tot_exposed, "steps": rows}, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
