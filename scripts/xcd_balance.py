"""Per-XCD balance of the schedule-3 step launches, from a unit trace (scripts/unit_trace.py):
for each main-stream launch, each XCD's last workgroup exit relative to the launch's end, its
last rest-unit exit and its summed unit time (which role ends each XCD's work). Tells whether a
launch's end drain is the last round of units on every XCD alike or one XCD finishing late.

    python scripts/xcd_balance.py trace.npz [--json out.json]"""
import json
import sys

import numpy as np


def main():
    d = np.load(sys.argv[1])
    rec = d["rec"].astype(np.uint64)
    t0, t1, hw, tag = rec[:, 0].astype(np.int64), rec[:, 1].astype(np.int64), rec[:, 2], rec[:, 3]
    launch = (tag >> np.uint64(40)).astype(np.int64)
    role = ((tag >> np.uint64(32)) & np.uint64(0xFF)).astype(np.int64)
    xcd = ((hw >> np.uint64(32)) & np.uint64(0xF)).astype(np.int64)
    rows = []
    for L in np.unique(launch):
        if L & (1 << 23):
            continue
        m = (launch == L) & (t0 > 0)
        if m.sum() < 2000:
            continue
        a, b, x, r = t0[m], t1[m], xcd[m], role[m]
        end, start = b.max(), a.min()
        per = []
        for k in range(8):
            mk = x == k
            if not mk.any():
                continue
            rest = mk & (r == 2)
            per.append(dict(xcd=k, last_exit_us=float((end - b[mk].max()) * 0.01),
                            last_rest_exit_us=float((end - b[rest].max()) * 0.01) if rest.any() else None,
                            busy_ms=float((b[mk] - a[mk]).sum() * 1e-5), units=int(mk.sum())))
        lag = [p["last_exit_us"] for p in per]
        rows.append(dict(launch=int(L), span_us=float((end - start) * 0.01), xcd=per,
                         spread_last_exit_us=float(max(lag) - min(lag))))
        print(f"launch {L:3d} span {(end - start) * 0.01:8.1f} us  per-XCD idle at end: "
              + " ".join(f"{v:6.1f}" for v in lag)
              + "  last rest exit before end: "
              + " ".join(f"{p['last_rest_exit_us']:6.1f}" for p in per if p["last_rest_exit_us"] is not None)
              + "  busy ms: " + " ".join(f"{p['busy_ms']:6.1f}" for p in per))
    if "--json" in sys.argv:
        json.dump(rows, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
