"""Where a schedule-3 step launch's workgroup slots sit idle, from a unit trace
(scripts/unit_trace.py): per main-stream launch, the summed idle slot time (4 slots per CU
times the launch span, less the summed workgroup durations) split into
  ramp   before the CU first holds 4 workgroups,
  drain  after the CU last holds 4 workgroups,
  gaps   in between (a slot refilled late: dispatch, workgroup start-up),
and the median refill latency (a workgroup's exit to the next entry on the same CU).

    python scripts/unit_trace_report.py trace.npz [--json out.json]
"""
import json
import sys

import numpy as np

SLOTS_PER_CU = 4


def main():
    d = np.load(sys.argv[1])
    rec = d["rec"].astype(np.uint64)
    t0, t1, hw, tag = rec[:, 0].astype(np.int64), rec[:, 1].astype(np.int64), rec[:, 2], rec[:, 3]
    launch = (tag >> np.uint64(40)).astype(np.int64)
    role = ((tag >> np.uint64(32)) & np.uint64(0xFF)).astype(np.int64)
    cu = ((hw & np.uint64(0xFF00)) >> np.uint64(8)).astype(np.int64) | \
        ((hw >> np.uint64(32)) & np.uint64(0xF)).astype(np.int64) << 8
    base = t0[t0 > 0].min()
    rows = []
    tot = dict(ramp=0.0, drain=0.0, gaps=0.0, busy=0.0, span=0.0)
    for L in np.unique(launch):
        if L & (1 << 23):
            continue  # helper launches (side CUs)
        m = (launch == L) & (t0 > 0)
        a, b, c, r = t0[m], t1[m], cu[m], role[m]
        span = (b.max() - a.min()) * 0.01
        lo = a.min()
        cus = np.unique(c)
        ramp = drain = gaps = 0.0
        refill = []
        for k in cus:
            mk = c == k
            s, e = a[mk], b[mk]
            ev = np.concatenate([np.stack([s, np.ones_like(s)], 1), np.stack([e, -np.ones_like(e)], 1)])
            ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
            t_prev, act = lo, 0
            full_first = full_last = None
            idle_segs = []
            for t, dlt in ev:
                if t > t_prev:
                    idle_segs.append((t_prev, t, SLOTS_PER_CU - act))
                act += dlt
                if act >= SLOTS_PER_CU:
                    if full_first is None:
                        full_first = t
                    full_last = t
                t_prev = t
            end = b.max()
            if t_prev < end:
                idle_segs.append((t_prev, end, SLOTS_PER_CU - act))
            # the last instant the CU held 4: the latest entry that brought it to 4
            for (x0, x1, idle) in idle_segs:
                dur = (x1 - x0) * 0.01 * idle
                if full_first is None or x1 <= full_first:
                    ramp += dur
                elif x0 >= full_last:
                    drain += dur
                else:
                    gaps += dur
            # refill latency: each exit -> the next entry after it on this CU
            ss = np.sort(s)
            for x in e:
                j = np.searchsorted(ss, x)
                if j < len(ss):
                    refill.append((ss[j] - x) * 0.01)
            drain += (b.max() - end) * 0.01 * SLOTS_PER_CU
        nslots = SLOTS_PER_CU * len(cus)
        busy = ((b - a) * 0.01).sum()
        idle_all = nslots * span - busy
        row = dict(launch=int(L), units=int(m.sum()), cus=int(len(cus)),
                   start_us=(lo - base) * 0.01, span_us=span, occupancy=busy / (nslots * span),
                   idle_slot_us=idle_all, ramp=ramp, gaps=gaps,
                   drain=drain + (idle_all - ramp - gaps - drain),
                   refill_median_us=float(np.median(refill)) if refill else None,
                   roles={int(x): int((r == x).sum()) for x in np.unique(r)})
        rows.append(row)
        for k in ("ramp", "drain", "gaps"):
            tot[k] += row[k] / nslots
        tot["span"] += span
        print(f"launch {L:3d} start {row['start_us']:9.1f} span {span:8.1f} us occ {row['occupancy']:.3f} "
              f"idle/slot: ramp {ramp / nslots:6.1f} gaps {gaps / nslots:6.1f} drain {row['drain'] / nslots:6.1f} "
              f"refill med {row['refill_median_us'] or 0:5.2f} us  units {row['units']}")
    print(f"total span {tot['span']:.1f} us; idle per slot: ramp {tot['ramp']:.1f}, gaps {tot['gaps']:.1f}, "
          f"drain {tot['drain']:.1f} us")
    if "--json" in sys.argv:
        json.dump(dict(rows=rows, total=tot), open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
