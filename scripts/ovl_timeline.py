"""Timeline of C3's restart pipeline from a rocprofv3 kernel trace (scripts/gpu_r06.sh ovltrace).

    python scripts/ovl_timeline.py gpurun_out/r06_ovltrace_0 gpurun_out/r06_ovltrace_1 [--json out]

An evaluation is the kernels from its tables_kernel to its finalize_kernel. Per trace: the
period between consecutive finalize ends (one evaluation's share of the wall), the tail (from
the first step launch with fewer than 6144 trailing rows — approximated as the last 44 step
launches of the evaluation — to its finalize), and, with the pipeline on, each evaluation's
prologue (its kernels before its second step launch) against the previous evaluation's
finalize: how much of it ran under that tail, and how long the bulk stream then waited."""

from __future__ import annotations

import csv
import glob
import json
import os
import sys

import numpy as np


def load(d):
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no kernel trace under {d}")
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                             r["Kernel_Name"], r.get("Queue_Id", r.get("Stream_Id", "?"))))
    rows.sort()
    return rows


def summarize(d):
    rows = load(d)
    fins = [r for r in rows if "finalize_kernel" in r[2]]
    q_main = max(set(r[3] for r in fins), key=lambda q: sum(1 for r in fins if r[3] == q))
    chains = [r for r in rows if "chain_kernel" in r[2]]
    q_side = max(set(r[3] for r in chains), key=lambda q: sum(1 for r in chains if r[3] == q))
    fin = np.array(sorted(r[1] for r in fins), dtype=np.float64)
    tab = np.array(sorted(r[0] for r in rows if "tables_kernel" in r[2]), dtype=np.float64)
    per = np.diff(fin) * 1e-3  # us
    out = {"trace": d, "evaluations": int(fin.size), "main_queue": q_main, "side_queue": q_side,
           "period_us_median": float(np.median(per)),
           "period_us_p10": float(np.percentile(per, 10)),
           "period_us_p90": float(np.percentile(per, 90))}
    msteps = np.array(sorted(r[0] for r in rows if "step_kernel" in r[2] and r[3] == q_main),
                      dtype=np.float64)
    other = [r for r in rows if r[3] not in (q_main, q_side)]
    tails, pro_end, l1 = [], [], []
    for k in range(1, fin.size):
        # this evaluation's launches on the bulk queue: after the previous finalize
        mine = msteps[(msteps > fin[k - 1]) & (msteps < fin[k])]
        if mine.size > 46:
            tails.append((fin[k] - mine[-44]) * 1e-3)
        if mine.size:
            l1.append((mine[0] - fin[k - 1]) * 1e-3)
        # its prologue: kernels off the pair's queues from its tables kernel on
        t0 = tab[(tab > fin[k - 1] - 30e6) & (tab < fin[k])]
        if t0.size:
            st = t0[0]
            nxt = tab[tab > st]
            end = nxt[0] if nxt.size else np.inf
            pk = [r for r in other if st <= r[0] < end]
            if pk:
                pro_end.append((max(r[1] for r in pk) - fin[k - 1]) * 1e-3)
    if tails:
        out["tail_us_median"] = float(np.median(tails))
    if pro_end:
        out["prologue_end_vs_prev_finalize_us_median"] = float(np.median(pro_end))
    if l1:
        out["first_bulk_launch_vs_prev_finalize_us_median"] = float(np.median(l1))
    return out


def main():
    args = sys.argv[1:]
    js = None
    if "--json" in args:
        i = args.index("--json")
        js = args[i + 1]
        args = args[:i] + args[i + 2:]
    res = [summarize(d) for d in args]
    for r in res:
        print(json.dumps(r))
    if js:
        with open(js, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
