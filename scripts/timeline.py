"""Analyse a rocprofv3 kernel trace of chol_sweep (look-ahead on): per block-column step the
main-stream SYRK span, the side chain (syrk next -> potrf -> trsm) span, and the idle time
of the main stream waiting for the side chain. Uses the last evaluation in the trace."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# split evaluations at gram kernels
evals, cur = [], []
for r in rows:
    if "gram_grid" in r["Kernel_Name"] and cur:
        evals.append(cur)
        cur = []
    cur.append(r)
evals.append(cur)
ev = evals[-1]
t0 = int(ev[0]["Start_Timestamp"])
by_q = defaultdict(list)
for r in ev:
    by_q[r["Queue_Id"]].append(r)
print("queues:", {q: len(v) for q, v in by_q.items()})
end = max(int(r["End_Timestamp"]) for r in ev)
print(f"eval span {(end - t0) / 1e6:.3f} ms")
kinds = defaultdict(float)
for r in ev:
    k = r["Kernel_Name"].split("(")[0].split("::")[-1]
    kinds[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
print({k: round(v, 3) for k, v in kinds.items()})
# main queue = the one with gram; idle gaps there
mainq = next(r["Queue_Id"] for r in ev if "gram_grid" in r["Kernel_Name"])
m = by_q[mainq]
gaps = []
for a, b in zip(m, m[1:]):
    g = int(b["Start_Timestamp"]) - int(a["End_Timestamp"])
    gaps.append((g, b["Kernel_Name"].split("(")[0].split("::")[-1], int(a["End_Timestamp"]) - t0))
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in m)
print(f"main queue busy {busy / 1e6:.3f} ms, idle {sum(g for g, _, _ in gaps) / 1e6:.3f} ms")
# bucket idle by time into the eval (ms)
buckets = defaultdict(float)
for g, name, t in gaps:
    buckets[int(t / 5e6)] += g / 1e6
print("main idle per 5 ms window:", {f"{5 * k}-{5 * k + 5}": round(v, 3) for k, v in sorted(buckets.items())})
side = [r for q, v in by_q.items() if q != mainq for r in v]
for name in ("potrf", "trsm", "syrk"):
    d = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in side if name in r["Kernel_Name"])
    if d:
        print(f"side {name}: n={len(d)} median {d[len(d) // 2]:.1f} us, p90 {d[int(len(d) * .9)]:.1f} us")
