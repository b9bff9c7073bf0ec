"""Per-dispatch durations of the schedule-3 kernels of ONE evaluation from a rocprofv3
--kernel-trace CSV (no device stamps: the launches' own durations), step plan alongside.

    python scripts/dispatch_times.py <kernel_trace.csv> [N]"""
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from step_timeline import NB, plan  # noqa: E402


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    rows = list(csv.DictReader(open(path)))
    step = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
                  if "step_kernel" in r["Kernel_Name"])
    chain = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
                   if "chain_kernel" in r["Kernel_Name"])
    steps = plan(n)
    S = len(steps)
    per = S  # step launches per evaluation: X_0 + S - 1 updates
    last = step[-per:]
    t0 = last[0][0]
    Mp = (n + 1 + NB - 1) // NB * NB
    tot = 0.0
    print(" i  w   m_tr  start[us]  dur[us]  TF/s(update)")
    for i, (a, b) in enumerate(last):
        dur = (b - a) * 1e-3
        tot += dur
        if i == 0:
            print(f"{i:2d}  X0        {(a - t0) * 1e-3:9.1f} {dur:8.1f}")
            continue
        s = i - 1
        k, w = steps[s]
        K1 = (k + w) * NB
        m = n - K1
        wn = steps[s + 1][1]
        d = min(wn * NB, m)
        alg = 2.0 * w * NB * (m * (m + 1) / 2 + m - d * (d + 1) / 2)
        print(f"{i:2d} {w:2d} {m:6d} {(a - t0) * 1e-3:9.1f} {dur:8.1f} {alg / (dur * 1e-6) / 1e12:6.1f}")
    span = (last[-1][1] - last[0][0]) * 1e-3
    print(f"sum of step launches {tot:.1f} us, span {span:.1f} us, chain launches in trace "
          f"{len(chain)}")


if __name__ == "__main__":
    main()
