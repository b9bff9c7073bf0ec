"""Latency of the farm's result exchange through liblfm (lfm_farm_allgather_f64) on ONE GPU: a
1-rank RCCL communicator, so no xGMI transfer — what is measured is the library's own path
around the collective (staging copies, the enqueue, the bounded host wait on the stream).
Interleaved over library builds (LFM_LIBRARY paths; one child process per build per round).

    python scripts/farm_latency.py [--json out] [--iters 400] [--rounds 3] lib.so [lib.so ...]
"""

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys, time
sys.path.insert(0, sys.argv[1])
import numpy as np
from dis_project_amd import _lib, farm
ctx = _lib.Context(0)
g = farm.RcclGather(ctx, 1, 0, farm.RcclGather.unique_id(ctx))
out = {}
for slots in (2, 4, 32):
    send = np.arange(slots, dtype=np.float64)
    for _ in range(20):
        g(send)
    lat = []
    for _ in range(int(sys.argv[2])):
        t0 = time.perf_counter()
        r = g(send)
        lat.append((time.perf_counter() - t0) * 1e6)
    assert np.array_equal(r, send)
    out[str(8 * slots)] = {"median_us": float(np.median(lat)), "p10_us": float(np.percentile(lat, 10)),
                           "p90_us": float(np.percentile(lat, 90))}
g.close()
ctx.close()
print(json.dumps(out))
"""


def main():
    p = argparse.ArgumentParser()
    p.add_argument("libs", nargs="+")
    p.add_argument("--iters", type=int, default=400)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--json")
    a = p.parse_args()
    res = {lib: [] for lib in a.libs}
    for rnd in range(a.rounds):
        for lib in a.libs:
            env = dict(os.environ, LFM_LIBRARY=os.path.abspath(lib))
            r = subprocess.run([sys.executable, "-c", CHILD, ROOT, str(a.iters)], env=env,
                               capture_output=True, text=True, timeout=300)
            if r.returncode:
                print(r.stderr, file=sys.stderr)
                raise SystemExit(r.returncode)
            res[lib].append(json.loads(r.stdout.strip().splitlines()[-1]))
            print(rnd, lib, res[lib][-1], flush=True)
    summary = {}
    for lib, runs in res.items():
        summary[lib] = {b: float(sorted(x[b]["median_us"] for x in runs)[len(runs) // 2])
                        for b in runs[0]}
    out = {"what": "lfm_farm_allgather_f64 on a 1-rank RCCL communicator (no xGMI transfer): "
                   "median latency per call in us by bytes per rank, median over rounds",
           "iters": a.iters, "rounds": a.rounds, "median_us_by_bytes": summary, "runs": res}
    print(json.dumps(summary, indent=1))
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
