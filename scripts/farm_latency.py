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


CHILD = r"""
# raw ctypes on the five entry points used (older builds lack later ABI additions)
import ctypes, json, sys, time
import numpy as np
lib = ctypes.CDLL(sys.argv[1])
vp = ctypes.c_void_p
lib.lfm_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
lib.lfm_farm_unique_id.argtypes = [vp, ctypes.POINTER(ctypes.c_ubyte)]
lib.lfm_farm_init.argtypes = [vp, ctypes.POINTER(ctypes.c_ubyte), ctypes.c_int, ctypes.c_int]
lib.lfm_farm_allgather_f64.argtypes = [vp, vp, ctypes.c_int64, vp]
lib.lfm_farm_destroy.argtypes = [vp]
lib.lfm_ctx_destroy.argtypes = [vp]
h = vp()
assert lib.lfm_ctx_create(0, ctypes.byref(h)) == 0
uid = (ctypes.c_ubyte * 128)()
assert lib.lfm_farm_unique_id(h, uid) == 0
assert lib.lfm_farm_init(h, uid, 1, 0) == 0
out = {}
for slots in (2, 4, 32):
    send = np.arange(slots, dtype=np.float64)
    recv = np.empty(slots)
    def g():
        assert lib.lfm_farm_allgather_f64(h, send.ctypes.data, slots, recv.ctypes.data) == 0
    for _ in range(20):
        g()
    lat = []
    for _ in range(int(sys.argv[2])):
        t0 = time.perf_counter()
        g()
        lat.append((time.perf_counter() - t0) * 1e6)
    assert np.array_equal(recv, send)
    out[str(8 * slots)] = {"median_us": float(np.median(lat)), "p10_us": float(np.percentile(lat, 10)),
                           "p90_us": float(np.percentile(lat, 90))}
lib.lfm_farm_destroy(h)
lib.lfm_ctx_destroy(h)
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
            r = subprocess.run([sys.executable, "-c", CHILD, os.path.abspath(lib), str(a.iters)],
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
