"""Recover the lane maps of v_mfma_f64_4x4x4_4b_f64 (and its A broadcast) by one-hot probing."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dis_project_amd import _lib  # noqa: E402

ctx = _lib.get_context(0)


def run(a, b, c):
    a, b, c = (np.ascontiguousarray(v, dtype=np.float64) for v in (a, b, c))
    d = np.empty(5 * 64)
    ctx.check(ctx.diag.lfm_probe_mfma4_layout(ctx.handle, _lib.dptr(a), _lib.dptr(b), _lib.dptr(c),
                                             _lib.dptr(d)))
    return d.reshape(5, 64)


ones = np.ones(64)
zero = np.zeros(64)
out = {"a_lane_to_out_lanes": {}, "b_lane_to_out_lanes": {}, "c_identity": None}
for mode in range(5):
    amap, bmap = {}, {}
    for p in range(64):
        e = np.zeros(64); e[p] = 1.0
        amap[p] = [int(q) for q in np.nonzero(run(e, ones, zero)[mode])[0]]
        bmap[p] = [int(q) for q in np.nonzero(run(ones, e, zero)[mode])[0]]
    out["a_lane_to_out_lanes"][mode] = amap
    out["b_lane_to_out_lanes"][mode] = bmap
# C passes through to the same lane
cc = np.arange(64, dtype=np.float64)
out["c_identity"] = bool(np.all(run(zero, zero, cc)[0] == cc))
# a generic product check: assume block b = lane // 16, A[i][k] at lane 16b + i + 4k ... printed raw
print(json.dumps(out))
