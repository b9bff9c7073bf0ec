"""Time value_and_grad (lfm_mll_grad_f64) at N = G*T on the C2 workload; one JSON line with
ms per call, the kernel breakdown and the gradient's max |component|."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from dis_project_amd import CustomConjMLL, configs  # noqa: E402

G = int(os.environ.get("SWEEP_G", "64"))
T = int(os.environ.get("SWEEP_T", "256"))
work = configs.grid_workload("grad", G, T, seed_params=2, seed_y=3)
obj = CustomConjMLL(negative=True)
ts = []
for _ in range(4):
    t0 = time.perf_counter()
    v, g = obj.value_and_grad(work.model, work.data)
    ts.append((time.perf_counter() - t0) * 1e3)
ctx = work.model.ctx
ctx.profile(True)
ctx.profile_reset()
obj.value_and_grad(work.model, work.data)
st = {k: round(x["total_ms"], 3) for k, x in ctx.profile_read().items() if x["launches"]}
ctx.profile(False)
mll_ms = []
for _ in range(3):
    t0 = time.perf_counter()
    v2 = obj(work.model, work.data)
    mll_ms.append((time.perf_counter() - t0) * 1e3)
print(json.dumps({"n": G * T, "grad_ms_median": float(np.median(ts[1:])),
                  "mll_ms_median": float(np.median(mll_ms)), "value": v, "value_mll": v2,
                  "max_abs_grad": float(max(np.max(np.abs(np.atleast_1d(x))) for x in g.values())),
                  "kernel_ms_sum": st}), flush=True)
