"""Where a C5 step's wall time goes on the host (bench.py --workload c5's step at one rank):
the Python packing of the 15 models' hyperparameters (BatchEvaluator._pack), the library call
(lfm_batch_mll_f64: launch, the kernel, the bounded wait on the status words) and the step as
bench.py times it, medians over many steps.
    python scripts/c5_host_split.py [steps]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dis_project_amd import _lib, farm  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
ctx = _lib.get_context()
models, datasets = farm.workload("c5")
ev = farm.BatchEvaluator(ctx, datasets)
fm = farm.Farm(1, 0, None)
evaluate = lambda ms, ds: ev(ms)  # noqa: E731
lib = ctx.lib
for _ in range(300):
    fm.run_problems(models, datasets, evaluate)
pack, call, step = [], [], []
for _ in range(steps):
    t0 = time.perf_counter()
    ev._pack(models)
    t1 = time.perf_counter()
    rc = lib.lfm_batch_mll_f64(ctx.handle, ev.batch, ev._buf_ptr, 0, ev._out_ptr, ev._st_ptr)
    t2 = time.perf_counter()
    ctx.check(rc, allow_not_pd=True)
    pack.append(t1 - t0)
    call.append(t2 - t1)
for _ in range(steps):
    t0 = time.perf_counter()
    fm.run_problems(models, datasets, evaluate)
    step.append(time.perf_counter() - t0)
us = lambda v: float(np.median(v)) * 1e6  # noqa: E731
print(f"pack {us(pack):.2f} us  library call {us(call):.2f} us  bench step {us(step):.2f} us")
ev.close()
