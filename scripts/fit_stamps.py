"""Per-step phase times of small_fit_kernel's block 0 (problem 0) on the C5 batch, from a
library built with make EXTRA=-DLFM_FIT_STAMPS=1 (loaded with LFM_LIBRARY=; that build
overwrites problem 0's first twelve history entries with the phase sums).
    LFM_LIBRARY=ablibs/fitst/liblfm.so python scripts/fit_stamps.py [iters] [c5|pooled]
(pooled: configs.notebook_pooled, block 0 = the N = 105 problem on the two-wave path)"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dis_project_amd import _lib, configs, objectives, trainer  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 150
which = sys.argv[2] if len(sys.argv) > 2 else "c5"
ws = configs.c5_ablations() if which == "c5" else configs.notebook_pooled()
names = ["(loop top)", "gram (+ tables)", "factor | grad tables", "W (two waves)",
         "tr(W dK) reduction", "gradient out", "Adam + after_epoch + constrain",
         "  (inside phase 2) wave 0: factor done", "  (inside phase 2) wave 0: W written",
         "  (inside phase 2) wave 1: grad tables done",
         "  (inside phase 1) thread 0: gram tables + barrier", "  (inside phase 1) thread 0: gram elements"]
ctx = _lib.get_context(0)
res = []
for rep in range(5):
    bt = trainer.BatchTrainer([w.model for w in ws], objectives.CustomConjMLL(negative=True),
                              [w.data for w in ws], trainer.adam(0.01), num_iters=iters, ctx=ctx)
    t0 = time.perf_counter()
    bt.fit()
    wall = time.perf_counter() - t0
    print('raw', bt.history[0, :12])
    res.append(bt.history[0, :12] * 0.01 / iters)  # ticks of 10 ns -> us per step
    bt.close()
r = np.median(np.array(res), axis=0)
for nm, v in zip(names, r):
    print(f"{nm:34s} {v:7.2f} us/step")
print(f"{'sum of phases':34s} {r[:7].sum():7.2f} us/step; last fit wall {wall * 1e3:.2f} ms for {iters} steps")
