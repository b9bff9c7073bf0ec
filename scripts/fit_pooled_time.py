"""Wall time of BatchTrainer.fit on the notebook's pooled problems (configs.notebook_pooled: the
three replicates pooled, N = 105, and the five leave-one-gene-out sets, N = 84: the two-wave
gradient path) and on the C1 p53 problem (N = 35), 150 adam(0.01) steps, median of 5 fits.
    python scripts/fit_pooled_time.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dis_project_amd import _lib, configs, objectives, trainer  # noqa: E402

ctx = _lib.get_context(0)
for name, ws in (("pooled (N = 105, 84 x 5)", configs.notebook_pooled()),
                 ("C1 p53 (N = 35)", [configs.c1_p53()])):
    times = []
    for rep in range(6):
        bt = trainer.BatchTrainer([w.model for w in ws], objectives.CustomConjMLL(negative=True),
                                  [w.data for w in ws], trainer.adam(0.01), num_iters=150, ctx=ctx)
        t0 = time.perf_counter()
        bt.fit()
        times.append(time.perf_counter() - t0)
        bt.close()
    ms = float(np.median(times[1:])) * 1e3
    print(f"{name}: {len(ws)} problems, 150 steps: {ms:.2f} ms per fit, {ms / 150 * 1e3:.1f} us a step",
          flush=True)
