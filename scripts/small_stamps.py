"""Phase times of small_mll_kernel's block 0 on the C5 batch, from a library built with
make EXTRA=-DLFM_SMALL_STAMPS=1 (loaded with LFM_LIBRARY=; that build overwrites problems 1-5's
results with the stamps and the factor's shader clock, s_memtime counts per us).
    LFM_LIBRARY=ablibs/stamps/liblfm.so python scripts/small_stamps.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dis_project_amd import _lib, configs, farm  # noqa: E402

ws = configs.c5_ablations()
ev = farm.BatchEvaluator(_lib.get_context(0), [w.data for w in ws])
rows = []
for i in range(300):
    v = ev([w.model for w in ws])
    if i >= 30:
        rows.append(v[1:6].copy())
r = np.array(rows)
print("block 0 phase ends (us from its start): hyp+x+y staged, gram+residual, factor, output:",
      np.round(np.median(r[:, :4], axis=0), 2), "p10", np.round(np.percentile(r[:, :4], 10, axis=0), 2))
print("shader clock during the factor (MHz): median %.0f, p10 %.0f, p90 %.0f"
      % tuple(np.percentile(r[:, 4], [50, 10, 90])))
