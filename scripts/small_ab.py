"""Small-problem batch kernel (small_mll_kernel) of two library builds on the same 41 problems
(the C5 ablations, C1 and grid problems of n = 21 ... 64 under restart hyperparameters),
compared: bit for bit, else the largest relative difference.
    python scripts/small_ab.py libA libB"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(out):
    sys.path.insert(0, ROOT)
    from dis_project_amd import _lib, configs, farm
    ws = configs.c5_ablations() + [configs.c1_p53()]
    for G, T in ((4, 12), (3, 7), (7, 9), (2, 16), (8, 8)):
        base = configs.grid_workload("s", G, T, seed_params=G, seed_y=T)
        ws.append(base)
        for m in configs.c3_restarts(base, 4):
            ws.append(configs.Workload("r", m, base.data))
    ctx = _lib.get_context(0)
    ev = farm.BatchEvaluator(ctx, [w.data for w in ws])
    v = ev([w.model for w in ws])
    np.save(out, v)
    print([w.data.X.shape[0] for w in ws])


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        child(sys.argv[2])
        sys.exit(0)
    res = []
    for i, lib in enumerate(sys.argv[1:3]):
        env = dict(os.environ, LFM_LIBRARY=lib)
        subprocess.run([sys.executable, __file__, "--child", f"/tmp/small_ab_{i}.npy"], env=env,
                       check=True)
        res.append(np.load(f"/tmp/small_ab_{i}.npy"))
    a, b = res
    print("equal bits:", np.array_equal(a, b, equal_nan=True), "max rel diff:",
          float(np.nanmax(np.abs(a - b) / np.abs(a))), a[:3], b[:3])
