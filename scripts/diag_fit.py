import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
from dis_project_amd import _lib, farm
from dis_project_amd import trainer as TR
from oracle import lfm_oracle as O
ctx = _lib.get_context()
models, datasets = farm.workload("c5")
models, datasets = models[:5], datasets[:5]
ev = farm.BatchEvaluator(ctx, datasets, negative=True)
genes = [m.num_genes for m in models]
batch = ev.registered(genes)
raw0 = TR.pack_raw([TR.unconstrain(m) for m in models], [m.jitter for m in models])
opt = _lib.LfmAdam(0.01, 0.9, 0.999, 1e-8, 0.0, 30, 1)
a = raw0.copy(); ma = np.zeros_like(a); na = np.zeros_like(a)
ha = np.empty((80, 5))
ctx.check(ctx.lib.lfm_batch_fit_f64(ctx.handle, batch, _lib.ctypes.byref(opt), 1, 0, 80, _lib.dptr(a), _lib.dptr(ma), _lib.dptr(na), _lib.dptr(ha), None))
trainers = [TR.JaxTrainer(m, None, d, TR.adam(0.01), num_iters=80) for m, d in zip(models, datasets)]
raws = [t.raw for t in trainers]
states = [TR.adam(0.01).init(r) for r in raws]
hist = []
for s in range(80):
    cur = [TR.constrain(r, m) for r, m in zip(raws, models)]
    vals, grads = ev.value_and_grad(cur)
    hist.append(vals)
    rel = np.abs(vals - ha[s]) / np.abs(ha[s])
    if s % 5 == 0 or rel.max() > 1e-12:
        # oracle check of this step's gradient for the worst problem
        p = int(np.argmax(rel))
        m, d = cur[p], datasets[p]
        ref = O.mll_grad(d.X, d.y, m.true_d, m.true_s, m.true_b, m.l, m.obs_stddev, m.jitter, True)
        gerr = max(np.max(np.abs(grads[p][k] - ref[kk]) / (ref["scale_" + kk] + 1e-300))
                   for k, kk in (("true_d", "d"), ("true_s", "s"), ("true_b", "b"), ("l", "l"), ("obs_stddev", "obs_stddev")))
        print(s, "max rel diff fit vs host loop", rel.max(), "problem", p, "val", vals[p], "oracle", ref["value"], "grad err/scale", gerr, flush=True)
    for p in range(5):
        g = TR.chain_rule(raws[p], grads[p])
        upd, states[p] = TR.adam(0.01).update(g, states[p], raws[p])
        raws[p] = TR.apply_updates(raws[p], upd)
        if s % 30 == 0:
            raws[p] = TR.JaxTrainer.after_epoch(raws[p], True)
    if s > 40 and rel.max() > 1e-6: break
ev.close()
