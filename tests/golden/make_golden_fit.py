"""Golden training trajectories for the batched on-device fit (lfm_batch_fit_f64,
dis_project_amd.trainer.BatchTrainer): JaxTrainer.fit (src/trainer.py:162-228) driven by the CPU
oracle's value and gradient (oracle/lfm_oracle.py mll_grad: complex-step derivatives of the
reference kernel, explicit Sigma^{-1}), through the host restatement of the loop
(dis_project_amd/trainer.py: bijectors, chain rule, optax.adam, after_epoch).

    python tests/golden/make_golden_fit.py      # rewrites tests/golden/fit_*.npz (~2.5 min)

Cases (the reference's own training configurations):
  fit_c5        the 15 replicate x leave-one-gene-out problems of configs[4] (N = 28), the
                notebook's fit: adam(0.01), 150 steps, fix_params=False (notebook.py:55-75)
  fit_c1        the C1 problem (5 genes x 7 times, N = 35), main.py's fit: adam(0.01), 150
                steps, fix_params=True, num_steps_per_epoch=1000 (main.py:45-59)
  fit_c1_epoch  the same with num_steps_per_epoch=50: after_epoch's index-3 quirk on the
                unconstrained leaves at steps 0, 50 and 100 (trainer.py:205-210)
  fit_pooled    the notebook's own data (replicate=None: three replicates pooled, N = 105) and
                its 5 leave-one-gene-out ablations (N = 84), adam(0.01), 150 steps,
                fix_params=False (notebook.py:32-75)
Each holds, per problem, the packed raw parameters before and after, the loss history
[P, iters] and the final constrained parameters.
"""

from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from dis_project_amd import configs, farm  # noqa: E402
from dis_project_amd import trainer as TR  # noqa: E402
from oracle import lfm_oracle as O  # noqa: E402


class OracleObjective:
    def __init__(self, negative=True):
        self.negative = negative

    def value_and_grad(self, model, data):
        g = O.mll_grad(data.X, data.y, model.true_d, model.true_s, model.true_b, model.l,
                       model.obs_stddev, model.jitter, self.negative)
        return g["value"], {"true_d": g["d"], "true_s": g["s"], "true_b": g["b"],
                            "l": g["l"], "obs_stddev": g["obs_stddev"]}


def run(name, models, datasets, iters, fix_params, spe):
    raw0 = TR.pack_raw([TR.unconstrain(m) for m in models], [m.jitter for m in models])
    hists, raws, finals = [], [], []
    for m, d in zip(models, datasets):
        t = TR.JaxTrainer(m, OracleObjective(True), d, TR.adam(0.01), num_iters=iters)
        fm, h = t.fit(fix_params=fix_params, num_steps_per_epoch=spe)
        hists.append(h)
        raws.append(t.raw)
        finals.append(np.concatenate([fm.true_d, fm.true_s, fm.true_b, [fm.l, fm.obs_stddev]]))
    raw1 = TR.pack_raw(raws, [m.jitter for m in models])
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), raw0=raw0, raw1=raw1,
                        hist=np.asarray(hists), final=np.concatenate(finals),
                        genes=np.array([m.num_genes for m in models]), iters=iters,
                        fix_params=int(fix_params), spe=spe)
    print(f"{name:14s} P={len(models):2d} first {hists[0][0]:.10g} last {hists[0][-1]:.10g}")


def main():
    models, datasets = farm.workload("c5")
    run("fit_c5", models, datasets, 150, False, 1000)
    c1 = configs.c1_p53()
    run("fit_c1", [c1.model], [c1.data], 150, True, 1000)
    run("fit_c1_epoch", [c1.model], [c1.data], 150, True, 50)
    ws = configs.notebook_pooled()
    run("fit_pooled", [w.model for w in ws], [w.data for w in ws], 150, False, 1000)


if __name__ == "__main__":
    main()
