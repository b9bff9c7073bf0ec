"""Seeded synthetic workloads for the five BASELINE.json configs.

``C1``  p53 5 genes x 7 timepoints, reference init hyperparameters (model.py:99-114,
        jitter 1e-4 from main.py:41), N = 35.
``C2``  64 genes x 256 timepoints, N = 16384, fp64, one MLL evaluation.
``C3``  C2 data x 32 random restarts (raw ~ N(0,1) -> Softplus / Sigmoid(0.5, 3.5)).
``C4``  256 genes x 256 timepoints, N = 65536, fp32 gram fill.
``C5``  3 replicates x 5 leave-one-gene-out ablations, N = 28 each (notebook.py:33-75).
``notebook_pooled``  the notebook's own fit data: the 3 replicates pooled (replicate=None,
        notebook.py:36), the 5 genes (N = 105) and their 5 leave-one-gene-out ablations (N = 84).

Every config is generated with numpy's default_rng so the container and the GPU box
rebuild bit-identical inputs from the seed alone.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .dataset import BARENCO_GENES, Dataset, SyntheticP53Data, dataset_3d, grid_inputs
from .model import ExactLFM


def softplus(x):
    """tfb.Softplus forward (model.py:66, 79, 86, 93)."""
    return np.logaddexp(0.0, np.asarray(x, np.float64))


def softplus_inverse(y):
    y = np.asarray(y, np.float64)
    return y + np.log(-np.expm1(-y))


def sigmoid_bounded(x, low=0.5, high=3.5):
    """tfb.Sigmoid(low=0.5, high=3.5) forward (model.py:111)."""
    return low + (high - low) / (1.0 + np.exp(-np.asarray(x, np.float64)))


def logit_bounded(y, low=0.5, high=3.5):
    """sigmoid_bounded's inverse."""
    u = (np.asarray(y, np.float64) - low) / (high - low)
    return np.log(u) - np.log1p(-u)


@dataclass
class Workload:
    name: str
    model: ExactLFM
    data: Dataset

    @property
    def n(self) -> int:
        return self.data.n


def grid_workload(name, G, T, seed_params, seed_y, jitter=1e-4, obs_stddev=1.0, l=2.5):
    rng = np.random.default_rng(seed_params)
    D = rng.uniform(0.2, 1.0, G)
    S = rng.uniform(0.5, 1.5, G)
    B = rng.uniform(0.01, 0.1, G)
    x = grid_inputs(G, T)
    ry = np.random.default_rng(seed_y)
    y = np.repeat(B / D, T) + 0.5 * ry.standard_normal(G * T)
    model = ExactLFM(jitter=jitter, obs_stddev=obs_stddev, num_genes=G, true_d=D, true_s=S,
                     true_b=B, l=l)
    return Workload(name, model, Dataset(x, y.reshape(-1, 1)))


def c1_p53(seed=1) -> Workload:
    data = SyntheticP53Data(replicate=0, seed=seed)
    x, y, _ = dataset_3d(data)
    return Workload("p53_5x7", ExactLFM(jitter=1e-4, num_genes=5), Dataset(x, y))


def c2(G=64, T=256) -> Workload:
    return grid_workload(f"synthetic_{G}x{T}_fp64", G, T, seed_params=2, seed_y=3)


def c3_restarts(base: Workload, count=32, first_seed=100):
    """Restart r: raw ~ N(0,1) (seed 100 + r), constrained through the model's bijectors."""
    G = base.model.num_genes
    models = []
    for r in range(count):
        raw = np.random.default_rng(first_seed + r).standard_normal(3 * G + 2)
        models.append(base.model.replace(true_d=softplus(raw[:G]), true_s=softplus(raw[G:2 * G]),
                                         true_b=softplus(raw[2 * G:3 * G]),
                                         obs_stddev=float(softplus(raw[3 * G])),
                                         l=float(sigmoid_bounded(raw[3 * G + 1]))))
    return models


def c4(G=256, T=256) -> Workload:
    return grid_workload(f"synthetic_{G}x{T}_fp32", G, T, seed_params=4, seed_y=5)


def c5_ablations(seeds=(10, 11, 12)):
    """3 synthetic 5-gene replicates x drop-one-gene -> 15 problems at N = 28."""
    out = []
    for r, seed in enumerate(seeds):
        for drop in BARENCO_GENES:
            genes = [g for g in BARENCO_GENES if g != drop]
            data = SyntheticP53Data(replicate=0, selected_genes=genes, seed=seed)
            x, y, _ = dataset_3d(data)
            out.append(Workload(f"rep{r}_minus_{drop}", ExactLFM(jitter=1e-4, num_genes=4),
                                Dataset(x, y)))
    return out


def c5_rounds(base_models, rounds, first_seed=500):
    """Hyperparameter rounds of the C5 problems (bench.py --workload c5 --rounds):
    round 0 is the problems' own models (the reference init, notebook.py:51); round k > 0
    perturbs every problem's hyperparameters independently, raw + 0.5 N(0, 1) in the
    bijectors' unconstrained space (seed first_seed + k), like C3's restarts of C2. Returns the
    models round-major: [round 0's P models, round 1's, ...]."""
    out = list(base_models)
    for k in range(1, rounds):
        rng = np.random.default_rng(first_seed + k)
        for m in base_models:
            G = m.num_genes
            raw = 0.5 * rng.standard_normal(3 * G + 2)
            out.append(m.replace(
                true_d=softplus(softplus_inverse(m.true_d) + raw[:G]),
                true_s=softplus(softplus_inverse(m.true_s) + raw[G:2 * G]),
                true_b=softplus(softplus_inverse(m.true_b) + raw[2 * G:3 * G]),
                obs_stddev=float(softplus(softplus_inverse(m.obs_stddev) + raw[3 * G])),
                l=float(sigmoid_bounded(logit_bounded(m.l) + raw[3 * G + 1]))))
    return out


def notebook_pooled(seed=10):
    """notebook.py:32-75 with replicate=None: the three replicates pooled by dataset_3d
    (15 blocks of 7 timepoints, genes repeating per replicate), the 5 Barenco genes (N = 105)
    and each leave-one-gene-out gene set (N = 84); ExactLFM(jitter=1e-4, num_genes=len(genes))."""
    out = []
    for drop in [None] + list(BARENCO_GENES):
        genes = list(BARENCO_GENES) if drop is None else [g for g in BARENCO_GENES if g != drop]
        data = SyntheticP53Data(replicate=None, selected_genes=None if drop is None else genes,
                                seed=seed)
        x, y, _ = dataset_3d(data)
        out.append(Workload("pooled" if drop is None else f"pooled_minus_{drop}",
                            ExactLFM(jitter=1e-4, num_genes=len(genes)), Dataset(x, y)))
    return out
