"""Input side of the hot path: gpjax ``Dataset``, a synthetic stand-in for
``JaxP53Data`` and ``dataset_3d`` (wejpurvis/DIS_project src/dataset.py).

The Barenco CSVs are not shipped with the reference (data/README.md:3-5), so
``SyntheticP53Data`` produces arrays with the same shapes and attributes as
``JaxP53Data`` (dataset.py:21-210): ``gene_expressions`` (R, G, T),
``gene_variances`` (R, G, T), ``timepoints`` = linspace(0, 12, T) (dataset.py:108),
``data`` (list of (timepoints, expressions) per replicate x gene, replicate-major,
dataset.py:117-144), ``shape`` / ``__getitem__`` / ``__len__``.
This is host-side layout plumbing (O(N) bytes), not hot-path arithmetic.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np

BARENCO_GENES = ["DDB2", "BIK", "DR5", "p21", "SESN1"]  # dataset.py selected order


@dataclass
class Dataset:
    """gpjax.Dataset(X, y): X [N, D], y [N, 1]."""

    X: np.ndarray
    y: np.ndarray

    def __post_init__(self):
        self.X = np.asarray(self.X, dtype=np.float64)
        self.y = np.asarray(self.y, dtype=np.float64)
        if self.y.ndim == 1:
            self.y = self.y.reshape(-1, 1)
        if self.X.ndim != 2 or self.y.ndim != 2 or self.X.shape[0] != self.y.shape[0]:
            raise ValueError("Dataset needs X [N, D] and y [N, 1] with matching N")

    @property
    def n(self) -> int:
        return self.X.shape[0]


class SyntheticP53Data:
    """Seeded stand-in for ``JaxP53Data(replicate, selected_genes)`` (dataset.py:45-144)."""

    def __init__(self, replicate=None, selected_genes=None, num_genes=5, num_timepoints=7,
                 num_replicates=3, seed=0, expressions=None, variances=None):
        all_genes = (BARENCO_GENES if num_genes == 5 else [f"g{i}" for i in range(num_genes)])
        if replicate is not None and not (0 <= replicate < num_replicates):
            raise AssertionError("Invalid replicate number")  # dataset.py:62
        rng = np.random.default_rng(seed)
        T = num_timepoints
        if expressions is None:
            expressions = rng.normal(0.5, 0.5, size=(num_replicates, len(all_genes), T))
        if variances is None:
            variances = rng.uniform(0.01, 0.05, size=expressions.shape)
        expressions = np.asarray(expressions, np.float64)
        variances = np.asarray(variances, np.float64)
        if selected_genes is not None:
            valid = set(all_genes)
            sel = set(selected_genes)
            if not sel.issubset(valid):
                raise ValueError(f"Invalid gene names provided: {', '.join(sel - valid)}")
            if len(selected_genes) != len(sel):
                dup = {g for g in selected_genes if selected_genes.count(g) > 1}
                raise ValueError(f"Duplicate genes provided: {', '.join(dup)}")
            if len(selected_genes) == 0:
                raise ValueError("Empty list of genes selected, set 'selected_genes' to None")
            indices = [i for i, g in enumerate(all_genes) if g in selected_genes]
            self.selected_indices = [all_genes.index(g) for g in selected_genes]
            self.gene_names = list(selected_genes)
            expressions = expressions[:, indices]
            variances = variances[:, indices]
        else:
            self.selected_indices = list(range(len(all_genes)))
            self.gene_names = list(all_genes)
        self.num_genes = len(self.gene_names)
        self.timepoints = np.linspace(0, 12, T)
        self.f_observed = np.array([0.1845, 1.1785, 1.6160, 0.8156, 0.6862, -0.1828,
                                    0.5131]).reshape(1, 1, 7)
        self.gene_variances_raw = variances
        if replicate is None:
            self.gene_expressions = expressions
            self.data = [(self.timepoints, expressions[r, i])
                         for r in range(expressions.shape[0]) for i in range(self.num_genes)]
            self.gene_variances = np.array([variances[r, i] for r in range(expressions.shape[0])
                                            for i in range(self.num_genes)])
        else:
            self.gene_expressions = expressions[replicate:replicate + 1]
            self.data = [(self.timepoints, self.gene_expressions[0, i])
                         for i in range(self.num_genes)]
            self.gene_variances = variances[replicate:replicate + 1]

    def __getitem__(self, index):
        if index < 0 or index >= len(self.data):
            raise IndexError("Index out of range")
        return self.data[index]

    def __len__(self):
        return len(self.data)

    @property
    def shape(self):
        return np.array(self.data).shape


def dataset_3d(data):
    """dataset.py:358-399: x rows (t, gene, 1) ordered replicate-major, gene-major, time.

    Returns (x [N, 3], y [N, 1], variances [N, 1]) with N = genes * timepoints * replicates.
    """
    num_genes = data.num_genes
    replicates = data.shape[0] // num_genes
    gene_data = np.array([data[i] for i in range(len(data))])
    time_points = gene_data[0, 0, :]
    time_points_repeated = np.tile(time_points, gene_data.shape[0])
    gene_indices = np.tile(np.repeat(np.arange(num_genes), len(time_points)), replicates)
    ones = np.ones(num_genes * len(time_points) * replicates, dtype=np.int64)
    training_times = np.stack((time_points_repeated, gene_indices, ones), axis=-1).astype(np.float64)
    gene_expressions = gene_data[:, 1, :].flatten().reshape(-1, 1)
    variances = np.asarray(data.gene_variances).flatten().reshape(-1, 1)
    return training_times, gene_expressions, variances


def grid_inputs(num_genes: int, num_timepoints: int, replicates: int = 1, t_max: float = 12.0):
    """x for R replicates x G genes x T points of linspace(0, t_max, T) in dataset_3d order."""
    t = np.linspace(0, t_max, num_timepoints)
    x = np.stack((np.tile(t, num_genes * replicates),
                  np.tile(np.repeat(np.arange(num_genes), num_timepoints), replicates),
                  np.ones(num_genes * num_timepoints * replicates)), axis=-1)
    return x.astype(np.float64)


def generate_test_times(t: int = 100) -> np.ndarray:
    """utils.py:268-287: latent-force test inputs (linspace(0, 13, t), gene -1, flag 0).
    Gene -1 wraps to the last gene under JAX gather semantics; with flag 0 only the
    kff / kxf branches read it."""
    times = np.linspace(0, 13, t)
    return np.stack((times, np.repeat(-1.0, t), np.repeat(0.0, t)), axis=-1)


def generate_test_times_pred(t: int = 100, num_genes: int = 5) -> np.ndarray:
    """utils.py:290-314 (and GeneExpressionPredictor.generate_test_times_pred, utils.py:81-98):
    gene-expression test inputs with 1-based gene indices 1..num_genes and flag 1. Index
    num_genes is out of range and clamps to the last gene (JAX gather), a reference quirk
    kept for parity."""
    times = np.linspace(0, 13, t)
    return np.stack((np.tile(times, num_genes), np.repeat(np.arange(1, num_genes + 1), t),
                     np.ones(t * num_genes)), axis=1).astype(np.float64)
