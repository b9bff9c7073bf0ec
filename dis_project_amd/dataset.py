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


# ------------------------------------------------------------ Barenco CSV loader
# dataset.py:213-321. The CSVs themselves are not distributed with the reference
# (data/README.md); the format is: a probe-ID index column, then columns
# cARP{r}-{t}hrs.CEL (r = 1..3, t = 0, 2, ..., 12), PUMA log-expressions in
# barencoPUMA_exprs.csv and their standard errors in barencoPUMA_se.csv.
BARENCO_PROBES = {
    "203409_at": "DDB2",
    "202284_s_at": "p21",
    "218346_s_at": "SESN1",
    "205780_at": "BIK",
    "209295_at": "DR5",
    "211300_s_at": "p53",
}
BARENCO_ORDER = ["DDB2", "BIK", "DR5", "p21", "SESN1", "p53"]
BARENCO_COLUMNS = [f"cARP{r}-{t}hrs.CEL" for r in range(1, 4) for t in np.arange(7) * 2]


def load_barenco_data(dir_path):
    """dataset.py:213-321: read the two CSVs, keep the six known probes in the order
    DDB2, BIK, DR5, p21, SESN1, p53, log-normal transform (mean e^{mu + s^2/2}, variance
    (e^{s^2} - 1) e^{2 mu + s^2}) and rescale each gene by the ddof=1 standard deviation of
    its first replicate. Falls back to ../data like the reference."""
    import os

    import pandas as pd

    def read(name):
        try:
            with open(os.path.join(dir_path, name)) as f:
                return pd.read_csv(f, index_col=0)
        except FileNotFoundError:
            with open(os.path.join("../data", name)) as f:
                return pd.read_csv(f, index_col=0)

    exprs = read("barencoPUMA_exprs.csv")
    se = read("barencoPUMA_se.csv")
    genes = exprs[exprs.index.isin(list(BARENCO_PROBES))][BARENCO_COLUMNS]
    genes_se = se[se.index.isin(list(BARENCO_PROBES))][BARENCO_COLUMNS]
    genes = genes.rename(index=BARENCO_PROBES).reindex(BARENCO_ORDER)
    genes_se = genes_se.rename(index=BARENCO_PROBES).reindex(BARENCO_ORDER)

    mu = genes.values  # [6, 21]
    var = genes_se.values ** 2
    full = np.exp(mu + var / 2)
    var_full = (np.exp(var) - 1) * np.exp(2 * mu + var)
    scale = np.sqrt(np.var(full[:, :7], axis=1, ddof=1))[:, None]  # first replicate, per gene
    expr = full / scale
    varr = var_full / scale**2
    return {
        "gene_names": list(genes.index[:-1]),
        "gene_expressions": np.float64(expr[:-1]).reshape((5, 3, 7)).swapaxes(0, 1),
        "gene_variances": np.float64(varr[:-1]).reshape((5, 3, 7)).swapaxes(0, 1),
        "p53_expressions": np.float64(expr[-1:]).reshape((3, 1, 7)),
        "p53_variances": np.float64(varr[-1:]).reshape((3, 1, 7)),
    }


class JaxP53Data(SyntheticP53Data):
    """dataset.py:21-210: the Barenco data from CSV (load_barenco_data), with the same
    replicate / gene selection and layout as the synthetic stand-in."""

    def __init__(self, replicate=None, data_dir="data", selected_genes=None):
        d = load_barenco_data(data_dir)
        if replicate is not None and not (0 <= replicate < 3):
            raise AssertionError("Invalid replicate number")  # dataset.py:62
        super().__init__(replicate=replicate, selected_genes=selected_genes, num_genes=5,
                         num_timepoints=7, num_replicates=3,
                         expressions=d["gene_expressions"], variances=d["gene_variances"])

    def params_ground_truth(self):
        """dataset.py:194-210: Barenco et al. (2006) measured B, S, D, filtered by the
        selected genes."""
        B = np.array([0.0649, 0.0069, 0.0181, 0.0033, 0.0869])
        D = np.array([0.2829, 0.3720, 0.3617, 0.8000, 0.3573])
        S = np.array([0.9075, 0.9748, 0.9785, 1.0000, 0.9680])
        idx = self.selected_indices
        return B[idx], S[idx], D[idx]


def write_barenco_csv(dir_path, log_expr, se, extra_probes=2, seed=0):
    """Write log-expressions [6, 21] and standard errors [6, 21] (rows in BARENCO_ORDER) as
    the two Barenco CSVs, probes shuffled among `extra_probes` unrelated rows and extra
    columns — the on-disk format load_barenco_data reads (tests / synthetic runs)."""
    import os

    import pandas as pd

    rng = np.random.default_rng(seed)
    inv = {v: k for k, v in BARENCO_PROBES.items()}
    probes = [inv[g] for g in BARENCO_ORDER] + [f"9999{i}_at" for i in range(extra_probes)]
    cols = BARENCO_COLUMNS + ["cMOCK1-0hrs.CEL"]
    order = rng.permutation(len(probes))
    for name, arr in (("barencoPUMA_exprs.csv", log_expr), ("barencoPUMA_se.csv", se)):
        full = np.concatenate([np.asarray(arr, np.float64),
                               rng.normal(5, 1, (extra_probes, 21))], 0)
        full = np.concatenate([full, rng.normal(5, 1, (len(probes), 1))], 1)
        df = pd.DataFrame(full[order], index=[probes[i] for i in order], columns=cols)
        df.to_csv(os.path.join(dir_path, name))
