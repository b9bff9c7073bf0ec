"""dis_project_amd — MI355X-native drop-in for the GPJax hot path of wejpurvis/DIS_project:
the SIM latent-force-model covariance (src/model.py) and its Cholesky-based log marginal
likelihood (src/objectives.py), on hand-written gfx950 HIP kernels behind a ctypes C-ABI
(``liblfm.so``, declared in ``include/lfm.h``).
"""

from ._lib import LfmError, device_count, get_context, load_library  # noqa: F401
from .dataset import Dataset, SyntheticP53Data, dataset_3d  # noqa: F401
from .distributions import GaussianDistribution  # noqa: F401
from .model import ExactLFM  # noqa: F401
from .objectives import CustomConjMLL  # noqa: F401

__all__ = [
    "CustomConjMLL",
    "Dataset",
    "ExactLFM",
    "GaussianDistribution",
    "LfmError",
    "SyntheticP53Data",
    "dataset_3d",
    "device_count",
    "get_context",
    "load_library",
]
