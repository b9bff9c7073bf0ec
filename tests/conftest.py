"""Test configuration.

Markers: ``gpu`` — needs an MI355X and the built liblfm.so (run with ``-m gpu``);
everything else runs on the CPU (``-m "not gpu"``).

torch (when installed) is imported first so that, in processes that also use
torch.distributed, liblfm binds to the HIP runtime torch already loaded
(see dis_project_amd/_lib.py).
"""

import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

try:  # noqa: SIM105
    import torch  # noqa: F401
except Exception:  # pragma: no cover
    pass

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU and liblfm.so")
    config.addinivalue_line("markers", "slow: long-running parity case")


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture
def golden():
    return load_golden
