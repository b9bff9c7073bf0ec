"""CPU checks of the drop-in boundary: liblfm.so loads, exports exactly what
include/lfm.h declares, and fails loudly (no CPU fallback) without a GPU."""

import ctypes
import os
import re

import numpy as np
import pytest

from dis_project_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "lfm.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(lfm_[a-z0-9_]+)\s*\(", src)))


def test_library_builds_and_loads():
    lib = _lib.load_library()
    assert lib.lfm_abi_version() == 1


def test_every_header_symbol_is_exported_and_bound():
    lib = _lib.load_library()
    declared = header_functions()
    assert len(declared) >= 30
    bound = {name for name, _, _ in _lib.SIGNATURES}
    for name in declared:
        assert hasattr(lib, name), f"{name} declared in include/lfm.h but not exported"
        assert name in bound, f"{name} has no ctypes signature in _lib.SIGNATURES"
    assert bound == set(declared)


def test_exports_are_c_symbols():
    out = os.popen(f"nm -D --defined-only {_lib.LIB_PATH}").read()
    for name in header_functions():
        assert re.search(rf"\bT {name}$", out, re.M), f"{name} is not an extern \"C\" symbol"


def test_struct_layouts_match_header():
    assert ctypes.sizeof(_lib.LfmHyp) == 7 * 8
    assert ctypes.sizeof(_lib.LfmProblem) == 3 * 8 + 7 * 8
    assert ctypes.sizeof(_lib.LfmKstat) == 32 + 8 * 4


def test_null_ctx_is_rejected():
    lib = _lib.load_library()
    assert lib.lfm_ctx_synchronize(None) == _lib.LFM_E_ARG
    assert lib.lfm_mll_f64(None, None, None, 0, None, 0, None) == _lib.LFM_E_ARG
    assert lib.lfm_ctx_create(0, None) == _lib.LFM_E_ARG


@pytest.mark.skipif(_lib.device_count() > 0, reason="host has a GPU")
def test_no_gpu_fails_loudly():
    with pytest.raises(_lib.LfmError):
        _lib.Context(0)
    from dis_project_amd import CustomConjMLL, Dataset, ExactLFM

    x = np.stack((np.linspace(0, 12, 7), np.zeros(7), np.ones(7)), -1)
    with pytest.raises(_lib.LfmError):
        CustomConjMLL(negative=True)(ExactLFM(num_genes=1, device=0), Dataset(x, np.zeros(7)))


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(_lib.LfmError):
        _lib.load_library(str(tmp_path / "nope.so"))
