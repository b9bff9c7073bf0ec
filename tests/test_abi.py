"""CPU checks of the drop-in boundary: liblfm.so loads, exports exactly what
include/lfm.h declares, and fails loudly (no CPU fallback) without a GPU; the diagnostics of
include/lfm_diag.h live in liblfm_diag.so and nowhere in the product library."""

import ctypes
import os
import re

import numpy as np
import pytest

from dis_project_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions(name="lfm.h"):
    src = open(os.path.join(ROOT, "include", name)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(lfm_[a-z0-9_]+)\s*\(", src)))


def test_library_builds_and_loads():
    lib = _lib.load_library()
    assert lib.lfm_abi_version() == _lib.ABI_VERSION == 5


@pytest.mark.parametrize("header,sigs", [("lfm.h", "PRODUCT_SIGNATURES"),
                                         ("lfm_diag.h", "DIAG_SIGNATURES")])
def test_every_header_symbol_is_exported_and_bound(header, sigs):
    """lfm.h declares the product ABI only; the probes and stamps live in lfm_diag.h, exported
    by liblfm_diag.so."""
    lib = _lib.load_library() if header == "lfm.h" else _lib.load_diag()
    declared = header_functions(header)
    bound = {name for name, _, _ in getattr(_lib, sigs)}
    for name in declared:
        assert hasattr(lib, name), f"{name} declared in include/{header} but not exported"
        assert name in bound, f"{name} has no ctypes signature in _lib.{sigs}"
    assert bound == set(declared)
    if header == "lfm.h":
        assert len(declared) >= 28
        assert not [d for d in declared if "probe" in d or "debug" in d]


def test_exports_are_c_symbols():
    out = os.popen(f"nm -D --defined-only {_lib.LIB_PATH}").read()
    for name in header_functions():
        assert re.search(rf"\bT {name}$", out, re.M), f"{name} is not an extern \"C\" symbol"
    diag = os.popen(f"nm -D --defined-only {_lib.DIAG_PATH}").read()
    for name in header_functions("lfm_diag.h"):
        assert re.search(rf"\bT {name}$", diag, re.M), f"{name} is not exported by liblfm_diag.so"
        # the product library carries no diagnostic entry point (and no probe kernel)
        assert not re.search(rf"\b{name}$", out, re.M), f"{name} is in the product liblfm.so"
    for kernel in ("rsq_probe_kernel", "fill_hash_kernel", "mfma_rate_kernel"):
        assert kernel not in out and kernel not in os.popen(f"nm {_lib.LIB_PATH}").read()


def test_struct_layouts_match_header():
    assert ctypes.sizeof(_lib.LfmHyp) == 7 * 8
    assert ctypes.sizeof(_lib.LfmProblem) == 3 * 8 + 7 * 8
    assert ctypes.sizeof(_lib.LfmKstat) == 32 + 8 * 5
    assert ctypes.sizeof(_lib.LfmAdam) == 5 * 8 + 8 + 8  # int fix_params padded to 8


def test_no_measured_null_variants_in_the_product():
    """The A/B variants round 4 measured inside the noise (32-row w = 1 units, rest-unit
    stealing across XCDs) are not compiled into liblfm.so."""
    syms = os.popen(f"nm {_lib.LIB_PATH}").read()
    for name in ("step_kernel32", "rest_claim", "steal"):
        assert name not in syms, name
    src = open(os.path.join(ROOT, "dis_project_amd", "csrc", "lfm_chol.hip")).read()
    assert "LFM_TR32" not in src and "LFM_STEAL" not in src


def test_error_codes_match_header():
    src = open(os.path.join(ROOT, "include", "lfm.h")).read()
    codes = dict((k, int(v)) for k, v in re.findall(r"\b(LFM_E_[A-Z_]+|LFM_OK) = (\d+)", src))
    for k, v in codes.items():
        assert getattr(_lib, k) == v, k
    assert codes["LFM_E_TIMEOUT"] == 7


def test_timeout_is_never_swallowed():
    """check(allow_not_pd=True) maps only LFM_E_NOT_PD to a NaN result; a device-side
    timeout raises (a stalled hand-off is not a property of the input)."""

    class Fake(_lib.Context):
        def __init__(self):
            self.lib = _lib.load_library()
            self.handle = None

    ctx = Fake()
    assert ctx.check(_lib.LFM_E_NOT_PD, allow_not_pd=True) == _lib.LFM_E_NOT_PD
    with pytest.raises(_lib.LfmError) as ei:
        ctx.check(_lib.LFM_E_TIMEOUT, allow_not_pd=True)
    assert ei.value.code == _lib.LFM_E_TIMEOUT


def test_contexts_are_per_thread(monkeypatch):
    """get_context caches one context per (thread, device): threads never share one."""
    import threading

    made = []

    class Fake:
        def __init__(self, dev):
            made.append((threading.get_ident(), dev))

    monkeypatch.setattr(_lib, "Context", Fake)
    monkeypatch.setattr(_lib, "_tls", threading.local())
    a = _lib.get_context(0)
    assert _lib.get_context(0) is a
    other = []
    t = threading.Thread(target=lambda: other.append(_lib.get_context(0)))
    t.start()
    t.join()
    assert other[0] is not a and len(made) == 2


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
