"""The trailing-update kernel alone for PMC passes (lfm_probe_syrk, include/lfm_diag.h):
T tiles of 128, depth KD, C I/O, random operands; PMC_CIO selects the variant (88: the step
kernel's rest role on the bulk CUs, the production unit; 9: syrk_kernel's 64 x 128 units).

    PMC_T=127 PMC_KD=640 PMC_CIO=88 python scripts/pmc_syrk.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dis_project_amd import _lib  # noqa: E402

ctx = _lib.get_context(0)
us = _lib.c_double()
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
T = int(os.environ.get("PMC_T", "126"))
kd = int(os.environ.get("PMC_KD", "512"))
cio = int(os.environ.get("PMC_CIO", "9"))
ctx.check(ctx.diag.lfm_probe_syrk(ctx.handle, T, kd, cio, reps, _lib.ctypes.byref(us)))
print(f"T {T} kd {kd} cio {cio}: us/launch {us.value:.1f}  TF/s "
      f"{T * (T + 1) / 2 * 128 * 128 * kd * 2 / (us.value * 1e-6) / 1e12:.2f}")
