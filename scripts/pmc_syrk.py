"""The trailing-update kernel alone (lfm_probe_syrk: T = 126 tiles of 128, depth 512, C I/O,
random operands) for PMC passes: python scripts/pmc_syrk.py [reps]."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dis_project_amd import _lib  # noqa: E402

ctx = _lib.get_context(0)
us = _lib.c_double()
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
ctx.check(ctx.lib.lfm_probe_syrk(ctx.handle, 126, 512, 9, reps, _lib.ctypes.byref(us)))
T = 126
print(f"us/launch {us.value:.1f}  TF/s {T * (T + 1) / 2 * 128 * 128 * 512 * 2 / (us.value * 1e-6) / 1e12:.2f}")
