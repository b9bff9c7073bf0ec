"""Ablation timing of the diagonal-block kernel phases (see lfm_probe_potrf)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dis_project_amd import _lib  # noqa: E402

ctx = _lib.get_context(0)
for mask in (0, 8, 1, 2, 4, 6, 7, 15):
    us = _lib.c_double()
    ctx.check(ctx.lib.lfm_probe_potrf(ctx.handle, mask, 50, _lib.ctypes.byref(us)))
    print(json.dumps({"mask": mask, "us": round(us.value, 2)}), flush=True)
