"""Panel-solve kernel variants alone at tail-relevant and full row counts."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dis_project_amd import _lib  # noqa: E402

ctx = _lib.get_context(0)
variants = [int(v) for v in sys.argv[1:]] or [2, 3]
for rows in (512, 1024, 2048, 4096, 8192, 16384):
    for v in variants:
        us = _lib.c_double()
        ctx.check(ctx.lib.lfm_probe_trsm(ctx.handle, v, rows, 20, _lib.ctypes.byref(us)))
        print(json.dumps({"variant": v, "rows": rows, "us": round(us.value, 2)}), flush=True)
