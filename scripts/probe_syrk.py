"""SYRK kernel alone: depth 128 vs 256, with and without the C tile HBM traffic."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dis_project_amd import _lib  # noqa: E402

ctx = _lib.get_context(0)
# cio: bit 0 = C tile I/O, bit 3 = random operands, bit 4 = the CU-masked bulk stream,
# bit 6 = the schedule-3 step kernel's rest role (the production unit), bit 5 = its C loads off
TS = [int(v) for v in os.environ.get("PROBE_T", "126,64,32").split(",")]
KDS = [int(v) for v in os.environ.get("PROBE_KD", "128,256,512").split(",")]
CIOS = [int(v) for v in os.environ.get("PROBE_CIO", "1,0,9").split(",")]
for T in TS:
    for kd in KDS:
        for cio in CIOS:
            us = _lib.c_double()
            ctx.check(ctx.diag.lfm_probe_syrk(ctx.handle, T, kd, cio, 5, _lib.ctypes.byref(us)))
            tiles = T * (T + 1) // 2  # 128-tiles (two 64-row slabs each)
            tf = tiles * 128 * 128 * kd * 2 / (us.value * 1e-6) / 1e12
            print(json.dumps({"T": T, "kd": kd, "c_io": cio, "us": round(us.value, 1),
                              "tflops_full_tiles": round(tf, 2)}), flush=True)
