"""Average device time of one rest unit of the step kernel in the isolated probe
(lfm_probe_syrk with bit 6, include/lfm_diag.h), from the step kernel's own stamps: compare with
step_timeline.py's `rest unit` column for the same trailing size inside a real evaluation.

    PROBE_T=35 PROBE_KD=128 PROBE_CIO=88,984 python scripts/unit_time.py"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from dis_project_amd import _lib  # noqa: E402

REPS = 5


def main():
    ctx = _lib.Context(0)
    for T in [int(v) for v in os.environ.get("PROBE_T", "35").split(",")]:
        for kd in [int(v) for v in os.environ.get("PROBE_KD", "128").split(",")]:
            for cio in [int(v) for v in os.environ.get("PROBE_CIO", "88,984").split(",")]:
                ctx.check(ctx.diag.lfm_debug_stamps(ctx.handle, 1, None, 0))
                us = ctypes.c_double(0)
                ctx.check(ctx.diag.lfm_probe_syrk(ctx.handle, T, kd, cio, REPS, ctypes.byref(us)))
                buf = (ctypes.c_ulonglong * (256 * 24))()
                ctx.check(ctx.diag.lfm_debug_stamps(ctx.handle, 0, buf, 256 * 24))
                sp = np.frombuffer(buf, dtype=np.uint64)[256 * 16:].reshape(256, 8)
                nr = (T - 1) * T if cio & 128 else T * (T + 1)
                unit = float(sp[0][5]) * 0.01 / ((REPS + 1) * nr)
                mhz = float(sp[0][4]) / float(sp[0][5]) * 100.0 if sp[0][5] else 0.0
                print(json.dumps({"T": T, "kd": kd, "c_io": cio, "us": round(us.value, 1),
                                  "rest_unit_us": round(unit, 2), "clock_mhz": round(mhz)}),
                      flush=True)


if __name__ == "__main__":
    main()
