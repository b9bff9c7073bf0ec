"""Measure v_mfma_f64_16x16x4_f64 throughput on this device (sets the fp64 MFMA peak used
as the SYRK roofline denominator beside AMD's 78.6 TFLOP/s spec)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dis_project_amd import _lib  # noqa: E402

ctx = _lib.get_context(0)
res = []
for nblocks in (256, 512, 1024, 2048):
    tf, ms = _lib.c_double(), _lib.c_double()
    ctx.check(ctx.diag.lfm_probe_mfma_f64(ctx.handle, nblocks, 20000, _lib.ctypes.byref(tf),
                                         _lib.ctypes.byref(ms)))
    res.append({"blocks": nblocks, "waves_per_block": 4, "tflops": tf.value, "ms": ms.value})
    print(json.dumps(res[-1]), flush=True)
for nblocks in (256, 512, 2048):
    cyc, mhz = _lib.c_double(), _lib.c_double()
    ctx.check(ctx.diag.lfm_probe_mfma_f64_cycles(ctx.handle, nblocks, 20000, _lib.ctypes.byref(cyc),
                                                _lib.ctypes.byref(mhz)))
    print(json.dumps({"blocks": nblocks, "cycles_per_mfma_per_wave": cyc.value,
                      "shader_mhz": mhz.value}), flush=True)
for which, name in ((0, "valu_fma_f64"), (1, "mfma_f64_4x4x4_4b")):
    for nblocks in (1024, 2048, 4096):
        tf = _lib.c_double()
        ctx.check(ctx.diag.lfm_probe_rate(ctx.handle, which, nblocks, 20000, _lib.ctypes.byref(tf)))
        print(json.dumps({"probe": name, "blocks": nblocks, "tflops": tf.value}), flush=True)
