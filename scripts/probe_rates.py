"""fp64 rate probes on random register operands (lfm_probe_rate): which = 2 / 3 the
16x16x4 / 4x4x4_4b MFMA with 8 independent accumulator chains per wave; 256-thread blocks,
1-4 workgroups per CU. Measured r02: 16x16x4 44-58 TF/s, 4x4x4_4b 69-74 TF/s (the trailing
update's instruction)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dis_project_amd import _lib  # noqa: E402

ctx = _lib.get_context(0)
names = {2: "16x16x4", 3: "4x4x4_4b"}
for rep in range(2):
    for which in (2, 3):
        for nblocks in (256, 512, 1024):
            tf = _lib.c_double()
            ctx.check(ctx.diag.lfm_probe_rate(ctx.handle, which, nblocks, 4000, _lib.ctypes.byref(tf)))
            print(json.dumps({"probe": names[which], "blocks": nblocks, "tflops": round(tf.value, 2)}),
                  flush=True)
