"""Interleaved A/B timing of liblfm builds (compile-time variants) at N = 16384: each round
runs every library in its own child process (`--child LIB`: 3 warm evaluations, then 10 timed
ones on the HBM-resident C2 dataset), rounds alternate the order, so box and thermal drift hit
every variant alike. Usage (libraries built in-tree, e.g. make OUT=../liblfm_x.so EXTRA=-D...):

    python scripts/ab_lib.py dis_project_amd/liblfm.so dis_project_amd/liblfm_ab0.so

A variant may carry context-creation environment settings after '@', comma-separated:
    python scripts/ab_lib.py dis_project_amd/liblfm.so dis_project_amd/liblfm.so@LFM_SIDE_CUS=16

Prints per library: median / min ms per evaluation over the rounds and the MLL."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(variant):
    lib, _, env = variant.partition("@")
    for kv in filter(None, env.split(",")):
        k, v = kv.split("=", 1)
        os.environ[k] = v
    os.environ["LFM_LIBRARY"] = lib
    sys.path.insert(0, ROOT)
    import numpy as np

    from dis_project_amd import _lib, configs, farm

    work = configs.c2()
    ev = farm.ResidentEvaluator(_lib.get_context(0), work.data)
    for _ in range(3):
        v = ev([work.model])
    ctx = _lib.get_context(0)
    ts = []
    for _ in range(10):
        t0 = time.perf_counter()
        v = ev([work.model])
        ctx.check(ctx.lib.lfm_ctx_synchronize(ctx.handle))
        ts.append((time.perf_counter() - t0) * 1e3)
    print(json.dumps({"lib": variant, "ms": ts, "mll": float(v[0])}))
    ev.close()


def main():
    if sys.argv[1] == "--child":
        return child(sys.argv[2])
    libs = sys.argv[1:]
    rounds = int(os.environ.get("AB_ROUNDS", "3"))
    res = {lib: [] for lib in libs}
    mll = {}
    for r in range(rounds):
        order = libs if r % 2 == 0 else libs[::-1]
        for lib in order:
            out = subprocess.run([sys.executable, __file__, "--child", lib], capture_output=True,
                                 text=True, timeout=300)
            if out.returncode:
                print(out.stderr[-2000:], file=sys.stderr)
                raise SystemExit(out.returncode)
            d = json.loads(out.stdout.strip().splitlines()[-1])
            res[lib] += d["ms"]
            mll[lib] = d["mll"]
            print(f"round {r} {lib}: median {sorted(d['ms'])[5]:.3f} ms", flush=True)
    for lib in libs:
        v = sorted(res[lib])
        print(f"{lib}: median {v[len(v) // 2]:.3f} ms, min {v[0]:.3f} ms, mll {mll[lib]!r}")


if __name__ == "__main__":
    main()
