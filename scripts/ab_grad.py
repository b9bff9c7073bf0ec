"""Interleaved A/B of value_and_grad (lfm_mll_grad_f64) at N = 16384 across library builds:
each round runs every library in its own child process (scripts/grad_time.py's workload;
2 warm + 5 timed calls), rounds alternate the order. Usage:

    python scripts/ab_grad.py dis_project_amd/liblfm.so dis_project_amd/liblfm_x.so"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(variant):
    # a variant may carry environment settings after '@' (as scripts/ab_lib.py)
    lib, _, env = variant.partition("@")
    for kv in filter(None, env.split(",")):
        k, v = kv.split("=", 1)
        os.environ[k] = v
    os.environ["LFM_LIBRARY"] = lib
    sys.path.insert(0, ROOT)
    from dis_project_amd import CustomConjMLL, configs

    work = configs.grid_workload("grad", 64, 256, seed_params=2, seed_y=3)
    obj = CustomConjMLL(negative=True)
    for _ in range(2):
        obj.value_and_grad(work.model, work.data)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        v, g = obj.value_and_grad(work.model, work.data)
        ts.append((time.perf_counter() - t0) * 1e3)
    print(json.dumps({"lib": variant, "ms": ts, "value": v}))


def main():
    if sys.argv[1] == "--child":
        return child(sys.argv[2])
    libs = sys.argv[1:]
    rounds = int(os.environ.get("AB_ROUNDS", "3"))
    res = {lib: [] for lib in libs}
    for r in range(rounds):
        for lib in (libs if r % 2 == 0 else libs[::-1]):
            out = subprocess.run([sys.executable, __file__, "--child", lib], capture_output=True,
                                 text=True, timeout=300)
            if out.returncode:
                print(out.stderr[-2000:], file=sys.stderr)
                raise SystemExit(out.returncode)
            d = json.loads(out.stdout.strip().splitlines()[-1])
            res[lib] += d["ms"]
            print(f"round {r} {lib}: median {sorted(d['ms'])[2]:.3f} ms value {d['value']!r}",
                  flush=True)
    for lib in libs:
        v = sorted(res[lib])
        print(f"{lib}: median {v[len(v) // 2]:.3f} ms, min {v[0]:.3f} ms")


if __name__ == "__main__":
    main()
