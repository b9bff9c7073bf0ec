"""The MLL past BASELINE.json's sizes: G genes x 256 timepoints (N = 256 G; G = 256 gives
N = 65536, a 34 GB factor) on schedule 3 and on schedule 1 (two different kernel sets: the
factor chain on its own CUs against the look-ahead on every CU), and the C++ restatement
(oracle/lfm_cpu.cpp) on the same inputs on this host's CPU share — one JSON line.

    python scripts/scale_check.py [--genes 256] [--no-cpu] [--json out]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--genes", type=int, default=256)
    p.add_argument("--timepoints", type=int, default=256)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--json", default=None)
    a = p.parse_args()
    from dis_project_amd import _lib, configs, farm

    work = configs.grid_workload(f"synthetic_{a.genes}x{a.timepoints}_fp64", a.genes,
                                 a.timepoints, seed_params=2, seed_y=3)
    m = work.model
    out = {"N": work.n, "genes": a.genes, "timepoints": a.timepoints}
    for sched in ("3", "1"):
        os.environ["LFM_SCHED"] = sched  # read at context creation
        ctx = _lib.Context(0)
        ev = farm.ResidentEvaluator(ctx, work.data)
        try:
            v = float(ev([m])[0])  # first call: workspace allocation
            t0 = time.perf_counter()
            v2 = float(ev([m])[0])
            dt = time.perf_counter() - t0
            out[f"s{sched}"] = {"mll": v, "repeat_identical": v2 == v, "s": dt,
                                "tflops": work.n ** 3 / 3 / dt / 1e12,
                                "fallbacks": ctx.fallbacks}
        finally:
            ev.close()
            ctx.close()
        print(json.dumps(out), flush=True)
    os.environ.pop("LFM_SCHED", None)
    s3, s1 = out["s3"]["mll"], out["s1"]["mll"]
    out["s3_vs_s1_rel"] = abs(s3 - s1) / abs(s1)
    if not a.no_cpu:
        from oracle import lfm_cpu

        lfm_cpu.load()
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
        t0 = time.perf_counter()
        import threading

        stop = threading.Event()

        def beat():  # a line every 30 s: the CPU leg runs minutes at N = 65536
            while not stop.wait(30.0):
                print(f"cpu port running, {time.perf_counter() - t0:.0f} s", flush=True)

        threading.Thread(target=beat, daemon=True).start()
        cpu, info = lfm_cpu.mll(work.data.X, work.data.y, m.true_d, m.true_s, m.true_b, m.l,
                                m.obs_stddev, m.jitter, threads=min(threads, 32))
        out["cpu"] = {"mll": cpu, "fail": info["fail"], "threads": min(threads, 32),
                      "s": time.perf_counter() - t0, "gram_s": info["t_gram"],
                      "chol_s": info["t_chol"]}
        stop.set()
        out["s3_vs_cpu_rel"] = abs(s3 - cpu) / abs(cpu)
        out["s1_vs_cpu_rel"] = abs(s1 - cpu) / abs(cpu)
    line = json.dumps(out)
    print(line, flush=True)
    if a.json:
        with open(a.json, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
