"""C3 throughput with K concurrent evaluation workers on one GPU: K host threads, each with its
own context (its own streams and workspace), splitting the 32 restarts of C3 between them.
ctypes releases the GIL during the library calls, so the K evaluations run concurrently on the
device.

    python scripts/concurrency_probe.py K [rounds]

Environment toggles (to tell apart what the bench process does differently):
  PROBE_TORCH=1   import torch first (bench.py does: liblfm then binds torch's HIP runtime)
  PROBE_IDLE=n    create n idle contexts before the workers (bench.py's main context)
  PROBE_SCHED=s   worker schedule set through lfm_ctx_set_schedule (default 1)
  PROBE_FARM=1    farm.ConcurrentEvaluator (dynamic pulling, thread pool) instead of a static
                  split over fresh threads"""
import os
import sys
import threading
import time

if os.environ.get("PROBE_TORCH") == "1":
    import torch  # noqa: F401

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from dis_project_amd import _lib, farm  # noqa: E402


def main():
    K = int(sys.argv[1])
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    sched = int(os.environ.get("PROBE_SCHED", "1"))
    tag = " ".join(f"{k}={os.environ[k]}" for k in
                   ("PROBE_TORCH", "PROBE_IDLE", "PROBE_SCHED", "PROBE_FARM", "GPU_MAX_HW_QUEUES")
                   if k in os.environ)
    models, datasets = farm.workload("c3", 64, 256, 32)
    idle = [_lib.Context(0) for _ in range(int(os.environ.get("PROBE_IDLE", "0")))]
    out = np.empty(len(models))
    if os.environ.get("PROBE_FARM") == "1":
        main_ctx = idle[0] if idle else _lib.Context(0)
        ev = farm.ConcurrentEvaluator(main_ctx, datasets[0], workers=K)

        def run():
            out[:] = ev(models)

        close = ev.close
    else:
        ctxs = [_lib.Context(0) for _ in range(K)]
        for c in ctxs:
            c.schedule = sched
        evs = [farm.ResidentEvaluator(c, datasets[0]) for c in ctxs]
        parts = [list(range(k, len(models), K)) for k in range(K)]

        def work(k):
            idx = parts[k]
            out[idx] = evs[k]([models[i] for i in idx])

        def run():
            th = [threading.Thread(target=work, args=(k,)) for k in range(K)]
            for t in th:
                t.start()
            for t in th:
                t.join()

        def close():
            for e in evs:
                e.close()

    for r in range(rounds + 1):
        t0 = time.perf_counter()
        run()
        dt = time.perf_counter() - t0
        if r > 0:
            print(f"K={K} sched={sched} {tag} round {r}: {len(models) / dt:.2f} evals/s "
                  f"({dt * 1e3:.1f} ms), finite {int(np.isfinite(out).sum())}/{len(out)}",
                  flush=True)
    close()


if __name__ == "__main__":
    main()
