"""Benchmark of the MI355X hot path: log-marginal-likelihood evaluations per second of the
SIM latent force model at N = 16384 (BASELINE.json configs[1]: 64 genes x 256 timepoints,
fp64, one MLL evaluation per step), plus the fp64 Cholesky rate.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One process per GPU. A step = one complete MLL evaluation on each rank (gram fill,
Sigma assembly, blocked Cholesky with the residual row, logdet + quadratic form), on
x / y already resident in HBM, followed by the farm's RCCL all-gather of the per-rank
results (a fixed-size fp64 slot per rank) — the replicas-only multi-GPU scheme of
SURVEY.md §8e. torch.distributed (gloo, CPU) is only the control plane: barrier,
max-over-ranks timing and shipping the RCCL unique id.

Rank 0 prints ONE JSON line. ``value`` = evaluations completed by all ranks / the slowest
rank's wall time of the K timed steps.
"""

from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch  # first: liblfm then binds to the HIP runtime torch loaded (see _lib.py)
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from dis_project_amd import _lib  # noqa: E402
from dis_project_amd import configs  # noqa: E402

FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X dense fp64 matrix, AMD spec (not in the local guide)
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--genes", type=int, default=64)
    p.add_argument("--timepoints", type=int, default=256)
    p.add_argument("--hyper", choices=["base", "restarts"], default="base",
                   help="base: every rank evaluates config 2's hyperparameters; restarts: "
                        "rank r, step s evaluates config-3 restart (s*W + r) %% 32")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=0)
    p.add_argument("--no-profile", action="store_true",
                   help="do not record per-kernel HIP events in the timed region")
    return p.parse_args()


def cpu_baseline(work, threads):
    """Oracle (numpy/scipy restatement, 'port') on the host cores, bounded sample:
    the full N x N Cholesky + solve at N = 16384 (scipy LAPACK potrf, what JAX-CPU calls)
    timed in full, the O(N^2) gram timed on a 1024-row slab and scaled by N / 1024."""
    from concurrent.futures import ThreadPoolExecutor

    import scipy.linalg

    from oracle import lfm_oracle as O

    m, d = work.model, work.data
    x = d.X
    n = x.shape[0]
    y = d.y.reshape(-1)
    D, S, B = m.true_d, m.true_s, m.true_b
    slab = 1024
    chunks = np.array_split(np.arange(slab), threads)
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(lambda ix: O.cross_covariance(x[ix], x, D, S, m.l, chunk=32), chunks))
    t_gram = (time.perf_counter() - t0) * (n / slab)
    # Sigma for the Cholesky: the device-identical structured gram would cost the full
    # t_gram again; the factorisation is what is timed here, on an SPD matrix of the
    # same size and conditioning class (noise-dominated: K + (jitter + sigma^2) I).
    rng = np.random.default_rng(0)
    A = rng.standard_normal((n, 64))
    Sig = (A @ A.T) / 64.0
    Sig[np.diag_indices(n)] += m.jitter + m.obs_stddev**2
    mx = O.mean_function(x, D, B, m.num_genes).reshape(-1)
    t1 = time.perf_counter()
    c = scipy.linalg.cho_factor(Sig, lower=True, overwrite_a=True, check_finite=False)
    logdet = 2.0 * np.sum(np.log(np.diag(c[0])))
    quad = (y - mx) @ scipy.linalg.cho_solve(c, y - mx, check_finite=False)
    _ = -0.5 * (n * math.log(2 * math.pi) + logdet + quad)
    t_chol = time.perf_counter() - t1
    total = t_gram + t_chol
    return {
        "value": 1.0 / total,
        "unit": "MLL evals/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"oracle/lfm_oracle.py at N={n}: gram on a {slab}-row slab x{n // slab} "
                   f"({t_gram:.2f} s est.), scipy cho_factor+cho_solve on a full {n}x{n} SPD "
                   f"({t_chol:.2f} s measured); {threads} threads"),
        "cholesky_gflops": (n**3 / 3.0) / t_chol / 1e9,
    }


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus and not (world == 1 and a.gpus == 1):
        if world == 1:
            raise SystemExit("--gpus > 1 needs torch.distributed.run (one process per GPU)")
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)

    ctx = _lib.Context(local)
    lib, h = ctx.lib, ctx.handle

    # RCCL farm (replicas-only exchange of per-rank results)
    if world > 1:
        uid = (_lib.ctypes.c_ubyte * 128)()
        if rank == 0:
            ctx.check(lib.lfm_farm_unique_id(h, uid))
        obj = [bytes(uid)]
        dist.broadcast_object_list(obj, src=0)
        uid = (_lib.ctypes.c_ubyte * 128).from_buffer_copy(obj[0])
        ctx.check(lib.lfm_farm_init(h, uid, world, rank))

    work = configs.grid_workload(f"synthetic_{a.genes}x{a.timepoints}_fp64", a.genes,
                                 a.timepoints, seed_params=2, seed_y=3)
    n = work.n
    x = np.ascontiguousarray(work.data.X)
    y = np.ascontiguousarray(work.data.y.reshape(-1))
    dx, dy = _lib.c_void_p(), _lib.c_void_p()
    ctx.check(lib.lfm_dev_alloc(h, x.nbytes, _lib.ctypes.byref(dx)))
    ctx.check(lib.lfm_dev_alloc(h, y.nbytes, _lib.ctypes.byref(dy)))
    ctx.check(lib.lfm_memcpy_h2d(h, dx, x.ctypes.data, x.nbytes))
    ctx.check(lib.lfm_memcpy_h2d(h, dy, y.ctypes.data, y.nbytes))
    # the dataset handle: x's layout is read back and analysed once (a Dataset is immutable),
    # not on every evaluation
    data = _lib.c_void_p()
    ctx.check(lib.lfm_data_create(h, dx, dy, n, _lib.ctypes.byref(data)))

    restarts = configs.c3_restarts(work, 32) if a.hyper == "restarts" else None
    hyps = {}

    def hyp_for(step):
        mdl = work.model if restarts is None else restarts[(step * world + rank) % 32]
        key = id(mdl)
        if key not in hyps:
            hyps[key] = mdl.hyp()
        return hyps[key]

    out = np.empty(1)
    gathered = np.empty(world)
    results = []

    def step(s):
        hp = hyp_for(s)
        rc = lib.lfm_mll_f64_data(h, data, hp.ref, 1, _lib.dptr(out))
        ctx.check(rc, allow_not_pd=True)
        if world > 1:
            ctx.check(lib.lfm_farm_allgather_f64(h, _lib.dptr(out), 1, _lib.dptr(gathered)))
        else:
            gathered[0] = out[0]
        results.append(gathered.copy())

    def barrier():
        ctx.check(lib.lfm_ctx_synchronize(h))
        if world > 1:
            dist.barrier()

    for s in range(a.warmup):
        step(s)
    prof = not a.no_profile
    # HIP events around the priced kernels' launches of the FIRST timed step only: an event
    # record between two dependent launches widens the dispatch gap, ≈ 0.5 ms per evaluation
    # with all 65 step launches instrumented; one instrumented step of K costs 0.5 / K ms
    prof_steps = 1 if prof else 0
    if prof:
        ctx.profile(False)
        ctx.profile_reset()
    barrier()
    t0 = time.perf_counter()
    for s in range(a.steps):
        if s < prof_steps:
            # only the two kernels the JSON line prices
            ctx.profile(True, classes=["syrk", "gram_grid"])
        step(a.warmup + s)
        if s + 1 == prof_steps:
            ctx.profile(False)
    barrier()
    elapsed = time.perf_counter() - t0
    if prof:
        stats = ctx.profile_read()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    evals = world * a.steps
    value = evals / elapsed
    ms_per_step = elapsed / a.steps * 1e3
    chol_flops = n**3 / 3.0
    line = {
        "metric": "log-marginal-likelihood evals/sec + fp64 Cholesky GFLOP/s at N=16384",
        "value": value,
        "unit": "MLL evals/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded numpy: D~U[.2,1], S~U[.5,1.5], B~U[.01,.1], y = B/D + "
                "0.5 N(0,1), t = linspace(0,12,T)); hyperparameters " + a.hyper,
        "config": {"workload": f"configs[1]: one MLL eval, {a.genes} genes x {a.timepoints} "
                               f"timepoints, N={n}, fp64", "N": n, "genes": a.genes,
                   "timepoints": a.timepoints, "parallelism": f"replicas{world}",
                   "exchange": "RCCL all-gather of per-rank results" if world > 1 else "none"},
        "cholesky_gflops_per_gpu": chol_flops / (ms_per_step * 1e-3) / 1e9,
        "mll_last": float(results[-1][0]) if results else None,
    }
    if prof and rank == 0:
        syrk = stats.get("syrk", {})
        gram = stats.get("gram_grid", {})
        per = {k: round(v["total_ms"] / prof_steps, 4) for k, v in stats.items()
               if v["launches"]}
        line["kernel_ms_per_eval"] = per
        if syrk.get("launches"):
            ach = syrk["flops"] / (syrk["total_ms"] * 1e-3) / 1e12
            traffic = None
            tf = os.path.join(ROOT, "profiles", "syrk_traffic.json")
            if os.path.exists(tf):
                try:
                    # PMC bytes per evaluation over this run's launches per evaluation
                    per_eval = json.load(open(tf)).get("hbm_bytes_per_eval")
                    traffic = per_eval / (syrk["launches"] / prof_steps) if per_eval else None
                except Exception:
                    traffic = None
            line["roofline"] = {
                "kernel": "step_kernel (fp64 MFMA trailing update + tall panel-solve GEMM)",
                "bound": "mfma", "achieved": ach, "peak": FP64_MFMA_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": ach / FP64_MFMA_PEAK_TFLOPS, "traffic": traffic,
                "launches": syrk["launches"],
                "avg_launch_ms": syrk["total_ms"] / syrk["launches"],
                "flops_per_launch": syrk["flops"] / syrk["launches"],
            }
        if gram.get("launches"):
            gbs = gram["bytes"] / (gram["total_ms"] * 1e-3) / 1e9
            line["gram_roofline"] = {
                "kernel": "gram_grid_kernel (lower-triangle fp64 fill)", "bound": "hbm",
                "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": gbs / HBM_PEAK_GBS,
                "bytes_per_launch": gram["bytes"] / gram["launches"],
                "avg_launch_ms": gram["total_ms"] / gram["launches"],
            }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        threads = a.cpu_threads or int(os.environ.get("OMP_NUM_THREADS", "0")) or \
            len(os.sched_getaffinity(0))
        threads = max(1, min(threads, 64))
        line["cpu_baseline"] = cpu_baseline(work, threads)
    if rank == 0:
        print(json.dumps(line), flush=True)
    lib.lfm_data_destroy(data)
    lib.lfm_dev_free(h, dx)
    lib.lfm_dev_free(h, dy)
    if world > 1:
        lib.lfm_farm_destroy(h)
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
