"""Benchmark of the MI355X hot path: log-marginal-likelihood evaluations per second of the
SIM latent force model at N = 16384 (BASELINE.json configs[1]: 64 genes x 256 timepoints,
fp64, one MLL evaluation per step), plus the fp64 Cholesky rate.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c3|c5]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port P bench.py --gpus N --steps K --warmup W

One process per GPU. Workloads:
  c2 (default)  a step = one complete MLL evaluation on each rank (gram fill, Sigma assembly,
                blocked Cholesky with the residual row, logdet + quadratic form) on x / y
                resident in HBM, then the RCCL all-gather of the per-rank results (one fp64 slot
                per rank). Weak scaling: value = evaluations by all ranks / wall.
  c3            configs[2]: a step = the 32 random restarts of C2, statically partitioned over
                the ranks (farm.partition, ceil(32/W) slots per rank), one RCCL all-gather of
                the NaN-padded slots. Strong scaling: value = 32 x steps / wall. Each rank keeps
                --workers (3) evaluations in flight (farm.ConcurrentEvaluator).
  c5            configs[4]: a step = the 15 replicate x leave-one-gene-out problems (N = 28),
                each rank's share in one batched launch, then the all-gather. Strong scaling.
torch.distributed (gloo, CPU) is only the control plane: barrier, max-over-ranks timing and
shipping the RCCL unique id.

Rank 0 prints ONE JSON line; ``value`` = evaluations completed by all ranks / the slowest
rank's wall time of the K timed steps. Every result of the timed steps must be finite, and
(c2, one rank) the GPU MLL is checked against the C++ CPU restatement on the same inputs.
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
from dis_project_amd import configs, farm  # noqa: E402

FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X dense fp64 matrix, AMD spec (not in the local guide)
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
METRIC = "log-marginal-likelihood evals/sec + fp64 Cholesky GFLOP/s at N=16384"
PARITY_RTOL = 1e-9             # GPU vs C++ CPU restatement (north_star: 1e-5)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--workload", choices=["c2", "c3", "c5"], default="c2")
    p.add_argument("--genes", type=int, default=64)
    p.add_argument("--timepoints", type=int, default=256)
    p.add_argument("--restarts", type=int, default=32)
    p.add_argument("--workers", type=int, default=3,
                   help="c3: evaluations in flight per GPU (farm.ConcurrentEvaluator, schedule-1 "
                        "worker contexts); 1 = one schedule-3 context, one evaluation at a time")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=0)
    p.add_argument("--no-profile", action="store_true",
                   help="do not record per-kernel HIP events in the timed region")
    p.add_argument("--gather", choices=["rccl", "gloo"], default="rccl",
                   help="rehearsal only: gloo all-gather and ranks sharing the visible GPUs "
                        "(W ranks on fewer cards); the measured configuration is rccl")
    p.add_argument("--share-gpus", action="store_true",
                   help="rehearsal only: ranks share the visible GPUs (rank -> local %% count) "
                        "with the RCCL all-gather")
    return p.parse_args(argv)


def cpu_threads(a):
    t = a.cpu_threads or int(os.environ.get("OMP_NUM_THREADS", "0")) or \
        len(os.sched_getaffinity(0))
    return max(1, min(t, 64))


def cpu_baseline(work, threads, gpu_value):
    """The C++ / OpenMP CPU restatement (oracle/lfm_cpu.cpp, 'port') of ONE complete C2
    evaluation on the box's host cores, timed in full and not extrapolated: the reference's
    gram formula (every kernel branch, std::erf) on the real inputs, Sigma, a blocked fp64
    Cholesky of that Sigma, the forward solve and the log-density. Its MLL is also the
    independent full-size check of the GPU value."""
    from oracle import lfm_cpu

    m, d = work.model, work.data
    t0 = time.perf_counter()
    v, info = lfm_cpu.mll(d.X, d.y, m.true_d, m.true_s, m.true_b, m.l, m.obs_stddev, m.jitter,
                          negative=False, threads=threads)
    total = time.perf_counter() - t0
    n = work.n
    rel = abs(v - gpu_value) / abs(v)
    return {
        "value": 1.0 / total,
        "unit": "MLL evals/s",
        "cores": int(info["threads"]),
        "kind": "port",
        "sample": (f"oracle/lfm_cpu.cpp: one full C2 evaluation at N={n} on the real Sigma "
                   f"(gram {info['t_gram']:.2f} s, Cholesky {info['t_chol']:.2f} s, solve "
                   f"{info['t_solve']:.2f} s; {int(info['threads'])} OpenMP threads of "
                   f"{os.cpu_count()} host CPUs); timed once, not extrapolated"),
        "host_cpus": os.cpu_count(),
        "cholesky_gflops": (n**3 / 3.0) / info["t_chol"] / 1e9,
        "mll": v,
        "gpu_vs_cpu_rel": rel,
    }


def main(argv=None):
    a = parse(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus and world == 1:
        raise SystemExit("--gpus > 1 needs torch.distributed.run (one process per GPU)")
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)

    # one GPU per rank; the gloo rehearsal may put several ranks on one card
    dev = local % max(1, _lib.device_count()) if a.gather == "gloo" or a.share_gpus else local
    ctx = _lib.get_context(dev)
    lib, h = ctx.lib, ctx.handle

    # RCCL farm communicator (replicas-only exchange of per-rank results)
    gather = None
    if world > 1 and a.gather == "gloo":
        gather = farm.TorchGather(world)
    elif world > 1:
        obj = [farm.RcclGather.unique_id(ctx) if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        gather = farm.RcclGather(ctx, world, rank, obj[0])
    else:
        gather = lambda send: np.asarray(send, np.float64).copy()  # noqa: E731
    fm = farm.Farm(world, rank, gather)

    if a.workload == "c2":
        work = configs.grid_workload(f"synthetic_{a.genes}x{a.timepoints}_fp64", a.genes,
                                     a.timepoints, seed_params=2, seed_y=3)
        n = work.n
        ev = farm.ResidentEvaluator(ctx, work.data, negative=False)
        close = ev.close
        per_step = world

        def step():
            # one evaluation per rank, gathered: P = world problems, one slot each
            return fm.run(world, lambda idx: ev([work.model]))
    else:
        models, datasets = farm.workload(a.workload, a.genes, a.timepoints, a.restarts)
        n = datasets[0].n
        evaluate, close = farm.gpu_evaluator(ctx, datasets, negative=False,
                                           workers=a.workers)
        per_step = len(models)

        def step():
            return fm.run_problems(models, datasets, evaluate)

    results = []

    def barrier():
        ctx.check(lib.lfm_ctx_synchronize(h))
        if world > 1:
            dist.barrier()

    for _ in range(a.warmup):
        results.append(step())
    prof = not a.no_profile and a.workload == "c2"
    # HIP events around the priced kernels' launches of the FIRST timed step only: an event
    # record between two dependent launches widens the dispatch gap, ≈ 0.5 ms per evaluation
    # with all 65 step launches instrumented; one instrumented step of K costs 0.5 / K ms
    prof_steps = 1 if prof else 0
    if prof:
        ctx.profile(False)
        ctx.profile_reset()
    timed = []
    barrier()
    t0 = time.perf_counter()
    for s in range(a.steps):
        if s < prof_steps:
            ctx.profile(True, classes=["syrk", "gram_grid", "potrf", "syrk_side"])
        timed.append(step())
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
    # the exchange step alone (collective latency reported separately): the same
    # RCCL all-gather of this workload's NaN-padded slots, outside the timed region
    collective = None
    if world > 1:
        slots = max(farm.slots_per_rank(per_step, world), 1)
        lat = []
        for _ in range(25):
            barrier()
            t1 = time.perf_counter()
            gather(np.full(slots, np.nan))
            lat.append((time.perf_counter() - t1) * 1e6)
        lt = torch.tensor([float(np.median(lat[5:]))], dtype=torch.float64)
        dist.all_reduce(lt, op=dist.ReduceOp.MAX)
        collective = {"op": "ncclAllGather (RCCL)" if a.gather == "rccl" else "gloo all_gather",
                      "bytes_per_rank": 8 * slots,
                      "latency_us_median": float(lt.item())}
    # the timed region's results: all finite, every step the same values (same inputs)
    res = np.array(timed)
    if not np.all(np.isfinite(res)):
        raise SystemExit(f"non-finite MLL in the timed region: {res[~np.isfinite(res)][:4]}")
    if not np.all(res == res[0]):
        raise SystemExit("timed steps disagree (the same inputs gave different MLLs)")

    evals = per_step * a.steps
    value = evals / elapsed
    ms_per_step = elapsed / a.steps * 1e3
    chol_flops = n**3 / 3.0
    strong = a.workload != "c2"
    if a.workload == "c2":
        wl = (f"configs[1]: one MLL eval per rank, {a.genes} genes x {a.timepoints} timepoints, "
              f"N={n}, fp64")
    elif a.workload == "c3":
        wl = (f"configs[2]: {len(res[0])} random restarts of the {a.genes}x{a.timepoints} grid "
              f"(N={n}, fp64) per step, farmed over {world} GPU(s), "
              + (f"{a.workers} concurrent schedule-1 evaluations per GPU" if a.workers > 1
                 else "one schedule-3 evaluation at a time per GPU"))
    else:
        wl = (f"configs[4]: 3 replicates x 5 leave-one-gene-out ablations (N={n}) per step, "
              f"farmed over {world} GPU(s), one batched launch per rank")
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "MLL evals/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded numpy: D~U[.2,1], S~U[.5,1.5], B~U[.01,.1], y = B/D + "
                "0.5 N(0,1), t = linspace(0,12,T))",
        "config": {"workload": wl, "N": n,
                   "genes": a.genes if a.workload != "c5" else 4,
                   "timepoints": a.timepoints if a.workload != "c5" else 7,
                   "problems_per_step": per_step, "parallelism": f"replicas{world}",
                   "exchange": "RCCL all-gather of NaN-padded per-rank result slots"
                               if world > 1 else "none"},
        "mll_first": float(res[0][0]),
    }
    if collective:
        line["collective"] = collective
    if a.workload == "c2":
        line["cholesky_gflops_per_gpu"] = chol_flops / (ms_per_step * 1e-3) / 1e9
    if prof and rank == 0:
        syrk = stats.get("syrk", {})
        gram = stats.get("gram_grid", {})
        chain = stats.get("potrf", {})
        line["kernel_ms_per_eval"] = {k: round(v["total_ms"] / prof_steps, 4)
                                      for k, v in stats.items() if v["launches"]}
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
                "kernel": "step_kernel (fp64 MFMA trailing update + tall panel solve)",
                "bound": "mfma", "achieved": ach, "peak": FP64_MFMA_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": ach / FP64_MFMA_PEAK_TFLOPS, "traffic": traffic,
                "launches": syrk["launches"],
                "avg_launch_ms": syrk["total_ms"] / syrk["launches"],
                "flops_per_launch": syrk["flops"] / syrk["launches"],
                "flops_basis": "algorithmic: 2 W per updated lower element of the unpadded "
                               "augmented trailing matrix + W'^2 per solved row (sum over a "
                               "factorisation with the chain's share = N^3/3 + O(N^2))",
                "issued_flops_per_launch": syrk["issued_flops"] / syrk["launches"],
            }
            if chain.get("launches"):
                # the side stream's factor chain (its event span includes its device-side
                # input waits, so only its algorithmic share is reported)
                line["roofline"]["chain_flops_per_eval"] = chain["flops"] / prof_steps
            # the whole evaluation: the factorisation's N^3/3 over the evaluation's wall time
            # (the step kernel above runs on the 224 main CUs, the chain and the helper on 32)
            line["roofline"]["evaluation_tflops"] = chol_flops / (ms_per_step * 1e-3) / 1e12
            line["roofline"]["evaluation_frac"] = \
                line["roofline"]["evaluation_tflops"] / FP64_MFMA_PEAK_TFLOPS
            side = stats.get("syrk_side", {})
            if side.get("launches"):
                # the tail of long steps' trailing updates run on the 32 side CUs between
                # chains (same kernel; its flops are not in flops_per_launch above)
                line["roofline"]["side_helper"] = {
                    "launches_per_eval": side["launches"] / prof_steps,
                    "flops_per_eval": side["flops"] / prof_steps,
                    "avg_launch_ms": side["total_ms"] / side["launches"],
                    "achieved": side["flops"] / (side["total_ms"] * 1e-3) / 1e12,
                }
        if gram.get("launches"):
            gbs = gram["bytes"] / (gram["total_ms"] * 1e-3) / 1e9
            # fused (the schedule-3 default on this layout): the gram kernel writes only the
            # first block column and the next super-panel's diagonal block; the first trailing
            # update generates every other Sigma tile from the tables
            fused = gram["bytes"] < 0.5 * 8.0 * n * (n + 1) / 2 * prof_steps
            if fused:
                # no HBM roofline to claim: the fill is no longer a kernel of its own
                line["gram"] = {
                    "fused": True,
                    "kernel": "gram_region_kernel (first block column + next diagonal block; "
                              "the rest of Sigma is generated inside the first trailing update)",
                    "bytes_per_eval": gram["bytes"] / prof_steps,
                    "ms_per_eval": gram["total_ms"] / prof_steps,
                    "unfused_bytes": 8.0 * n * (n + 1) / 2,
                }
            else:
                line["gram_roofline"] = {
                    "kernel": "gram_grid_aligned_kernel (lower-triangle fp64 fill)",
                    "bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": gbs / HBM_PEAK_GBS,
                    "bytes_per_launch": gram["bytes"] / gram["launches"],
                    "avg_launch_ms": gram["total_ms"] / gram["launches"],
                }
    if rank == 0 and world == 1 and a.workload == "c2" and not a.no_cpu_baseline:
        cb = cpu_baseline(work, cpu_threads(a), float(res[0][0]))
        line["cpu_baseline"] = cb
        if not cb["gpu_vs_cpu_rel"] <= PARITY_RTOL:
            print(json.dumps(line), flush=True)
            raise SystemExit(f"GPU MLL {res[0][0]!r} differs from the CPU restatement "
                             f"{cb['mll']!r} by {cb['gpu_vs_cpu_rel']:.2e} relative")
    if rank == 0:
        print(json.dumps(line), flush=True)
    close()
    if world > 1:
        gather.close()
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
