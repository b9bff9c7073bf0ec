"""Benchmark of the MI355X hot path: log-marginal-likelihood evaluations per second of the
SIM latent force model at N = 16384 (BASELINE.json configs[1]: 64 genes x 256 timepoints,
fp64, one MLL evaluation per step), plus the fp64 Cholesky rate.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c3|c4|c5]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port P bench.py --gpus N --steps K --warmup W

One process per GPU. Started as a plain command with --gpus N > 1 (no WORLD_SIZE in the
environment), this process is only a launcher: it never touches a GPU, starts N fresh rank
processes of itself with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set,
forwards their output and exits with the first non-zero exit code (the other ranks are then
stopped). Workloads; the default is c2 on one GPU and c3 on several:
  c2  configs[1]: a step = one complete MLL evaluation on each rank (gram fill, Sigma
      assembly, blocked Cholesky with the residual row, logdet + quadratic form) on x / y
      resident in HBM, then the RCCL all-gather of the per-rank results (one fp64 slot per
      rank). Weak scaling: value = evaluations by all ranks / wall.
  c3  configs[2]: a step = the 32 random restarts of C2, statically partitioned over the
      ranks (farm.partition, ceil(32/W) slots per rank), one RCCL all-gather of the NaN-padded
      slots. Strong scaling: value = 32 x steps / wall. Each rank keeps --workers evaluations
      in flight (farm.ConcurrentEvaluator; default: farm.choose_workers for its share).
  c4  configs[3]: a step = one fp32 lower-triangle gram fill at N = 65536 (256 genes x 256
      timepoints, 8.6 GB written) into a 17.2 GB device buffer; the HBM roofline of the fill.
      One GPU (replicas at N > 1: every rank fills its own; weak scaling).
  c5  configs[4]: a step = the 15 replicate x leave-one-gene-out problems (N = 28) at --rounds
      R hyperparameter rounds per rank (default 1 on one GPU: configs[4]'s own step; 16 on
      several), each rank's R x 15 in one batched launch, then one all-gather. Weak scaling
      over rounds (a round is one hyperparameter set of each of the 15 problems).
  c5fit  configs[4]'s actual workflow (notebook.py:55-75): a step = JaxTrainer.fit of the 15
      problems, 150 steps of adam(0.01) on CustomConjMLL(negative=True) each, in ONE launch
      (lfm_batch_fit_f64: every problem's value_and_grad + Adam loop inside one workgroup).
      value = problem training steps / s (15 x 150 per step). Several GPUs: the 15 fits
      partitioned (farm.partition), one all-gather of their final raw parameters and loss
      histories (trainer.FarmTrainer's exchange). Strong scaling.
torch.distributed (gloo, CPU) is only the control plane: barrier, max-over-ranks timing and
shipping the RCCL unique id.

Rank 0 prints ONE JSON line; ``value`` = work completed by all ranks / the slowest rank's
wall time of the K timed steps. Every result of the timed steps must be finite and identical
across steps, and (one rank) the GPU values are checked against the C++ CPU restatement on
the same inputs in the cpu_baseline leg.
"""

from __future__ import annotations

import argparse
import datetime
import json
import os
import signal
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# torch and liblfm are imported by the rank path only (_load): the launcher of `--gpus N` must
# stay free of the HIP runtime — importing torch maps libamdhip64, and a process that has
# initialised HIP must not start GPU processes (tests/test_bench_launcher.py checks both)
torch = dist = _lib = configs = farm = None


def _load():
    """Import torch (first: liblfm then binds to the HIP runtime torch loaded, see _lib.py),
    torch.distributed and the product package into this module's namespace."""
    global torch, dist, _lib, configs, farm
    if _lib is not None:
        return
    import torch as _torch
    import torch.distributed as _dist

    from dis_project_amd import _lib as _l
    from dis_project_amd import configs as _c
    from dis_project_amd import farm as _f

    torch, dist, _lib, configs, farm = _torch, _dist, _l, _c, _f

FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X dense fp64 matrix, AMD spec (not in the local guide)
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
METRIC = "log-marginal-likelihood evals/sec + fp64 Cholesky GFLOP/s at N=16384"
PARITY_RTOL = 1e-9             # GPU vs C++ CPU restatement (north_star: 1e-5)
# c5 at W > 1: hyperparameter rounds of the 15 problems per rank per step (240 workgroups: one
# per CU, one launch and one exchange per step)
C5_ROUNDS_MULTI = 16
EPS64 = np.finfo(np.float64).eps


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--workload", choices=["c2", "c3", "c4", "c5", "c5fit"], default=None,
                   help="default: c2 on one GPU, c3 (configs[2], the multi-GPU config) on several")
    p.add_argument("--genes", type=int, default=None)
    p.add_argument("--timepoints", type=int, default=256)
    p.add_argument("--restarts", type=int, default=32)
    p.add_argument("--workers", type=int, default=0,
                   help="c3: evaluations in flight per GPU (farm.ConcurrentEvaluator, schedule-1 "
                        "worker contexts); 1 = one schedule-3 context, one evaluation at a time; "
                        "0 (default) = farm.choose_workers for the rank's share")
    p.add_argument("--rounds", type=int, default=0,
                   help="c5: hyperparameter rounds of the 15 problems per rank per step (weak "
                        "scaling over rounds, one launch and one exchange per step); 0 (default) "
                        "= 1 on one GPU (configs[4]'s step), 16 on several")
    p.add_argument("--fit-iters", type=int, default=150,
                   help="c5fit: Adam steps per fit (notebook.py:64 / main.py:54: 150)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=0)
    p.add_argument("--no-profile", action="store_true",
                   help="do not record per-kernel HIP events in the timed region")
    p.add_argument("--gather", choices=["rccl", "gloo"], default="rccl",
                   help="rehearsal only: gloo all-gather and ranks sharing the visible GPUs "
                        "(W ranks on fewer cards); the measured configuration is rccl")
    p.add_argument("--share-gpus", action="store_true",
                   help="rehearsal only: ranks share the visible GPUs (rank -> local %% count)")
    p.add_argument("--require-rccl", dest="require_rccl", action="store_true", default=None,
                   help="an RCCL communicator failure on any rank ends the run (non-zero exit, "
                        "the cause on stderr) instead of exchanging over gloo; the default "
                        "unless rehearsing (--share-gpus / --gather gloo)")
    p.add_argument("--no-require-rccl", dest="require_rccl", action="store_false")
    a = p.parse_args(argv)
    if a.require_rccl is None:
        a.require_rccl = not (a.share_gpus or a.gather == "gloo")
    if a.workload is None:
        a.workload = "c2" if a.gpus == 1 else "c3"
    if a.genes is None:
        a.genes = 256 if a.workload == "c4" else 64
    if a.rounds <= 0:
        a.rounds = 1 if a.gpus == 1 else C5_ROUNDS_MULTI
    return a


# ------------------------------------------------------------------ launcher
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


KFD_TOPOLOGY = "/sys/class/kfd/kfd/topology/nodes"


class GpuCountError(RuntimeError):
    """The launcher could not count the GPUs without the HIP runtime."""


def _kfd_gpus(root: str) -> list:
    """The GPU agents of the KFD topology (sysfs), in node order — the order the ROCm runtime
    enumerates them: a node with gpu_id != 0 whose DRM render node (/dev/dri/renderD<minor>,
    from its properties) exists and is readable and writable by this process (a container sees
    the render nodes of its own cards only). Returns [{"node", "unique_id"}]. Reads text files
    only: no HIP, no /dev/kfd."""
    try:
        nodes = sorted((int(d) for d in os.listdir(root) if d.isdigit()))
    except OSError as e:
        raise GpuCountError(f"cannot read the KFD topology at {root}: {e}") from None
    dri = os.environ.get("LFM_DRI_DIR", "/dev/dri")
    out = []
    for k in nodes:
        base = os.path.join(root, str(k))
        try:
            with open(os.path.join(base, "gpu_id")) as f:
                gpu_id = int(f.read().strip() or "0")
        except (OSError, ValueError):
            continue
        if gpu_id == 0:  # a CPU agent
            continue
        props = {}
        try:
            with open(os.path.join(base, "properties")) as f:
                for line in f:
                    kv = line.split()
                    if len(kv) == 2:
                        props[kv[0]] = kv[1]
        except OSError:
            pass
        minor = props.get("drm_render_minor")
        if minor is not None and int(minor) > 0:
            dev = os.path.join(dri, f"renderD{int(minor)}")
            if not os.access(dev, os.R_OK | os.W_OK):
                continue
        out.append({"node": k, "unique_id": int(props.get("unique_id", "0") or 0)})
    return out


def _apply_visible(agents: list, spec: str | None) -> list:
    """Narrow a device list by a *_VISIBLE_DEVICES value as the runtime does: comma-separated
    indices into the list (or GPU-<hex unique id>), parsing stops at the first entry that names
    no device; unset keeps the list, empty hides every device."""
    if spec is None:
        return agents
    out = []
    for tok in (t.strip() for t in spec.split(",")):
        if not tok:
            break
        if tok.upper().startswith("GPU-"):
            try:
                uid = int(tok[4:], 16)
            except ValueError:
                break
            hit = [a for a in agents if a.get("unique_id") == uid]
            if not hit:
                break
            out.append(hit[0])
            continue
        try:
            i = int(tok)
        except ValueError:
            break
        if not 0 <= i < len(agents):
            break
        out.append(agents[i])
    return out


def visible_gpus() -> int:
    """GPUs a rank process of this launcher could use, counted WITHOUT the HIP runtime (the
    launcher then starts the rank processes; a parent that had initialised HIP must not): the
    KFD topology's GPU agents with an accessible render node (``LFM_KFD_TOPOLOGY`` overrides
    the sysfs path, for tests), narrowed by ROCR_VISIBLE_DEVICES, then HIP_VISIBLE_DEVICES (or
    CUDA_VISIBLE_DEVICES). Raises GpuCountError if the topology cannot be read — the launcher
    then refuses rather than fall back to a count that initialises HIP."""
    agents = _kfd_gpus(os.environ.get("LFM_KFD_TOPOLOGY", KFD_TOPOLOGY))
    agents = _apply_visible(agents, os.environ.get("ROCR_VISIBLE_DEVICES"))
    hip = os.environ.get("HIP_VISIBLE_DEVICES")
    if hip is None:
        hip = os.environ.get("CUDA_VISIBLE_DEVICES")
    return len(_apply_visible(agents, hip))


def self_launch(a, argv, script=None) -> int:
    """Start a.gpus rank processes of this script (never touching a GPU here) and wait for
    them. Returns the first non-zero exit code (the other ranks are then stopped), else 0."""
    n = a.gpus
    if n < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        return 2
    if not (a.share_gpus or a.gather == "gloo"):
        try:
            vis = visible_gpus()
        except GpuCountError as e:
            print(f"bench.py: {e}; refusing to start {n} rank processes (the launcher never "
                  "initialises HIP to count GPUs; run under torch.distributed.run, or rehearse "
                  "with --share-gpus --gather gloo)", file=sys.stderr)
            return 3
        if vis < n:
            print(f"bench.py: --gpus {n} requested but only {vis} GPU(s) are visible "
                  "(rehearsal on fewer cards: --share-gpus --gather gloo)", file=sys.stderr)
            return 3
    port = _free_port()
    script = script or os.path.abspath(__file__)
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", script] + list(argv), env=env))
    rc = 0
    try:
        while procs:
            for p in list(procs):
                code = p.poll()
                if code is None:
                    continue
                procs.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    print(f"bench.py: rank process {p.pid} exited with {code}; stopping the "
                          "others", file=sys.stderr)
                    _stop(procs)
            time.sleep(0.05)
    except KeyboardInterrupt:
        _stop(procs)
        raise
    return rc


def _stop(procs, grace=30.0):
    for p in procs:
        if p.poll() is None:
            p.send_signal(signal.SIGTERM)
    t_end = time.monotonic() + grace
    for p in procs:
        try:
            p.wait(timeout=max(0.1, t_end - time.monotonic()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()


# ------------------------------------------------------------- CPU baselines
def cpu_threads(a):
    return max(1, a.cpu_threads or int(os.environ.get("OMP_NUM_THREADS", "0")) or
               len(os.sched_getaffinity(0)))


def cpu_baseline_c2(work, threads, gpu_value):
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
        "gpu_vs_cpu_rel": abs(v - gpu_value) / abs(v),
    }


def cpu_baseline_c3(models, data, threads, gpu_values):
    """C3 on the CPU: ONE full evaluation of restart 0 (the C++ restatement, all allowed cores)
    timed and extrapolated to the 32 restarts (every restart is the same N = 16384 work);
    its MLL checks the GPU farm's restart-0 value."""
    from oracle import lfm_cpu

    m = models[0]
    t0 = time.perf_counter()
    v, info = lfm_cpu.mll(data.X, data.y, m.true_d, m.true_s, m.true_b, m.l, m.obs_stddev,
                          m.jitter, negative=False, threads=threads)
    t = time.perf_counter() - t0
    P = len(models)
    return {
        "value": 1.0 / t,
        "unit": "MLL evals/s",
        "cores": int(info["threads"]),
        "kind": "port",
        "sample": (f"oracle/lfm_cpu.cpp: one full evaluation of restart 0 at N={data.n} "
                   f"({t:.2f} s on {int(info['threads'])} OpenMP threads of {os.cpu_count()} "
                   f"host CPUs), extrapolated: {P} restarts x {t:.2f} s = {P * t:.1f} s per step"),
        "extrapolated": True,
        "seconds_per_step": P * t,
        "host_cpus": os.cpu_count(),
        "mll": v,
        "gpu_vs_cpu_rel": abs(v - gpu_values[0]) / abs(v),
    }


def cpu_baseline_c5(models, datasets, gpu_values, threads, min_seconds=2.0):
    """C5 on the CPU: the 15 problems evaluated sequentially on ONE core by the C++
    restatement, timed in full and repeated until min_seconds have passed (a step is 15
    evaluations of microseconds each); every value checks the GPU batch's."""
    from oracle import lfm_cpu

    vals, rounds = [], 0
    t0 = time.perf_counter()
    while True:
        vals = [lfm_cpu.mll(d.X, d.y, m.true_d, m.true_s, m.true_b, m.l, m.obs_stddev,
                            m.jitter, negative=False, threads=1)[0]
                for m, d in zip(models, datasets)]
        rounds += 1
        if time.perf_counter() - t0 >= min_seconds:
            break
    t = time.perf_counter() - t0
    ref = np.asarray(vals)
    rel = np.abs(ref - np.asarray(gpu_values)) / np.abs(ref)
    # the same problems across the box's CPU share (cpu_threads: OMP_NUM_THREADS, else the
    # process's affinity): one problem per OpenMP thread at a time (oracle/lfm_cpu.cpp
    # lfm_cpu_mll_batch), many rounds in one parallel loop
    thr = threads
    genes = [m.num_genes for m in models]
    hyp = np.concatenate([np.concatenate([m.true_d, m.true_s, m.true_b]) for m in models] +
                         [np.array([[m.l, m.obs_stddev, m.jitter] for m in models]).reshape(-1)])
    xs, ys = [d.X for d in datasets], [d.y for d in datasets]
    reps, tt = 64, 0.0
    while True:
        t1 = time.perf_counter()
        got = lfm_cpu.mll_batch(xs, ys, genes, hyp, threads=thr, reps=reps)
        tt = time.perf_counter() - t1
        if tt >= min_seconds or reps >= 1 << 24:
            break
        reps *= max(2, min(16, int(min_seconds / max(tt, 1e-3)) + 1))
    if not np.array_equal(got, ref):
        raise SystemExit("the threaded CPU baseline disagrees with the sequential one")
    return {
        "value": rounds * len(models) / t,
        "unit": "MLL evals/s",
        "cores": 1,
        "kind": "port",
        "sample": (f"oracle/lfm_cpu.cpp: the {len(models)} problems (N={datasets[0].n}) "
                   f"sequentially on ONE core, {rounds} full rounds in {t:.2f} s; "
                   "timed in full, not extrapolated"),
        "host_cpus": os.cpu_count(),
        "gpu_vs_cpu_rel": float(rel.max()),
        "threads": {
            "value": reps * len(models) / tt,
            "unit": "MLL evals/s",
            "cores": thr,
            "sample": (f"oracle/lfm_cpu.cpp lfm_cpu_mll_batch: {reps} rounds of the "
                       f"{len(models)} problems in one OpenMP loop, one problem per thread at a "
                       f"time on {thr} threads of {os.cpu_count()} host CPUs (the box's CPU "
                       f"share), {tt:.2f} s"),
        },
    }


def cpu_baseline_c5fit(models, datasets, raw0, iters, gpu_final, threads, min_seconds=2.0):
    """The C5 fit on the CPU: oracle/lfm_cpu.cpp's JaxTrainer.fit (value and gradient by dual
    numbers of the reference's erf formulas, explicit Sigma^{-1}, the same Adam loop) of the 15
    problems sequentially on ONE core, repeated until min_seconds have passed; the final losses
    check the GPU fit's."""
    from dis_project_amd import trainer as TR
    from oracle import lfm_cpu

    genes = [m.num_genes for m in models]
    nvec = 3 * sum(genes)
    rounds, finals = 0, None
    t0 = time.perf_counter()
    while True:
        finals, off = [], 0
        for p, (m, d) in enumerate(zip(models, datasets)):
            G = genes[p]
            r = np.concatenate([raw0[off:off + 3 * G], raw0[nvec + 3 * p: nvec + 3 * p + 3]])
            off += 3 * G
            h, _ = lfm_cpu.fit(d.X, d.y, G, r, iters, lr=0.01, spe=1000, fix=False,
                               negative=True)
            finals.append(h[-1])
        rounds += 1
        if time.perf_counter() - t0 >= min_seconds:
            break
    t = time.perf_counter() - t0
    ref = np.asarray(finals)
    rel = np.abs(ref - np.asarray(gpu_final)) / np.abs(ref)
    per_step = len(models) * iters
    # the same fits across the box's CPU share: one problem per OpenMP thread at a time
    # (lfm_cpu_fit_batch), repeated until min_seconds have passed
    thr = threads
    xs, ys = [d.X for d in datasets], [d.y for d in datasets]
    r0 = []
    off = 0
    for p, G in enumerate(genes):
        r0.append(np.concatenate([raw0[off:off + 3 * G], raw0[nvec + 3 * p: nvec + 3 * p + 3]]))
        off += 3 * G
    trounds, t1 = 0, time.perf_counter()
    while True:
        hist, _ = lfm_cpu.fit_batch(xs, ys, genes, [r.copy() for r in r0], iters, lr=0.01,
                                    spe=1000, fix=False, negative=True, threads=thr)
        trounds += 1
        if time.perf_counter() - t1 >= min_seconds:
            break
    tt = time.perf_counter() - t1
    if not np.array_equal(hist[:, -1], ref):
        raise SystemExit("the threaded CPU fit disagrees with the sequential one")
    return {
        "value": rounds * per_step / t,
        "unit": "problem training steps/s",
        "cores": 1,
        "kind": "port",
        "sample": (f"oracle/lfm_cpu.cpp fit: the {len(models)} problems (N={datasets[0].n}) x "
                   f"{iters} Adam steps sequentially on ONE core, {rounds} full fits in "
                   f"{t:.2f} s ({t / rounds * 1e3:.0f} ms per fit); timed in full"),
        "host_cpus": os.cpu_count(),
        "gpu_vs_cpu_rel": float(rel.max()),
        "threads": {
            "value": trounds * per_step / tt,
            "unit": "problem training steps/s",
            "cores": thr,
            "sample": (f"oracle/lfm_cpu.cpp lfm_cpu_fit_batch: the {len(models)} fits in one "
                       f"OpenMP loop, one problem per thread at a time on {thr} threads of "
                       f"{os.cpu_count()} host CPUs (the box's CPU share; at most "
                       f"{len(models)} busy), {trounds} rounds in {tt:.2f} s"),
        },
    }


def cpu_baseline_c4(work, threads, gpu_rows, check_rows):
    """C4 on the CPU: the reference formula (fp64, every kernel branch, std::erf; stored as
    float) over every 4th row of the N = 65536 lower triangle (a quarter of the rows, ~1/4 of
    the pairs), all allowed cores, extrapolated to the full fill by pair count. Checks the
    GPU's fp32 rows `check_rows` (a subset of the sample) within 16 eps64 M + 4e-6 max|K|
    (tests/test_gpu_regimes.py's C4 bound; M = the reference formula's intermediate
    magnitude, oracle.gram_error_scale)."""
    from oracle import lfm_cpu
    from oracle import lfm_oracle as O

    m, x = work.model, np.ascontiguousarray(work.data.X)
    n = work.n
    rows = np.arange(0, n, 4, dtype=np.int64)
    t0 = time.perf_counter()
    ref = lfm_cpu.gram_rows_f32(x, m.true_d, m.true_s, m.l, rows, 0.0, threads)
    t = time.perf_counter() - t0
    pairs_sample = float(np.sum(rows + 1))
    pairs_full = n * (n + 1) / 2.0
    t_full = t * pairs_full / pairs_sample
    # parity of the GPU rows against the sample (rows are multiples of 4)
    idx = np.searchsorted(rows, check_rows)
    assert np.all(rows[idx] == check_rows)
    scale = O.gram_error_scale(x[check_rows], x, m.true_d, m.true_s, m.l)
    kmax = float(np.abs(ref[idx]).max())
    worst = 0.0
    for q, r in enumerate(check_rows):
        tol = 16 * EPS64 * scale[q, : r + 1] + 4e-6 * kmax
        err = np.abs(gpu_rows[q, : r + 1].astype(np.float64) - ref[idx[q], : r + 1])
        worst = max(worst, float((err / tol).max()))
    return {
        "value": 1.0 / t_full,
        "unit": "fp32 gram fills/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"oracle/lfm_cpu.cpp gram: every 4th row of the N={n} lower triangle "
                   f"({rows.size} rows, {pairs_sample:.3g} of {pairs_full:.3g} pairs) in "
                   f"{t:.2f} s on {threads} OpenMP threads of {os.cpu_count()} host CPUs, "
                   f"extrapolated by pair count to {t_full:.1f} s per fill"),
        "extrapolated": True,
        "host_cpus": os.cpu_count(),
        "gpu_rows_checked": int(len(check_rows)),
        "gpu_vs_cpu_err_over_tol": worst,
    }


# ------------------------------------------------------------------ workloads
def c4_setup(ctx, a):
    """Device buffers of the C4 fill: x (N x 3) and the N x N fp32 output."""
    work = configs.c4(a.genes, a.timepoints)
    x = np.ascontiguousarray(work.data.X)
    n = work.n
    lib, h = ctx.lib, ctx.handle
    dx, dK = _lib.c_void_p(), _lib.c_void_p()
    ctx.check(lib.lfm_dev_alloc(h, x.nbytes, _lib.ctypes.byref(dx)))
    ctx.check(lib.lfm_dev_alloc(h, n * n * 4, _lib.ctypes.byref(dK)))
    ctx.check(lib.lfm_memcpy_h2d(h, dx, x.ctypes.data, x.nbytes))
    hp = work.model.hyp()

    def step():
        ctx.check(lib.lfm_gram_f32_dev(h, dx, n, hp.ref, 0.0, _lib.LFM_UPLO_LOWER, dK, n))
        # a checksum-free scalar per step: the last diagonal element (a device read of 4 B)
        out = np.empty(1, np.float32)
        ctx.check(lib.lfm_memcpy_d2h(h, out.ctypes.data,
                                     _lib.c_void_p(dK.value + (n * n - 1) * 4), 4))
        return np.array([float(out[0])])

    def rows(rr):
        got = np.empty((len(rr), n), np.float32)
        for i, r in enumerate(rr):
            ctx.check(lib.lfm_memcpy_d2h(h, got[i].ctypes.data,
                                         _lib.c_void_p(dK.value + int(r) * n * 4), n * 4))
        return got

    def close():
        lib.lfm_dev_free(h, dK)
        lib.lfm_dev_free(h, dx)

    return work, step, rows, close


def make_gather(ctx, world, rank, mode, rccl=None, require=False):
    """The farm's result exchange for this rank: (gather, kind). kind "rccl": the library's
    RCCL all-gather (non-blocking communicator, every wait bounded by LFM_RCCL_TIMEOUT_S);
    "gloo": the rehearsal's torch.distributed all-gather; "gloo-fallback": any rank's RCCL
    communicator failed to initialise, so every rank (they agree over the gloo control plane)
    exchanges over gloo instead — unless `require` (bench.py --require-rccl, the default outside
    rehearsals), when every rank exits non-zero naming the cause. rccl(ctx, world, rank, uid)
    builds the communicator (tests pass a stand-in); the unique id comes from rank 0."""
    _load()
    if world <= 1:
        return (lambda send: np.asarray(send, np.float64).copy()), "none"
    if mode == "gloo":
        return farm.TorchGather(world), "gloo"
    if rccl is None:
        rccl = farm.RcclGather
    # a peer that never joins ends the init after this bound (then the gloo fallback), not at
    # the library's 300 s default
    os.environ.setdefault("LFM_RCCL_TIMEOUT_S", "120")
    uid = None
    if rank == 0:
        uid = farm.RcclGather.unique_id(ctx) if rccl is farm.RcclGather else b"\0" * 128
    obj = [uid]
    dist.broadcast_object_list(obj, src=0)
    err, gather = None, None
    try:
        gather = rccl(ctx, world, rank, obj[0])
    except Exception as e:  # noqa: BLE001 — every rank must learn of any rank's failure
        err = e
    ok = torch.tensor([0 if err is not None else 1], dtype=torch.int32)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if int(ok.item()):
        return gather, "rccl"
    if gather is not None:
        gather.close()
    cause = err if err is not None else "failed on another rank"
    if require:
        # the measured configuration is RCCL over xGMI: no gloo line stands in for it
        raise SystemExit(f"rank {rank}: RCCL communicator unavailable ({cause}); "
                         "--require-rccl (the default outside rehearsals) ends the run")
    # one rank's communicator failed: every rank exchanges over gloo instead, and the line says
    # so (the evaluations themselves are unaffected)
    print(f"rank {rank}: RCCL communicator unavailable ({cause}); "
          "results exchanged over gloo", file=sys.stderr, flush=True)
    return farm.TorchGather(world), "gloo-fallback"


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    a = parse(argv)
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        return self_launch(a, argv)
    _load()
    if os.environ.get("LFM_BENCH_WATCHDOG"):
        # diagnostics: dump every thread's Python stack (and exit) if the run outlives this
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["LFM_BENCH_WATCHDOG"]), exit=True)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}: one process per GPU")
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=900))

    # one GPU per rank; the rehearsal may put several ranks on one card
    rehearsal = a.gather == "gloo" or a.share_gpus
    ndev = _lib.device_count()
    if not rehearsal and local >= ndev:
        raise SystemExit(f"rank {rank}: LOCAL_RANK {local} but only {ndev} GPU(s) visible")
    dev = local % max(1, ndev) if rehearsal else local
    ctx = _lib.get_context(dev)
    lib, h = ctx.lib, ctx.handle

    # farm communicator (replicas-only exchange of per-rank results)
    gather, exchange = make_gather(ctx, world, rank, a.gather, require=a.require_rccl)
    fm = farm.Farm(world, rank, gather)

    workers = None
    c4_rows = None
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
    elif a.workload == "c4":
        work, one_fill, c4_rows, close = c4_setup(ctx, a)
        n = work.n
        per_step = world

        def step():
            return fm.run(world, lambda idx: one_fill())
    elif a.workload == "c5fit":
        from dis_project_amd import trainer as TR

        models, datasets = farm.workload("c5")
        n = datasets[0].n
        P = len(models)
        genes = [m.num_genes for m in models]
        gmax = max(genes)
        # the fits farmed: rank r fits its static block (farm.partition) in one launch, then
        # one all-gather of every fit's final raw parameters and loss history
        # (Farm.run_records; trainer.FarmTrainer); one rank: the whole batch, no exchange
        mine = farm.partition(P, world, rank)
        my_models = [models[i] for i in mine]
        raw0 = TR.pack_raw([TR.unconstrain(m) for m in my_models], [m.jitter for m in my_models])
        # notebook.py:55-75: adam(0.01), fix_params=False, num_steps_per_epoch=1000
        fit_opt = _lib.LfmAdam(0.01, 0.9, 0.999, 1e-8, 0.0, 1000, 0)
        iters = a.fit_iters
        per_step = P * iters  # the 15 fits' training steps, each on exactly one rank
        fit_hist = np.empty((iters, len(mine)))
        close = (lambda: None)
        if len(mine):
            fit_ev = farm.BatchEvaluator(ctx, [datasets[i] for i in mine], negative=True)
            close = fit_ev.close
            batch = fit_ev.registered([m.num_genes for m in my_models])

        def fit_block():
            raw = raw0.copy()
            mu, nu = np.zeros_like(raw), np.zeros_like(raw)
            ctx.check(lib.lfm_batch_fit_f64(h, batch, _lib.ctypes.byref(fit_opt), 1, 0, iters,
                                            _lib.dptr(raw), _lib.dptr(mu), _lib.dptr(nu),
                                            _lib.dptr(fit_hist), None))
            return raw

        if world == 1:
            def step():
                fit_block()
                return fit_hist[-1].copy()  # each problem's final loss
        else:
            rec_len = 3 * gmax + 2 + iters

            def block(idx):
                raw = fit_block()
                return TR.fit_records(TR.unpack_raw(raw, [genes[i] for i in idx]), fit_hist.T,
                                      gmax)

            def step():
                rec = fm.run_records(P, rec_len, block)
                step.records = rec
                return rec[:, -1].copy()  # each problem's final loss
    elif a.workload == "c5":
        # rounds: R hyperparameter rounds of the 15 problems per rank (round-major, so the
        # static partition gives each rank whole rounds); a step evaluates this rank's R x 15
        # problems in ONE batched launch (hyperparameters packed once) and exchanges them in ONE
        # all-gather (over RCCL: the device-side round, lfm_farm_batch_mll_f64). One GPU with
        # R = 1 is configs[4]'s own step, the 15 problems
        R = a.rounds
        models, datasets = farm.workload("c5", rounds=world * R)
        n = datasets[0].n
        P = len(models)
        mine = farm.partition(P, world, rank)
        per_step = P
        fev = farm.BatchEvaluator(ctx, [datasets[i] for i in mine])
        close = fev.close
        c5_hyp = fev.pack([models[i] for i in mine])
        if world == 1:
            def step():
                return fev.evaluate_packed(c5_hyp)
        elif exchange == "rccl":
            def step():
                return fm.run_fused(P, lambda slots: fev.farm_round_packed(c5_hyp, slots))
        else:
            def step():
                return fm.run(P, lambda idx: fev.evaluate_packed(c5_hyp))
    else:
        models, datasets = farm.workload(a.workload, a.genes, a.timepoints, a.restarts)
        n = datasets[0].n
        mine = farm.partition(len(models), world, rank)
        workers = a.workers if a.workers > 0 else farm.choose_workers(len(mine))
        per_step = len(models)
        evaluate, close = farm.gpu_evaluator(ctx, datasets, negative=False, workers=workers)

        def step():
            return fm.run_problems(models, datasets, evaluate)

    results = []

    def barrier():
        ctx.check(lib.lfm_ctx_synchronize(h))
        if world > 1:
            dist.barrier()

    for _ in range(a.warmup):
        results.append(step())
    # HIP events around the priced kernels' launches: c2 in the FIRST timed step only (an
    # event record between two dependent launches widens the dispatch gap, ≈ 0.5 ms per
    # evaluation with all step launches instrumented; one instrumented step of K costs
    # 0.5 / K ms); c4 in every step (one fill launch per step)
    prof = not a.no_profile and a.workload in ("c2", "c4", "c5fit")
    prof_steps = (1 if a.workload == "c2" else a.steps) if prof else 0
    classes = {"c2": ["syrk", "gram_grid", "potrf", "syrk_side"], "c4": ["gram_grid", "tables"],
               "c5fit": ["small_grad"]}.get(a.workload)
    if prof:
        ctx.profile(False)
        ctx.profile_reset()
    timed, step_ms = [], []
    # schedule-3 stalls re-run on schedule 1 inside the call (lfm_ctx_fallbacks): counted over
    # the timed region, so a line can never price a fallback as the step kernel
    fb0 = ctx.fallbacks
    sched = ctx.schedule
    barrier()
    t0 = time.perf_counter()
    for s in range(a.steps):
        if s < prof_steps and s == 0:
            ctx.profile(True, classes=classes)
        ts = time.perf_counter()
        timed.append(step())
        step_ms.append((time.perf_counter() - ts) * 1e3)
        if s + 1 == prof_steps:
            ctx.profile(False)
    barrier()
    elapsed = time.perf_counter() - t0
    fallbacks = ctx.fallbacks - fb0
    if prof:
        stats = ctx.profile_read()
    # per-step wall (each step ends on the host: its results are read back), median per rank
    med_ms = float(np.median(step_ms))
    if world > 1:
        t = torch.tensor([elapsed, med_ms], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, med_ms = (float(v) for v in t.tolist())
        fb = torch.tensor([fallbacks], dtype=torch.int64)
        dist.all_reduce(fb, op=dist.ReduceOp.SUM)
        fallbacks = int(fb.item())
    # the exchange step alone (collective latency reported separately): the same
    # all-gather of this workload's NaN-padded slots, outside the timed region
    collective = None
    if world > 1:
        # this workload's own exchange size: the records of c5fit's fits, c5's rounds, c3's
        # restarts, one slot per rank for c2 / c4
        if a.workload == "c5fit":
            slots = farm.slots_per_rank(P, world) * (3 * gmax + 2 + iters)
        elif a.workload in ("c2", "c4"):
            slots = 1
        else:
            slots = max(farm.slots_per_rank(per_step, world), 1)
        lat = []
        for _ in range(25):
            barrier()
            t1 = time.perf_counter()
            gather(np.full(slots, np.nan))
            lat.append((time.perf_counter() - t1) * 1e6)
        lt = torch.tensor([float(np.median(lat[5:]))], dtype=torch.float64)
        dist.all_reduce(lt, op=dist.ReduceOp.MAX)
        collective = {"op": {"rccl": "ncclAllGather (RCCL)", "gloo": "gloo all_gather",
                             "gloo-fallback": "gloo all_gather (RCCL init failed)"}[exchange],
                      "bytes_per_rank": 8 * slots,
                      "latency_us_median": float(lt.item())}
        if a.workload == "c5" and exchange == "rccl":
            collective["in_step"] = ("chained on the device: batch kernel -> ncclAllGather -> "
                                     "publish kernel, one bounded host wait "
                                     "(lfm_farm_batch_mll_f64)")
    elif a.workload in ("c3", "c5"):
        # one GPU: the library's exchange path alone on a 1-rank RCCL communicator (staging
        # copies, enqueue, the bounded host wait; no xGMI transfer) — the floor the W > 1
        # all-gather adds to per step. Best effort: a box without RCCL just omits it.
        slots = max(per_step, 1)
        try:
            g1 = farm.RcclGather(ctx, 1, 0, farm.RcclGather.unique_id(ctx))
            try:
                lat = []
                for i in range(120):
                    t1 = time.perf_counter()
                    g1(np.full(slots, np.nan))
                    lat.append((time.perf_counter() - t1) * 1e6)
            finally:
                g1.close()
            collective = {"op": "ncclAllGather (RCCL, 1 rank: the library's host path only, "
                                "no xGMI transfer)",
                          "bytes_per_rank": 8 * slots,
                          "latency_us_median": float(np.median(lat[20:]))}
            if a.workload == "c5":
                # the whole device-side round on a 1-rank communicator: the batch kernel writing
                # its send slots, ncclAllGather behind it, the publish kernel, one host wait —
                # what a step costs per rank at W > 1 less the xGMI transfer itself
                g1 = farm.RcclGather(ctx, 1, 0, farm.RcclGather.unique_id(ctx))
                fev1 = farm.BatchEvaluator(ctx, datasets)
                try:
                    f1 = farm.Farm(1, 0, None)
                    want = np.asarray(timed[0])
                    rl = []
                    for i in range(300):
                        t1 = time.perf_counter()
                        got = f1.run_fused(len(models), lambda s_: fev1.farm_round(models, s_))
                        rl.append((time.perf_counter() - t1) * 1e6)
                    if not np.array_equal(got, want):
                        raise SystemExit("the device-side farm round disagrees with the step")
                finally:
                    fev1.close()
                    g1.close()
                collective["chained_round_us_median"] = float(np.median(rl[50:]))
                collective["chained_round"] = ("batch kernel -> ncclAllGather (1 rank) -> "
                                               "publish kernel, one host wait "
                                               "(lfm_farm_batch_mll_f64)")
        except SystemExit:
            raise
        except Exception as e:  # noqa: BLE001
            collective = {"op": "ncclAllGather (RCCL, 1 rank)", "error": str(e)}
    # the timed region's results: all finite, every step the same values (same inputs)
    res = np.array(timed)
    if not np.all(np.isfinite(res)):
        raise SystemExit(f"non-finite result in the timed region: {res[~np.isfinite(res)][:4]}")
    if not np.all(res == res[0]):
        raise SystemExit("timed steps disagree (the same inputs gave different results)")

    # multi-rank farms, checked after the timed region on rank 0: the gathered results are the
    # bits of one rank doing the whole step alone (the same kernels on the same inputs)
    if world > 1 and rank == 0 and a.workload == "c5":
        evl = farm.BatchEvaluator(ctx, datasets)
        try:
            local = evl.evaluate_packed(evl.pack(models))
        finally:
            evl.close()
        if not np.array_equal(local, res[0]):
            raise SystemExit("the gathered c5 rounds differ from one rank's evaluation of them")
    if world > 1 and rank == 0 and a.workload == "c5fit":
        from dis_project_amd import trainer as TR

        evl = farm.BatchEvaluator(ctx, datasets, negative=True)
        try:
            bl = evl.registered(genes)
            raw = TR.pack_raw([TR.unconstrain(m) for m in models], [m.jitter for m in models])
            mu, nu = np.zeros_like(raw), np.zeros_like(raw)
            hist1 = np.empty((iters, P))
            ctx.check(lib.lfm_batch_fit_f64(h, bl, _lib.ctypes.byref(fit_opt), 1, 0, iters,
                                            _lib.dptr(raw), _lib.dptr(mu), _lib.dptr(nu),
                                            _lib.dptr(hist1), None))
        finally:
            evl.close()
        want = TR.fit_records(TR.unpack_raw(raw, genes), hist1.T, gmax)
        if not np.array_equal(np.isnan(want), np.isnan(step.records)) or \
                not np.array_equal(want[~np.isnan(want)], step.records[~np.isnan(want)]):
            raise SystemExit("the gathered fits differ from one rank's fit of all 15")
    c5_rounds16 = None
    if world == 1 and a.workload == "c5" and a.rounds == 1:
        # the per-GPU capacity at the multi-GPU lines' round count (C5_ROUNDS_MULTI rounds of
        # the 15 in one launch): the W = 1 point of the weak-scaling curve over rounds
        m16, d16 = farm.workload("c5", rounds=C5_ROUNDS_MULTI)
        ev16 = farm.BatchEvaluator(ctx, d16)
        try:
            h16 = ev16.pack(m16)
            for _ in range(max(a.warmup, 10)):
                v16 = ev16.evaluate_packed(h16)
            t16 = []
            for _ in range(a.steps):
                t1 = time.perf_counter()
                v16 = ev16.evaluate_packed(h16)
                t16.append((time.perf_counter() - t1) * 1e3)
        finally:
            ev16.close()
        if not np.allclose(v16[:len(res[0])], res[0], rtol=1e-12, atol=0):
            raise SystemExit("round 0 of the 16-round batch differs from the 15-problem step")
        c5_rounds16 = {"rounds": C5_ROUNDS_MULTI, "problems_per_step": len(m16),
                       "ms_per_step": float(np.median(t16)),
                       "value": len(m16) * 1e3 / float(np.median(t16)), "unit": "MLL evals/s",
                       "note": "one launch of the 16 rounds x 15 problems (hyperparameters read "
                               "from pinned memory: more than 16 problems), the W = 1 point of "
                               "the multi-GPU lines' weak scaling over rounds"}

    # value: the median step, max over ranks — one slow step (a clock dip, the
    # first step's HIP-event records) does not move it; the mean over the K steps between the
    # barriers is kept beside it (mean_value, mean_ms_per_step)
    mean_ms = elapsed / a.steps * 1e3
    value = per_step * 1e3 / med_ms
    ms_per_step = med_ms
    chol_flops = n**3 / 3.0
    # c3 and c5fit: a fixed set of problems partitioned over the ranks; c5: R rounds per rank
    scaling = "strong" if a.workload in ("c3", "c5fit") else "weak"
    if a.workload == "c2":
        wl = (f"configs[1]: one MLL eval per rank, {a.genes} genes x {a.timepoints} timepoints, "
              f"N={n}, fp64")
    elif a.workload == "c3":
        wl = (f"configs[2]: {len(res[0])} random restarts of the {a.genes}x{a.timepoints} grid "
              f"(N={n}, fp64) per step, farmed over {world} GPU(s), "
              + (f"{workers} concurrent schedule-1 evaluations per GPU" if workers > 1
                 else "one schedule-3 evaluation at a time per GPU, restarts pipelined "
                      "(lfm_mll_multi_f64)"))
    elif a.workload == "c4":
        wl = (f"configs[3]: one fp32 lower-triangle gram fill per rank, {a.genes} genes x "
              f"{a.timepoints} timepoints, N={n} (Sigma stored as an N x N fp32 buffer)")
    elif a.workload == "c5fit":
        wl = (f"configs[4]'s training workflow (notebook.py:55-75): JaxTrainer.fit of the 15 "
              f"replicate x leave-one-gene-out problems (N={n}), {a.fit_iters} adam(0.01) steps "
              f"each, fix_params=False; each rank fits its block of the 15 in one launch "
              f"(lfm_batch_fit_f64)" + (", then one all-gather of the fits' final raw parameters "
                                        "and loss histories" if world > 1 else ""))
    else:
        wl = (f"configs[4]: 3 replicates x 5 leave-one-gene-out ablations (N={n}), "
              f"{a.rounds} hyperparameter round(s) of the 15 per rank per step "
              f"({per_step} evaluations over {world} GPU(s)), one batched launch per rank"
              + (" and one all-gather" if world > 1 else ""))
    c4 = a.workload == "c4"
    fit = a.workload == "c5fit"
    line = {
        "metric": ("fp32 gram fills/sec at N=65536 (configs[3])" if c4 else
                   "MLL value_and_grad + Adam training steps/sec (configs[4] fit, 15 problems x "
                   f"{a.fit_iters} steps)" if fit else METRIC),
        "value": value,
        "unit": ("fp32 gram fills/s" if c4 else "problem training steps/s" if fit
                 else "MLL evals/s"),
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": ms_per_step,
        "value_basis": "median step wall time (max over ranks of each rank's median)",
        "mean_value": per_step * a.steps / elapsed,
        "mean_ms_per_step": mean_ms,
        "timed_region_s": elapsed,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f64" if not c4 else "f32",
        "data": "synthetic (seeded numpy: D~U[.2,1], S~U[.5,1.5], B~U[.01,.1], y = B/D + "
                "0.5 N(0,1), t = linspace(0,12,T))",
        "config": {"workload": wl, "N": n,
                   "genes": a.genes if a.workload not in ("c5", "c5fit") else 4,
                   "timepoints": a.timepoints if a.workload not in ("c5", "c5fit") else 7,
                   "problems_per_step": per_step,
                   "parallelism": (f"replicas{world}: {a.rounds} hyperparameter round(s) of the "
                                   "15 problems per rank (weak scaling over rounds)"
                                   if a.workload == "c5" else
                                   f"replicas{world}: the 15 fits partitioned over the ranks"
                                   if a.workload == "c5fit" else f"replicas{world}"),
                   "exchange": {"rccl": "RCCL all-gather of NaN-padded per-rank result slots",
                                "gloo": "gloo all-gather (rehearsal)",
                                "gloo-fallback": "gloo all-gather of the same slots (the RCCL "
                                                 "communicator failed to initialise)"}[exchange]
                               if world > 1 else "none"},
        "result_first": float(res[0][0]),
        # the factorisation schedule the timed steps were meant to run (rank 0's context) and
        # the schedule-3 calls of the timed region, over all ranks, that stalled and were re-run
        # on schedule 1 (lfm_ctx_fallbacks): must be 0 for a c2 / c3 line to stand
        "schedule": sched if a.workload in ("c2", "c3") else None,
        "s3_fallbacks": fallbacks,
    }
    if workers is not None:
        line["config"]["workers_per_gpu"] = workers
    if collective:
        line["collective"] = collective
    if c5_rounds16:
        line["rounds16"] = c5_rounds16
    if a.workload in ("c2", "c3"):
        line["cholesky_gflops_per_gpu"] = chol_flops * value / world / 1e9
    if a.workload == "c3":
        # the whole factorisation's N^3/3 per evaluation over the wall time, per GPU: the farm's
        # schedule-1 workers interleave several kernels, so no single kernel is priced here
        ach = chol_flops * value / world / 1e12
        line["roofline"] = {
            "kernel": "whole evaluation (N^3/3 flop per MLL over the wall time, per GPU)",
            "bound": "mfma", "achieved": ach, "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": ach / FP64_MFMA_PEAK_TFLOPS, "traffic": None}
    if prof and rank == 0 and a.workload == "c2":
        syrk = stats.get("syrk", {})
        gram = stats.get("gram_grid", {})
        chain = stats.get("potrf", {})
        line["kernel_ms_per_eval"] = {k: round(v["total_ms"] / prof_steps, 4)
                                      for k, v in stats.items() if v["launches"]}
        if syrk.get("launches"):
            ach = syrk["flops"] / (syrk["total_ms"] * 1e-3) / 1e12
            traffic, tsrc = None, None
            tf = os.path.join(ROOT, "profiles", "syrk_traffic.json")
            if os.path.exists(tf):
                try:
                    rec = json.load(open(tf))
                    per_eval = rec.get("hbm_bytes_per_eval")
                    pmc_lpe = rec.get("launches", 0) / max(1, rec.get("evals", 1))
                    lpe = syrk["launches"] / prof_steps
                    if rec.get("n", 16384) != n:
                        # the counters were collected on another configuration's launches
                        tsrc = (f"none: the PMC record (profiles/syrk_traffic.json) is of "
                                f"N = {rec.get('n', 16384)}, this run is N = {n}")
                    elif rec.get("schedule") == "LFM_S3_EVENTS=2" and round(pmc_lpe) == round(lpe):
                        # the counters saw this schedule's own launches (serialised by events)
                        traffic = rec.get("hbm_bytes_per_launch")
                        tsrc = ("PMC (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, gfx950 correction) "
                                "per step launch, profiles/syrk_traffic.json: the timed "
                                "schedule's own launches, serialised by stream events "
                                f"(LFM_S3_EVENTS=2, {pmc_lpe:.0f} per evaluation, as here) so "
                                "their device-side waits are met under the counters' serialised "
                                "dispatch; per launch in its last_eval_launch_bytes")
                    else:
                        traffic = per_eval / lpe if per_eval else None
                        tsrc = ("PMC (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, gfx950 correction) "
                                "bytes per evaluation from profiles/syrk_traffic.json "
                                f"({pmc_lpe:.0f} step launches per eval, schedule "
                                f"{rec.get('schedule', 'LFM_S3_EVENTS=1')}) divided by this "
                                f"run's {lpe:.0f} launches per evaluation")
                except Exception:
                    traffic = None
            line["roofline"] = {
                "kernel": "step_kernel (fp64 MFMA trailing update + tall panel solve)",
                "bound": "mfma", "achieved": ach, "peak": FP64_MFMA_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": ach / FP64_MFMA_PEAK_TFLOPS, "traffic": traffic,
                "traffic_source": tsrc,
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
            else:  # LFM_GRAM_FUSE=0: the fp64 lower fill as its own kernel
                gbs = gram["bytes"] / (gram["total_ms"] * 1e-3) / 1e9
                line["gram_roofline"] = {
                    "kernel": "gram_grid_aligned_kernel (fp64 lower-triangle fill)",
                    "bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": gbs / HBM_PEAK_GBS,
                    "bytes_per_launch": gram["bytes"] / gram["launches"],
                    "avg_launch_ms": gram["total_ms"] / gram["launches"],
                }
    if prof and rank == 0 and fit:
        sg = stats.get("small_grad", {})
        if sg.get("launches"):
            launch_ms = sg["total_ms"] / sg["launches"]
            # algorithmic fp64 work of one training step of one problem (n = 28): the Cholesky
            # of the augmented matrix ((n+1)^3 / 3), the triangular inverse (n^3 / 3) and
            # Sigma^{-1} = X^T X (n^3 / 3); the kernel evaluations are transcendental-bound VALU
            # work on top. One workgroup per problem: 15 of the chip's 256 CUs — the bound is the
            # latency of one problem's step chain, not a throughput roofline
            fl = ((n + 1) ** 3 / 3.0 + 2 * n ** 3 / 3.0) * per_step
            ach = fl / (launch_ms * 1e-3) / 1e12
            line["roofline"] = {
                "kernel": "small_fit_kernel (one workgroup per problem, 150 steps in-kernel)",
                "bound": "mfma", "achieved": ach, "peak": FP64_MFMA_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": ach / FP64_MFMA_PEAK_TFLOPS, "traffic": None,
                "note": "latency-bound: 15 workgroups on 256 CUs; frac is of the whole chip",
                "launches": sg["launches"], "avg_launch_ms": launch_ms,
                "us_per_training_step": launch_ms * 1e3 / a.fit_iters,
            }
        # the per-call path this replaces: 15 sequential lfm_mll_grad_f64 calls per training step
        # (each the large-N machinery: a bordered 256 x 256 factorisation, several launches)
        seq = []
        hp = [m.hyp() for m in models]
        gbuf = np.empty(3 * max(m.num_genes for m in models) + 2)
        vbuf = np.empty(1)
        xs = [np.ascontiguousarray(d.X) for d in datasets]
        ys = [np.ascontiguousarray(d.y.reshape(-1)) for d in datasets]
        for r in range(12):
            t1 = time.perf_counter()
            for m, hpp, x_, y_ in zip(models, hp, xs, ys):
                ctx.check(lib.lfm_mll_grad_f64(h, _lib.dptr(x_), _lib.dptr(y_), x_.shape[0],
                                               hpp.ref, 1, _lib.dptr(vbuf), _lib.dptr(gbuf)))
            seq.append((time.perf_counter() - t1) * 1e6)
        seq_us = float(np.median(seq[2:]))
        line["per_call_path"] = {
            "op": "15 sequential lfm_mll_grad_f64 calls (one training step's gradients)",
            "us_per_training_step": seq_us,
            "speedup_of_fit_kernel": (seq_us / line["roofline"]["us_per_training_step"]
                                      if "roofline" in line else None),
        }
    if prof and rank == 0 and c4:
        gram = stats.get("gram_grid", {})
        tab = stats.get("tables", {})
        if gram.get("launches"):
            gbs = gram["bytes"] / (gram["total_ms"] * 1e-3) / 1e9
            line["roofline"] = {
                "kernel": "gram_grid_aligned_kernel (fp32 lower-triangle fill)",
                "bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": gbs / HBM_PEAK_GBS, "traffic": None,
                "bytes_per_launch": gram["bytes"] / gram["launches"],
                "bytes_basis": "algorithmic: 4 B per lower element incl. the diagonal, "
                               "4 N (N + 1) / 2",
                "launches": gram["launches"],
                "avg_launch_ms": gram["total_ms"] / gram["launches"],
            }
            if tab.get("launches"):
                line["roofline"]["tables_ms_per_fill"] = tab["total_ms"] / tab["launches"]
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        thr = cpu_threads(a)
        if a.workload == "c2":
            cb = cpu_baseline_c2(work, thr, float(res[0][0]))
            bad = not cb["gpu_vs_cpu_rel"] <= PARITY_RTOL
        elif a.workload == "c3":
            cb = cpu_baseline_c3(models, datasets[0], thr, res[0])
            bad = not cb["gpu_vs_cpu_rel"] <= PARITY_RTOL
        elif a.workload == "c5":
            cb = cpu_baseline_c5(models, datasets, res[0], thr)
            bad = not cb["gpu_vs_cpu_rel"] <= PARITY_RTOL
        elif a.workload == "c5fit":
            cb = cpu_baseline_c5fit(models, datasets, raw0, a.fit_iters, res[0], thr)
            bad = not cb["gpu_vs_cpu_rel"] <= PARITY_RTOL
        else:
            check = np.array([0, 4, 256, 32768, n - 4, 4 * 5000, 4 * 9999, 4 * 16000])
            cb = cpu_baseline_c4(work, thr, c4_rows(check), check)
            bad = not cb["gpu_vs_cpu_err_over_tol"] <= 1.0
        line["cpu_baseline"] = cb
        if bad:
            print(json.dumps(line), flush=True)
            raise SystemExit(f"GPU result differs from the CPU restatement beyond tolerance: "
                             f"{ {k: v for k, v in cb.items() if 'gpu_vs' in k} }")
    if rank == 0:
        print(json.dumps(line), flush=True)
    if fallbacks and a.workload in ("c2", "c3"):
        raise SystemExit(f"{fallbacks} timed schedule-3 call(s) stalled and were re-run on "
                         "schedule 1: the line above does not measure the priced schedule")
    close()
    if world > 1:
        gather.close()
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
