"""Multi-GPU farm of independent marginal-likelihood evaluations.

Replicas only: a single Cholesky is never sharded. P independent problems (random
restarts of config 3, replicate x ablation problems of config 5) are split over W ranks
(one process per GPU) by a static block partition — rank r owns problems
[r * ceil(P/W), min(P, (r + 1) * ceil(P/W))) — each rank evaluates its share on its own
GPU, and one all-gather of fixed-size, NaN-padded fp64 slots (ceil(P/W) per rank) returns
every result to every rank. On MI355X the all-gather is RCCL over xGMI
(`lfm_farm_allgather_f64`); the CPU tests drive the same logic over gloo.
"""

from __future__ import annotations

import concurrent.futures as cf
import itertools
import math
import operator
import threading
from typing import Callable, Sequence

import numpy as np

from . import _lib


def partition(nprob: int, world: int, rank: int) -> range:
    """Problems owned by `rank` under the static block partition."""
    if world < 1 or not 0 <= rank < world or nprob < 0:
        raise ValueError("bad partition arguments")
    per = math.ceil(nprob / world) if nprob else 0
    lo = min(nprob, rank * per)
    return range(lo, min(nprob, lo + per))


def slots_per_rank(nprob: int, world: int) -> int:
    return math.ceil(nprob / world) if nprob else 0


class RcclGather:
    """All-gather of fp64 slots through liblfm's RCCL communicator (one per context)."""

    def __init__(self, ctx: _lib.Context, world: int, rank: int, uid: bytes):
        self.ctx, self.world, self.rank = ctx, world, rank
        buf = (_lib.ctypes.c_ubyte * 128).from_buffer_copy(uid)
        ctx.check(ctx.lib.lfm_farm_init(ctx.handle, buf, world, rank))
        ctx.farm_ranks = world  # the device-side rounds' receive size (BatchEvaluator.farm_round)

    @staticmethod
    def unique_id(ctx: _lib.Context) -> bytes:
        uid = (_lib.ctypes.c_ubyte * 128)()
        ctx.check(ctx.lib.lfm_farm_unique_id(ctx.handle, uid))
        return bytes(uid)

    def __call__(self, send: np.ndarray) -> np.ndarray:
        send = np.ascontiguousarray(send, dtype=np.float64)
        recv = np.empty(send.size * self.world)
        self.ctx.check(self.ctx.lib.lfm_farm_allgather_f64(self.ctx.handle, _lib.dptr(send),
                                                           send.size, _lib.dptr(recv)))
        return recv

    def close(self):
        self.ctx.lib.lfm_farm_destroy(self.ctx.handle)


class TorchGather:
    """The same exchange over torch.distributed (gloo on CPU; used by the CPU tests)."""

    def __init__(self, world: int):
        import torch.distributed as dist

        self.dist, self.world = dist, world

    def __call__(self, send: np.ndarray) -> np.ndarray:
        import torch

        t = torch.from_numpy(np.ascontiguousarray(send, dtype=np.float64))
        out = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return torch.cat(out).numpy()

    def close(self):
        pass


class ResidentEvaluator:
    """MLL evaluations of many hyperparameter sets on ONE dataset held in HBM (the C3 random
    restarts; bench.py's C2 step): x / y are uploaded and their layout analysed once
    (``lfm_data_create``), each evaluation uploads only the 3G + 3 hyperparameters
    (``lfm_mll_f64_data``). Not PD -> NaN (JAX semantics); a device-side timeout raises.
    ``m.hyp()`` is read on every evaluation (microseconds beside a 29 ms MLL), so a model
    whose fields change between calls is evaluated with its current values."""

    def __init__(self, ctx: _lib.Context, data, negative: bool = False):
        self.ctx, self.negative = ctx, bool(negative)
        lib, h = ctx.lib, ctx.handle
        x = np.ascontiguousarray(data.X, dtype=np.float64).reshape(-1, 3)
        y = np.ascontiguousarray(data.y, dtype=np.float64).reshape(-1)
        self.n = x.shape[0]
        self.dx, self.dy, self.data = _lib.c_void_p(), _lib.c_void_p(), _lib.c_void_p()
        try:
            ctx.check(lib.lfm_dev_alloc(h, x.nbytes, _lib.ctypes.byref(self.dx)))
            ctx.check(lib.lfm_dev_alloc(h, y.nbytes, _lib.ctypes.byref(self.dy)))
            ctx.check(lib.lfm_memcpy_h2d(h, self.dx, x.ctypes.data, x.nbytes))
            ctx.check(lib.lfm_memcpy_h2d(h, self.dy, y.ctypes.data, y.nbytes))
            ctx.check(lib.lfm_data_create(h, self.dx, self.dy, self.n,
                                          _lib.ctypes.byref(self.data)))
        except Exception:
            self.close()
            raise
        self._out = np.empty(1)

    def __call__(self, models) -> np.ndarray:
        models = list(models)
        if len(models) > 1:
            # several sets: one call, pipelined on schedule 3 (lfm_mll_multi_f64: the next
            # set's prologue under the previous set's chain-bound tail; the same bits)
            hps = [m.hyp() for m in models]  # keep the buffers alive through the call
            arr = (_lib.LfmHyp * len(hps))(*[hp.struct for hp in hps])
            vals = np.empty(len(models))
            st = np.zeros(len(models), np.int32)
            rc = self.ctx.lib.lfm_mll_multi_f64(self.ctx.handle, self.data, len(hps), arr,
                                                int(self.negative), _lib.dptr(vals),
                                                _lib.dptr(st))
            self.ctx.check(rc, allow_not_pd=True)
            return vals
        vals = np.empty(len(models))
        for i, m in enumerate(models):
            hp = m.hyp()  # keeps the hyperparameter buffers alive through the call
            rc = self.ctx.lib.lfm_mll_f64_data(self.ctx.handle, self.data, hp.ref,
                                               int(self.negative), _lib.dptr(self._out))
            self.ctx.check(rc, allow_not_pd=True)
            vals[i] = self._out[0]
        return vals

    def close(self):
        lib, h = self.ctx.lib, self.ctx.handle
        if self.data:
            lib.lfm_data_destroy(self.data)
            self.data = None
        for p in ("dx", "dy"):
            ptr = getattr(self, p, None)
            if ptr:
                lib.lfm_dev_free(h, ptr)
                setattr(self, p, None)


# the packed layout of lfm_batch_mll_f64: these fields of each model, in this order
_VECS = operator.attrgetter("true_d", "true_s", "true_b")
_SCALARS = operator.attrgetter("l", "obs_stddev", "jitter")
_NUM_GENES = operator.attrgetter("num_genes")
_chain = itertools.chain.from_iterable


def unpack_grads(packed: np.ndarray, genes) -> list:
    """A packed gradient (lfm_batch_mll_grad_f64's layout: dD dS dB of each problem, then d l,
    d obs_stddev, 0 of each) as one ``CustomConjMLL.value_and_grad`` dict per problem."""
    out, off = [], 0
    nvec = 3 * sum(genes)
    for p, G in enumerate(genes):
        v = packed[off:off + 3 * G]
        sc = packed[nvec + 3 * p: nvec + 3 * p + 3]
        out.append({"true_d": v[:G].copy(), "true_s": v[G:2 * G].copy(),
                    "true_b": v[2 * G:].copy(), "l": float(sc[0]), "obs_stddev": float(sc[1])})
        off += 3 * G
    return out


class BatchEvaluator:
    """MLL evaluations of many small problems (n <= 128 each: the C5 ablations) in one batched
    launch per call, on a device-resident batch (``lfm_batch_create``: every problem's x / y in
    HBM once). A call packs every model's current hyperparameters into one array
    (``lfm_batch_mll_f64``'s layout: the true_d / true_s / true_b vectors of each problem, then
    each problem's l, obs_stddev, jitter), which the kernel reads straight from pinned host
    memory: one memcpy, one launch, one synchronise. Not PD -> NaN."""

    def __init__(self, ctx: _lib.Context, datasets, negative: bool = False):
        self.ctx, self.negative = ctx, bool(negative)
        self.datasets = list(datasets)  # held: the cache key of gpu_evaluator compares them
        self.batch = None
        probs = (_lib.LfmProblem * len(self.datasets))()
        keep = []
        for i, d in enumerate(self.datasets):
            x = np.ascontiguousarray(d.X, dtype=np.float64).reshape(-1, 3)
            y = np.ascontiguousarray(d.y, dtype=np.float64).reshape(-1)
            if y.size != x.shape[0]:
                raise ValueError("dataset x / y lengths differ")
            keep.append((x, y))
            probs[i].x = x.ctypes.data
            probs[i].y = y.ctypes.data
            probs[i].n = x.shape[0]
        self._probs, self._keep = probs, keep  # x / y kept: a new gene layout re-registers
        self._genes = None
        self.status = np.zeros(len(self.datasets), dtype=np.int32)
        self._out = np.empty(len(self.datasets))
        # raw addresses of the call's own buffers, taken once (``.ctypes.data`` costs ~1 µs each)
        self._st_ptr, self._out_ptr = self.status.ctypes.data, self._out.ctypes.data

    def _create(self, genes):
        for i, g in enumerate(genes):
            self._probs[i].hyp.num_genes = g
        h = _lib.c_void_p()
        self.ctx.check(self.ctx.lib.lfm_batch_create(self.ctx.handle, len(genes), self._probs,
                                                     _lib.ctypes.byref(h)))
        self.batch, self._genes = h, genes
        nvec = 3 * sum(genes)
        self._buf = np.empty(nvec + 3 * len(genes))
        self._vec, self._sc = self._buf[:nvec], self._buf[nvec:]
        self._buf_ptr = self._buf.ctypes.data

    def registered(self, genes) -> int:
        """The batch registered for this gene layout (re-registered if it changed): its handle."""
        genes = tuple(int(g) for g in genes)
        if genes != self._genes:
            if self.batch is not None:
                self.close()
            self._create(genes)
        return self.batch

    def _pack(self, models):
        models = list(models)
        if len(models) != len(self.datasets):
            raise ValueError("one model per registered dataset")
        self.registered(map(_NUM_GENES, models))
        np.concatenate(list(_chain(map(_VECS, models))), out=self._vec)
        self._sc[:] = list(_chain(map(_SCALARS, models)))
        return models

    def __call__(self, models) -> np.ndarray:
        self._pack(models)
        rc = self.ctx.lib.lfm_batch_mll_f64(self.ctx.handle, self.batch, self._buf_ptr,
                                            int(self.negative), self._out_ptr, self._st_ptr)
        self.ctx.check(rc, allow_not_pd=True)
        return self._out.copy()

    def pack(self, models) -> np.ndarray:
        """The models' hyperparameters in the library's packed layout (a copy; the batch is
        registered for their gene layout): a sweep whose hyperparameter sets are known up front
        packs them once and passes the array to ``evaluate_packed`` / ``farm_round_packed``."""
        self._pack(models)
        return self._buf.copy()

    def _packed(self, hyp) -> int:
        if self.batch is None or hyp.dtype != np.float64 or hyp.size != self._buf.size or \
                not hyp.flags.c_contiguous:
            raise ValueError("a packed array of this batch's layout (BatchEvaluator.pack)")
        return hyp.ctypes.data

    def evaluate_packed(self, hyp: np.ndarray) -> np.ndarray:
        """__call__ on pre-packed hyperparameters (``pack``)."""
        rc = self.ctx.lib.lfm_batch_mll_f64(self.ctx.handle, self.batch, self._packed(hyp),
                                            int(self.negative), self._out_ptr, self._st_ptr)
        self.ctx.check(rc, allow_not_pd=True)
        return self._out.copy()

    def farm_round_packed(self, hyp: np.ndarray, slots: int) -> np.ndarray:
        """farm_round on pre-packed hyperparameters (``pack``)."""
        nranks = max(1, int(getattr(self.ctx, "farm_ranks", 1)))
        recv = np.empty(nranks * int(slots))
        rc = self.ctx.lib.lfm_farm_batch_mll_f64(self.ctx.handle, self.batch, self._packed(hyp),
                                                 int(self.negative), int(slots), _lib.dptr(recv),
                                                 self._st_ptr)
        self.ctx.check(rc, allow_not_pd=True)
        return recv

    def farm_round(self, models, slots: int) -> np.ndarray:
        """One device-side farm round (``lfm_farm_batch_mll_f64``): this rank's problems
        evaluated straight into its ``slots`` RCCL send slots (NaN-padded), all-gathered on the
        device and published to the host in one chain; returns every rank's slots
        [nranks * slots]. The context's communicator must be initialised (RcclGather)."""
        self._pack(models)
        nranks = max(1, int(getattr(self.ctx, "farm_ranks", 1)))
        recv = np.empty(nranks * int(slots))
        rc = self.ctx.lib.lfm_farm_batch_mll_f64(self.ctx.handle, self.batch, self._buf_ptr,
                                                 int(self.negative), int(slots), _lib.dptr(recv),
                                                 self._st_ptr)
        self.ctx.check(rc, allow_not_pd=True)
        return recv

    def value_and_grad(self, models):
        """Every problem's value and gradient (constrained parameters, as
        ``CustomConjMLL.value_and_grad``) in ONE launch (``lfm_batch_mll_grad_f64``; n <= 127 per
        problem). Returns (values [P], [grads dict per problem]); NaN where not PD."""
        models = self._pack(models)
        grad = np.empty(self._buf.size)
        rc = self.ctx.lib.lfm_batch_mll_grad_f64(self.ctx.handle, self.batch, self._buf_ptr,
                                                 int(self.negative), self._out_ptr,
                                                 _lib.dptr(grad), self._st_ptr)
        self.ctx.check(rc, allow_not_pd=True)
        return self._out.copy(), unpack_grads(grad, self._genes)

    def close(self):
        if self.batch is not None:
            self.ctx.lib.lfm_batch_destroy(self.batch)
            self.batch = None
            self._genes = None


def workload(kind: str, genes: int = 64, timepoints: int = 256, restarts: int = 32,
             rounds: int = 1):
    """Problems of a farm workload as (models, datasets):

    ``c3``  BASELINE.json configs[2]: the C2 grid (``genes`` x ``timepoints``) under
            ``restarts`` random-restart hyperparameter sets (configs.c3_restarts), one dataset;
    ``c5``  configs[4]: 3 synthetic replicates x 5 leave-one-gene-out ablations at N = 28
            (configs.c5_ablations, notebook.py:33-75); ``rounds`` > 1: that many
            hyperparameter rounds of the 15 (configs.c5_rounds; round 0 the problems' own),
            round-major — farm.partition then gives each of W ranks whole rounds when W
            divides ``rounds``.
    """
    from . import configs

    if kind == "c3":
        base = configs.grid_workload(f"synthetic_{genes}x{timepoints}_fp64", genes, timepoints,
                                     seed_params=2, seed_y=3)
        models = configs.c3_restarts(base, restarts)
        return models, [base.data] * len(models)
    if kind == "c5":
        ws = configs.c5_ablations()
        models, datasets = [w.model for w in ws], [w.data for w in ws]
        if rounds > 1:
            models, datasets = configs.c5_rounds(models, rounds), datasets * rounds
        return models, datasets
    raise ValueError(f"unknown farm workload {kind!r}")


class Farm:
    """Evaluate P independent problems over W ranks and all-gather the results.

    `evaluate(indices) -> values` runs this rank's share (on this rank's GPU in the product
    path: e.g. ``CustomConjMLL.batch`` on its models / datasets); `gather(send) -> recv`
    exchanges the fixed-size slots.
    """

    def __init__(self, world: int, rank: int, gather: Callable[[np.ndarray], np.ndarray]):
        self.world, self.rank, self.gather = world, rank, gather

    def run(self, nprob: int, evaluate: Callable[[Sequence[int]], np.ndarray]) -> np.ndarray:
        if self.world == 1 and nprob:
            # one rank: every problem is this rank's and the exchange is the identity
            vals = np.asarray(evaluate(list(range(nprob))), dtype=np.float64).reshape(-1)
            if vals.size != nprob:
                raise ValueError("evaluate returned the wrong number of values")
            return vals.copy()
        per = slots_per_rank(nprob, self.world)
        mine = partition(nprob, self.world, self.rank)
        send = np.full(max(per, 1), np.nan)
        if len(mine):
            vals = np.asarray(evaluate(list(mine)), dtype=np.float64).reshape(-1)
            if vals.size != len(mine):
                raise ValueError("evaluate returned the wrong number of values")
            send[: len(mine)] = vals
        recv = self.gather(send).reshape(self.world, -1)
        out = np.empty(nprob)
        for r in range(self.world):
            rr = partition(nprob, self.world, r)
            out[rr.start:rr.stop] = recv[r, : len(rr)]
        return out

    def run_fused(self, nprob: int, round_fn: Callable[[int], np.ndarray]) -> np.ndarray:
        """One round whose evaluation and exchange are a single device-side chain:
        ``round_fn(slots) -> recv`` evaluates this rank's block into its NaN-padded ``slots``
        and returns every rank's slots, gathered (BatchEvaluator.farm_round over RCCL).
        Returns every problem's value, in problem order."""
        per = max(slots_per_rank(nprob, self.world), 1)
        recv = np.asarray(round_fn(per), dtype=np.float64).reshape(self.world, -1)
        out = np.empty(nprob)
        for r in range(self.world):
            rr = partition(nprob, self.world, r)
            out[rr.start:rr.stop] = recv[r, : len(rr)]
        return out

    def run_records(self, nprob: int, rec_len: int,
                    block_fn: Callable[[range], np.ndarray]) -> np.ndarray:
        """One round whose per-problem result is a fixed-length record (a fit's final raw
        parameters and loss history): ``block_fn(mine) -> [len(mine), rec_len]`` on this rank's
        block, then ONE all-gather of ceil(P/W) NaN-padded records per rank. Returns every
        problem's record [P, rec_len], in problem order, on every rank."""
        per = slots_per_rank(nprob, self.world)
        mine = partition(nprob, self.world, self.rank)
        send = np.full((max(per, 1), rec_len), np.nan)
        if len(mine):
            rec = np.asarray(block_fn(mine), dtype=np.float64)
            if rec.shape != (len(mine), rec_len):
                raise ValueError("block_fn returned records of the wrong shape")
            send[: len(mine)] = rec
        if self.world == 1:
            return send[:nprob].copy()
        recv = self.gather(send.reshape(-1)).reshape(self.world, -1, rec_len)
        out = np.empty((nprob, rec_len))
        for r in range(self.world):
            rr = partition(nprob, self.world, r)
            out[rr.start:rr.stop] = recv[r, : len(rr)]
        return out

    def run_problems(self, models, datasets, evaluate) -> np.ndarray:
        """One round over (models, datasets) — bench.py's step for ``--workload c3 / c5``:
        this rank evaluates its block through ``evaluate(models, datasets) -> values`` and the
        slots are all-gathered. Returns every problem's value on every rank."""
        if len(models) != len(datasets):
            raise ValueError("models and datasets must pair up")
        if self.world == 1 and len(models):
            # one rank: the whole round is this rank's block (no index lists, no exchange)
            vals = np.asarray(evaluate(models, datasets), dtype=np.float64).reshape(-1)
            if vals.size != len(models):
                raise ValueError("evaluate returned the wrong number of values")
            return vals.copy()
        return self.run(len(models), lambda idx: evaluate([models[i] for i in idx],
                                                          [datasets[i] for i in idx]))


# Measured C3 throughput on one MI355X at N = 16384 (scripts/concurrency_probe.py,
# profiles/r03_concurrency.json), evaluations / s with c schedule-1 evaluations in flight, and
# one schedule-3 evaluation at a time: the mean of round 3's two boxes (28.6 / 33.8 / 35.3 /
# 33.7 and 36.6; 28.0 / 33.6 / 36.6 / 33.3 and 36.5). One schedule-3 evaluation at a time is
# ahead of every concurrent count on average, and never runs an uneven remainder round.
_S1_RATE = {1: 28.3, 2: 33.7, 3: 35.95, 4: 33.5}
_S3_RATE = 36.55


def predicted_seconds(k: int, workers: int) -> float:
    """Model of a rank's wall time for k restarts with ``workers`` in flight (shared counter:
    full rounds of ``workers`` at the concurrent rate, then the remainder at its own)."""
    if k <= 0:
        return 0.0
    if workers <= 1:
        return k / _S3_RATE
    full, rem = divmod(k, workers)
    t = full * workers / _S1_RATE[min(workers, 4)]
    return t + (rem / _S1_RATE[rem] if rem else 0.0)


def choose_workers(k: int, max_workers: int = 4) -> int:
    """Evaluations in flight for a rank that owns k restarts of one large dataset: the count
    with the shortest predicted wall time (ties: fewer contexts). With the round-3 rates every
    share (32, 16, 8, 4 restarts) runs one schedule-3 evaluation at a time, so no rank runs an
    uneven remainder round (the round-2 rates chose 3 for 32 and 4 for the 8-GPU split's 4)."""
    best = 1
    for w in range(2, max(1, min(max_workers, k)) + 1):
        if predicted_seconds(k, w) < predicted_seconds(k, best) - 1e-9:
            best = w
    return best


class ConcurrentEvaluator:
    """Restart-farm throughput on one GPU (C3): ``workers`` contexts on factorisation schedule 1
    (look-ahead on every CU, include/lfm.h ``lfm_ctx_set_schedule``), each with its own HIP
    streams, workspace and resident copy of x / y, each driven by its own host thread (ctypes
    releases the GIL inside the library calls), pulling the next hyperparameter set from a
    shared counter. Several evaluations in flight fill the bubbles one evaluation's chain-bound
    tail leaves on the chip; since round 3's schedule-3 kernels, one schedule-3 evaluation at a
    time is faster (36.6 evals/s against 33.8 / 35.3 / 33.7 with 2 / 3 / 4
    schedule-1 workers), so bench.py uses this only when asked (--workers > 1).

    Worker 0 is the caller's context, switched to schedule 1 for the evaluator's lifetime and
    restored by ``close()`` (also when construction fails part-way): a schedule-3 context holds
    two CU-masked hardware queues even when idle, and idle queues beside the workers
    oversubscribe the hardware scheduler (measured -3 % with one, -10 % with two partitioned
    contexts idle). Results are per model and independent of which worker ran it (schedule 1
    is deterministic); not PD -> NaN. A worker's exception (e.g. LFM_E_TIMEOUT) stops the
    others at their next pull, and is re-raised in the caller once every worker has returned,
    so no worker thread outlives the call on these non-thread-safe contexts."""

    def __init__(self, ctx: _lib.Context, data, negative: bool = False, workers: int = 3):
        self.ctx, self._restore = ctx, ctx.schedule
        self.own, self.evs, self.pool = [], [], None
        try:
            ctx.schedule = 1
            for _ in range(max(1, int(workers)) - 1):
                c = _lib.Context(ctx.device)
                self.own.append(c)
                c.schedule = 1
            for c in [ctx] + self.own:
                self.evs.append(ResidentEvaluator(c, data, negative))
            self.pool = cf.ThreadPoolExecutor(max_workers=len(self.evs),
                                              thread_name_prefix="lfm-worker")
        except BaseException:
            self._release()
            raise

    def __call__(self, models) -> np.ndarray:
        models = list(models)
        if len(models) < 2:
            return self.evs[0](models)
        vals = np.empty(len(models))
        counter, lock, stop = itertools.count(), threading.Lock(), threading.Event()

        def work(ev):
            while not stop.is_set():
                with lock:
                    i = next(counter)
                if i >= len(models):
                    return
                try:
                    vals[i] = ev([models[i]])[0]
                except BaseException:
                    stop.set()
                    raise

        futs = [self.pool.submit(work, ev) for ev in self.evs]
        cf.wait(futs)  # every worker has returned before anything is re-raised
        for f in futs:
            f.result()  # re-raises the first worker's exception here
        return vals

    def _release(self):
        if self.pool is not None:
            self.pool.shutdown(wait=True)
            self.pool = None
        for ev in self.evs:
            ev.close()
        for c in self.own:
            c.close()
        self.evs, self.own = [], []
        self.ctx.schedule = self._restore

    def close(self):
        if self.pool is None and not self.evs and not self.own:
            return
        self._release()


def gpu_evaluator(ctx: _lib.Context, datasets, negative: bool = False, workers: int = 3):
    """The product evaluator of a farm round on this rank's GPU: problems sharing one large
    dataset go through a ConcurrentEvaluator (x / y in HBM once per worker context, ``workers``
    evaluations in flight; workers = 1: one ResidentEvaluator on ``ctx``, schedule 3;
    workers = 0: ``choose_workers`` for this rank's share); small ones through one batched
    launch (BatchEvaluator: one workgroup per problem, n <= 128, the datasets registered once;
    mixed sizes: ``CustomConjMLL.batch``)."""
    from .objectives import CustomConjMLL

    shared = len({id(d) for d in datasets}) == 1 and datasets[0].n > 128
    if shared:
        if workers <= 0:
            workers = choose_workers(len(datasets))
        if workers > 1:
            res = ConcurrentEvaluator(ctx, datasets[0], negative, workers)
        else:
            res = ResidentEvaluator(ctx, datasets[0], negative)
        return (lambda models, data: res(models)), res.close
    if all(d.n <= 128 for d in datasets):
        # registered once; a round passes this rank's block of the same datasets. The entry
        # holds the datasets themselves (BatchEvaluator.datasets), so an id() can never be
        # reused by a different dataset while its entry lives
        cache = []

        def evaluate(models, data):
            ev = cache[0] if cache else None
            if ev is None or len(ev.datasets) != len(data) or \
                    not all(map(operator.is_, ev.datasets, data)):
                close()
                ev = BatchEvaluator(ctx, data, negative)
                cache.append(ev)
            return ev(models)

        def close():
            while cache:
                cache.pop().close()

        return evaluate, close
    mll = CustomConjMLL(negative=negative)
    return (lambda models, data: mll.batch(models, data)), (lambda: None)
