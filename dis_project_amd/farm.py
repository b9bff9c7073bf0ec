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

import math
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


class Farm:
    """Evaluate P independent problems over W ranks and all-gather the results.

    `evaluate(indices) -> values` runs this rank's share (on this rank's GPU in the product
    path: e.g. ``CustomConjMLL.batch`` on its models / datasets); `gather(send) -> recv`
    exchanges the fixed-size slots.
    """

    def __init__(self, world: int, rank: int, gather: Callable[[np.ndarray], np.ndarray]):
        self.world, self.rank, self.gather = world, rank, gather

    def run(self, nprob: int, evaluate: Callable[[Sequence[int]], np.ndarray]) -> np.ndarray:
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
