"""The multi-GPU farm's partition / padding / gather logic, world_size 2 over gloo on the CPU.

The evaluator injected here is the CPU oracle (test-only); on the GPU box the product path
evaluates with liblfm and gathers with RCCL (bench.py, test_gpu_farm below)."""

import math
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from dis_project_amd import farm


def test_partition_covers_exactly_once():
    for P in (0, 1, 5, 15, 32, 33):
        for W in (1, 2, 3, 8):
            seen = []
            for r in range(W):
                seen += list(farm.partition(P, W, r))
            assert seen == list(range(P))
            assert all(len(farm.partition(P, W, r)) <= farm.slots_per_rank(P, W) for r in range(W))


def test_partition_rejects_bad_args():
    with pytest.raises(ValueError):
        farm.partition(4, 0, 0)
    with pytest.raises(ValueError):
        farm.partition(4, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_eval(models, datasets):
    from oracle import lfm_oracle as O

    return [O.mll(d.X, d.y, m.true_d, m.true_s, m.true_b, m.l, m.obs_stddev, m.jitter)
            for m, d in zip(models, datasets)]


# the farm workloads bench.py runs (--workload c5 / c3), c3 at a CPU-oracle size
WORKLOADS = [("c5", {}), ("c3", dict(genes=4, timepoints=16, restarts=5))]


def _worker(rank, world, port, q):
    import sys

    import torch.distributed as dist

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from dis_project_amd import farm as F

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    f = F.Farm(world, rank, F.TorchGather(world))
    outs = []
    for kind, kw in WORKLOADS:
        # the same round function bench.py's step calls, with the CPU oracle as evaluator
        models, datasets = F.workload(kind, **kw)
        outs.append(f.run_problems(models, datasets, _oracle_eval).tolist())
    out_odd = f.run(3, lambda idx: [float(i) for i in idx])  # fewer problems than slots
    q.put((rank, outs, out_odd.tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_farm_gloo_world2(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    refs = [_oracle_eval(*farm.workload(kind, **kw)) for kind, kw in WORKLOADS]
    for rank, outs, out_odd in res:
        for out, ref in zip(outs, refs):
            np.testing.assert_array_equal(np.array(out), np.array(ref))
            assert not any(math.isnan(v) for v in out)
        assert out_odd == [0.0, 1.0, 2.0]


@pytest.mark.gpu
@pytest.mark.parametrize("kind,kw", [("c5", {}), ("c3", dict(genes=4, timepoints=64, restarts=6))])
def test_farm_rccl_single_rank_liblfm(kind, kw):
    """Product path on one GPU, as bench.py --workload c3 / c5 runs it: the liblfm evaluator
    (one batched launch for C5; the HBM-resident dataset for C3, N = 256) and the RCCL
    all-gather (world 1), against the oracle."""
    from dis_project_amd import _lib

    ctx = _lib.get_context()
    models, datasets = farm.workload(kind, **kw)
    evaluate, close = farm.gpu_evaluator(ctx, datasets)
    g = farm.RcclGather(ctx, 1, 0, farm.RcclGather.unique_id(ctx))
    try:
        out = farm.Farm(1, 0, g).run_problems(models, datasets, evaluate)
    finally:
        g.close()
        close()
    np.testing.assert_allclose(out, _oracle_eval(models, datasets), rtol=1e-9)


@pytest.mark.gpu
def test_schedule_setter():
    """lfm_ctx_set_schedule / lfm_ctx_get_schedule: 1 and 3 round-trip, 0 restores the process
    default, anything else is LFM_E_ARG with the context unchanged."""
    from dis_project_amd import _lib

    ctx = _lib.Context(0)
    try:
        ctx.schedule = 1
        assert ctx.schedule == 1
        ctx.schedule = 3
        assert ctx.schedule == 3
        for bad in (2, 4, -1):
            with pytest.raises(_lib.LfmError):
                ctx.schedule = bad
            assert ctx.schedule == 3
        ctx.schedule = 1
        ctx.schedule = 0
        assert ctx.schedule == (1 if os.environ.get("LFM_SCHED") == "1" else 3)
    finally:
        ctx.close()


@pytest.mark.gpu
def test_concurrent_evaluator_c3_full_size():
    """C3 at full size (N = 16384) through the concurrent restart farm bench.py runs: three
    schedule-1 workers in flight (the caller's context among them, switched to schedule 1 and
    restored on close) against one schedule-3 evaluation and the C++ CPU restatement;
    deterministic across calls and independent of which worker took which restart; a worker's
    exception reaches the caller."""
    from dis_project_amd import _lib

    models, datasets = farm.workload("c3", 64, 256, 6)
    s3 = _lib.Context(0)
    try:
        assert s3.schedule == (1 if os.environ.get("LFM_SCHED") == "1" else 3)
        one = farm.ResidentEvaluator(s3, datasets[0])
        single = one(models[:2])
        one.close()
    finally:
        s3.close()
    ctx = _lib.Context(0)
    before = ctx.schedule
    ev = farm.ConcurrentEvaluator(ctx, datasets[0], workers=3)
    try:
        assert ctx.schedule == 1
        a = ev(models)
        b = ev(models[::-1])[::-1]
        np.testing.assert_array_equal(a, b)
        assert np.all(np.isfinite(a))
        np.testing.assert_allclose(a[:2], single, rtol=1e-10)

        class Broken:
            def hyp(self):
                raise RuntimeError("bad hyperparameters")

        with pytest.raises(RuntimeError, match="bad hyperparameters"):
            ev([models[0], Broken(), models[1]])
    finally:
        ev.close()
    assert ctx.schedule == before
    ctx.close()
    from oracle import lfm_cpu

    m, d = models[0], datasets[0]
    v, _ = lfm_cpu.mll(d.X, d.y, m.true_d, m.true_s, m.true_b, m.l, m.obs_stddev, m.jitter,
                       negative=False, threads=16)
    assert abs(a[0] - v) <= 1e-9 * abs(v)
