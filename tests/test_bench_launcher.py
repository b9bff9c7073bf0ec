"""bench.py's self-launch (``python bench.py --gpus N`` without torch.distributed.run): the
parent starts N rank processes with the torch.distributed environment, never touches a GPU,
and propagates the first failure (stopping the other ranks). CPU only: the rank processes here
are a stand-in script that reports its environment."""

import json
import os
import sys
import textwrap
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

RANK_SCRIPT = textwrap.dedent("""
    import json, os, sys, time
    out = sys.argv[1]
    rank = int(os.environ["RANK"])
    keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
    with open(os.path.join(out, f"rank{rank}.json"), "w") as f:
        json.dump({k: os.environ.get(k) for k in keys} | {"argv": sys.argv[1:]}, f)
    mode = sys.argv[2]
    if mode == "fail1" and rank == 1:
        sys.exit(7)
    if mode == "fail1":
        time.sleep(120)   # must be stopped by the launcher
    if mode == "signal" and rank == 0:
        os.kill(os.getpid(), 9)
    sys.exit(0)
""")


@pytest.fixture
def rank_script(tmp_path):
    p = tmp_path / "rank.py"
    p.write_text(RANK_SCRIPT)
    return str(p)


def _args(n, extra=()):
    return bench.parse(["--gpus", str(n), "--share-gpus", "--gather", "gloo", *extra])


def test_default_workload_follows_gpu_count():
    assert bench.parse([]).workload == "c2"
    assert bench.parse(["--gpus", "8"]).workload == "c3"
    assert bench.parse(["--gpus", "2", "--workload", "c5"]).workload == "c5"
    assert bench.parse(["--workload", "c4"]).genes == 256
    assert bench.parse(["--workload", "c3"]).genes == 64


def test_launcher_wires_every_rank(tmp_path, rank_script):
    out = tmp_path / "out"
    out.mkdir()
    rc = bench.self_launch(_args(3), [str(out), "ok"], script=rank_script)
    assert rc == 0
    envs = [json.load(open(out / f"rank{r}.json")) for r in range(3)]
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]
    assert {e["WORLD_SIZE"] for e in envs} == {"3"}
    assert {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in envs}) == 1
    assert all(e["argv"] == [str(out), "ok"] for e in envs)


def test_launcher_propagates_a_rank_failure_and_stops_the_rest(tmp_path, rank_script):
    out = tmp_path / "out"
    out.mkdir()
    t0 = time.monotonic()
    rc = bench.self_launch(_args(2), [str(out), "fail1"], script=rank_script)
    assert rc == 7
    assert time.monotonic() - t0 < 60, "the sleeping rank was not stopped"


def test_launcher_reports_a_killed_rank(tmp_path, rank_script):
    out = tmp_path / "out"
    out.mkdir()
    rc = bench.self_launch(_args(2), [str(out), "signal"], script=rank_script)
    assert rc == 128 + 9


def test_launcher_refuses_more_gpus_than_visible(tmp_path, rank_script, monkeypatch):
    monkeypatch.setattr(bench, "visible_gpus", lambda: 1)
    a = bench.parse(["--gpus", "2"])
    assert bench.self_launch(a, ["x", "ok"], script=rank_script) == 3
    assert not list(tmp_path.glob("rank*.json"))


def test_rank_processes_do_not_relaunch(monkeypatch):
    """With WORLD_SIZE set (a rank, or torch.distributed.run) main() runs the rank path: a
    mismatch between --gpus and WORLD_SIZE is refused before any GPU work."""
    monkeypatch.setenv("WORLD_SIZE", "3")
    monkeypatch.setenv("RANK", "0")
    with pytest.raises(SystemExit, match="WORLD_SIZE=3"):
        bench.main(["--gpus", "2"])


def _gather_rank(rank, world, port, fail_rank, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        class Stub:
            """Stands in for farm.RcclGather (no GPU here): fails on `fail_rank`."""

            closed = False

            def __init__(self, ctx, world, rank, uid):
                if rank == fail_rank:
                    raise RuntimeError("LFM_E_RCCL: stand-in failure")

            def __call__(self, send):
                raise AssertionError("the failed communicator must not be used")

            def close(self):
                Stub.closed = True

        import numpy as np

        gather, kind = bench.make_gather(None, world, rank, "rccl", rccl=Stub)
        recv = None if kind == "rccl" else gather(np.array([float(rank), float(10 + rank)]))
        q.put((rank, kind, Stub.closed, None if recv is None else recv.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fail_rank", [0, 1, -1])
def test_gather_falls_back_to_gloo_on_every_rank(fail_rank):
    """bench.make_gather: when any rank's RCCL communicator fails to initialise, every rank
    (agreeing over the gloo control plane) exchanges its slots over gloo and labels the line
    "gloo-fallback"; a rank whose own communicator came up closes it. With no failure every
    rank keeps the communicator ("rccl")."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = bench._free_port()
    ps = [ctx.Process(target=_gather_rank, args=(r, 2, port, fail_rank, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, kind, closed, recv in res:
        if fail_rank < 0:
            assert kind == "rccl" and not closed  # the communicator is kept
            continue
        assert kind == "gloo-fallback"
        assert recv == [0.0, 10.0, 1.0, 11.0]
        assert closed == (rank != fail_rank)
