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
