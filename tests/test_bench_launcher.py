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
    # c5's hyperparameter rounds per rank: configs[4]'s own 15-problem step on one GPU, 16
    # rounds (one launch of 240 problems and one exchange per step) on several
    assert bench.parse(["--workload", "c5"]).rounds == 1
    assert bench.parse(["--gpus", "2", "--workload", "c5"]).rounds == bench.C5_ROUNDS_MULTI == 16
    assert bench.parse(["--gpus", "8", "--workload", "c5", "--rounds", "4"]).rounds == 4


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


def _gather_rank(rank, world, port, fail_rank, q, require=False):
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

        try:
            gather, kind = bench.make_gather(None, world, rank, "rccl", rccl=Stub,
                                             require=require)
        except SystemExit as e:
            q.put((rank, "exit", Stub.closed, str(e)))
            return
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


# ------------------------------------------------- GPU count without the HIP runtime
def _fake_kfd(root, dri, cards):
    """A KFD topology (node 0 a CPU agent) with `cards` GPU nodes and their render nodes.
    cards: list of (unique_id, render node present)."""
    os.makedirs(dri, exist_ok=True)
    n0 = os.path.join(root, "0")
    os.makedirs(n0)
    open(os.path.join(n0, "gpu_id"), "w").write("0\n")
    open(os.path.join(n0, "properties"), "w").write("cpu_cores_count 16\nsimd_count 0\n")
    for i, (uid, ok) in enumerate(cards, start=1):
        d = os.path.join(root, str(i))
        os.makedirs(d)
        open(os.path.join(d, "gpu_id"), "w").write(f"{1000 + i}\n")
        minor = 127 + i
        open(os.path.join(d, "properties"), "w").write(
            f"cpu_cores_count 0\nsimd_count 1024\ndrm_render_minor {minor}\nunique_id {uid}\n")
        if ok:  # a container sees only its own cards' render nodes
            open(os.path.join(dri, f"renderD{minor}"), "w").close()


def _clear_visible(monkeypatch):
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)


def test_visible_gpus_reads_the_kfd_topology(tmp_path, monkeypatch):
    root, dri = str(tmp_path / "nodes"), str(tmp_path / "dri")
    _fake_kfd(root, dri, [(0x11, True), (0x22, True), (0x33, False), (0x44, True)])
    monkeypatch.setenv("LFM_KFD_TOPOLOGY", root)
    monkeypatch.setenv("LFM_DRI_DIR", dri)
    _clear_visible(monkeypatch)
    assert bench.visible_gpus() == 3  # the CPU node and the inaccessible card are not counted


def test_visible_gpus_applies_the_visibility_variables(tmp_path, monkeypatch):
    root, dri = str(tmp_path / "nodes"), str(tmp_path / "dri")
    _fake_kfd(root, dri, [(0xA0 + i, True) for i in range(8)])
    monkeypatch.setenv("LFM_KFD_TOPOLOGY", root)
    monkeypatch.setenv("LFM_DRI_DIR", dri)
    _clear_visible(monkeypatch)
    assert bench.visible_gpus() == 8
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "1,3,5,GPU-a7")
    assert bench.visible_gpus() == 4
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,2")    # indices into ROCr's list
    assert bench.visible_gpus() == 2
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,9,1")  # parsing stops at the invalid index
    assert bench.visible_gpus() == 1
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    monkeypatch.setenv("CUDA_VISIBLE_DEVICES", "")      # empty hides every device
    assert bench.visible_gpus() == 0


def test_launcher_refuses_without_a_topology(tmp_path, rank_script, monkeypatch):
    """No KFD topology: exit 3 with the cause, no rank started — never a HIP-initialising
    fallback count."""
    monkeypatch.setenv("LFM_KFD_TOPOLOGY", str(tmp_path / "absent"))
    a = bench.parse(["--gpus", "2"])
    assert bench.self_launch(a, [str(tmp_path), "ok"], script=rank_script) == 3
    assert not list(tmp_path.glob("rank*.json"))


PROBE = textwrap.dedent("""
    import json, os, subprocess, sys
    sys.path.insert(0, sys.argv[1])
    out, rank_script = sys.argv[2], sys.argv[3]
    real_popen = subprocess.Popen
    state = {}

    def probe(args, **kw):
        # the launcher's state at the moment it starts a rank process
        if not state:
            maps = open("/proc/self/maps").read()
            fds = []
            for fd in os.listdir("/proc/self/fd"):
                try:
                    fds.append(os.readlink(f"/proc/self/fd/{fd}"))
                except OSError:
                    pass
            state.update(hip=[l.split()[-1] for l in maps.splitlines() if "amdhip" in l],
                         torch="torch" in sys.modules,
                         kfd=[f for f in fds if f.startswith("/dev/kfd") or "/dev/dri" in f])
            json.dump(state, open(os.path.join(out, "launcher.json"), "w"))
        return real_popen([sys.executable, rank_script, out, "ok"], **{k: v for k, v in kw.items()
                                                                       if k == "env"})

    subprocess.Popen = probe
    import bench
    sys.exit(bench.main(["--gpus", "2", "--workload", "c5"]))
""")


def test_launcher_process_stays_free_of_hip(tmp_path, rank_script):
    """`python bench.py --gpus 2` in a fresh interpreter, up to the moment it starts its first
    rank process: libamdhip64 is not mapped, torch is not imported and no /dev/kfd or render
    node is open (a parent that initialised HIP must not start GPU processes)."""
    import subprocess

    root, dri = str(tmp_path / "nodes"), str(tmp_path / "dri")
    _fake_kfd(root, dri, [(1, True), (2, True)])
    out = tmp_path / "out"
    out.mkdir()
    probe = tmp_path / "probe.py"
    probe.write_text(PROBE)
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "ROCR_VISIBLE_DEVICES",
                        "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")}
    env.update(LFM_KFD_TOPOLOGY=root, LFM_DRI_DIR=dri)
    r = subprocess.run([sys.executable, str(probe), ROOT, str(out), rank_script], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    st = json.load(open(out / "launcher.json"))
    assert st == {"hip": [], "torch": False, "kfd": []}, st
    assert sorted(p.name for p in out.glob("rank*.json")) == ["rank0.json", "rank1.json"]


def test_require_rccl_defaults(monkeypatch):
    assert bench.parse(["--gpus", "8"]).require_rccl is True
    assert bench.parse(["--gpus", "2", "--share-gpus"]).require_rccl is False
    assert bench.parse(["--gpus", "2", "--gather", "gloo"]).require_rccl is False
    assert bench.parse(["--gpus", "2", "--share-gpus", "--require-rccl"]).require_rccl is True
    assert bench.parse(["--gpus", "8", "--no-require-rccl"]).require_rccl is False


@pytest.mark.parametrize("fail_rank", [0, 1])
def test_require_rccl_ends_the_run_on_every_rank(fail_rank):
    """--require-rccl (the default outside rehearsals): one rank's communicator failure makes
    EVERY rank exit (SystemExit naming the cause) instead of printing a gloo-fallback line; a
    rank whose own communicator came up closes it first."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = bench._free_port()
    ps = [ctx.Process(target=_gather_rank, args=(r, 2, port, fail_rank, q, True))
          for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, kind, closed, msg in res:
        assert kind == "exit", (rank, kind)
        assert "RCCL communicator unavailable" in msg and "--require-rccl" in msg
        if rank == fail_rank:
            assert "stand-in failure" in msg
        else:
            assert "failed on another rank" in msg and closed
