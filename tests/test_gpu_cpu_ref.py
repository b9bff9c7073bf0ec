"""Full-size cross-check of the GPU MLL against the independent C++ / OpenMP CPU restatement
(oracle/lfm_cpu.cpp: the reference's gram formula with std::erf, a blocked fp64 Cholesky of
its own), both evaluated on the GPU box on the same seeded inputs (configs.c2 /
configs.c3_restarts) — no numpy oracle, no LAPACK on either side.

Tolerances: 1e-9 relative for the C2 base point and C3 restart 0; the ill-conditioned
restart 1 (logdet -7.1e4, quadratic form 7.6e6) and the small-noise point are held to the
north_star 1e-5 (the reference formula's own gram rounding, ~eps M, moves their MLL by up to
~5e-7: tests/test_gpu_full.py)."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c2():
    from dis_project_amd import _lib, configs, farm
    from oracle import lfm_cpu

    lfm_cpu.load()
    work = configs.c2()
    ev = farm.ResidentEvaluator(_lib.get_context(0), work.data)
    yield work, ev
    ev.close()


@pytest.mark.parametrize("case,rtol", [("c2", 1e-9), ("c3_r0", 1e-9), ("c3_r1", 1e-5),
                                       ("c2_j6", 1e-5)])
def test_mll_n16384_gpu_vs_cpp(c2, case, rtol):
    import os

    from dis_project_amd import configs
    from oracle import lfm_cpu

    work, ev = c2
    if case == "c2":
        model = work.model
    elif case == "c2_j6":
        model = work.model.replace(jitter=1e-6, obs_stddev=0.05)
    else:
        model = configs.c3_restarts(work, 2)[int(case[-1])]
    gpu = float(ev([model])[0])
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    cpu, info = lfm_cpu.mll(work.data.X, work.data.y, model.true_d, model.true_s, model.true_b,
                            model.l, model.obs_stddev, model.jitter, threads=min(threads, 32))
    print(f"{case}: gpu {gpu!r} cpu {cpu!r} rel {abs(gpu - cpu) / abs(cpu):.2e} "
          f"(cpu gram {info['t_gram']:.1f} s, chol {info['t_chol']:.1f} s)")
    assert info["fail"] == -1
    assert abs(gpu - cpu) <= rtol * abs(cpu), (gpu, cpu)


def test_mll_n32768_both_schedules_vs_cpp(monkeypatch):
    """Twice configs[1]'s size: 128 genes x 256 timepoints, N = 32768 (an 8.6 GB factor), the
    MLL on schedule 3 (the default) and on schedule 1 (LFM_SCHED=1, the look-ahead on every CU)
    against the C++ restatement at 1e-9 relative, and the two schedules against each other."""
    import os

    from dis_project_amd import _lib, configs, farm
    from oracle import lfm_cpu

    lfm_cpu.load()
    work = configs.grid_workload("synthetic_128x256_fp64", 128, 256, seed_params=2, seed_y=3)
    assert work.n == 32768
    m = work.model
    got = {}
    for sched in ("3", "1"):
        monkeypatch.setenv("LFM_SCHED", sched)
        ctx = _lib.Context(0)
        ev = farm.ResidentEvaluator(ctx, work.data)
        try:
            got[sched] = float(ev([m])[0])
            assert ctx.fallbacks == 0
        finally:
            ev.close()
            ctx.close()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    cpu, info = lfm_cpu.mll(work.data.X, work.data.y, m.true_d, m.true_s, m.true_b, m.l,
                            m.obs_stddev, m.jitter, threads=min(threads, 32))
    print(f"n32768: gpu s3 {got['3']!r} s1 {got['1']!r} cpu {cpu!r} "
          f"(cpu gram {info['t_gram']:.1f} s, chol {info['t_chol']:.1f} s)")
    assert info["fail"] == -1
    for s, v in got.items():
        assert abs(v - cpu) <= 1e-9 * abs(cpu), (s, v, cpu)
    assert abs(got["3"] - got["1"]) <= 1e-9 * abs(cpu)


def test_mll_n65536_both_schedules_vs_cpp_golden(monkeypatch):
    """Four times configs[1]'s size: 256 genes x 256 timepoints, N = 65536 (a 34 GB factor; the
    C4 grid in fp64), on schedule 3 and schedule 1, against the C++ restatement's MLL on the same
    seeded inputs (tests/golden/scale_n65536.json, made by scripts/scale_check.py on the GPU
    box's host in 193 s — too long to repeat per run) at 1e-9 relative, and the schedules
    against each other."""
    import json
    import os

    from dis_project_amd import _lib, configs, farm

    with open(os.path.join(os.path.dirname(__file__), "golden", "scale_n65536.json")) as f:
        g = json.load(f)
    work = configs.grid_workload("synthetic_256x256_fp64", g["genes"], g["timepoints"],
                                 seed_params=g["seed_params"], seed_y=g["seed_y"])
    assert work.n == g["N"] == 65536
    ref = g["mll_cpu_port"]
    got = {}
    for sched in ("3", "1"):
        monkeypatch.setenv("LFM_SCHED", sched)
        ctx = _lib.Context(0)
        ev = farm.ResidentEvaluator(ctx, work.data)
        try:
            got[sched] = float(ev([work.model])[0])
            assert ctx.fallbacks == 0
        finally:
            ev.close()
            ctx.close()
    print(f"n65536: gpu s3 {got['3']!r} s1 {got['1']!r} cpu port {ref!r}")
    for s, v in got.items():
        assert abs(v - ref) <= 1e-9 * abs(ref), (s, v, ref)
    assert abs(got["3"] - got["1"]) <= 1e-9 * abs(ref)
