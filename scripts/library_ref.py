"""Vendor-library reference points on the GPU box, beside the step kernel's numbers: what the
ROCm libraries behind torch reach on the same fp64 shapes.

  * DGEMM (hipBLASLt / rocBLAS through torch.matmul, fp64): C (m x m) = A (m x W) B (W x m) at
    the bulk update's shape (m = 16384 - 128 k, W = 640) and a square 8192^3;
  * SYRK-shaped: torch.addmm(C, A, A^T, beta=1, alpha=-1) at m = 16384, W = 640 (the library
    computes the full square, twice the lower triangle's flops; reported on both bases);
  * Cholesky: torch.linalg.cholesky on an SPD fp64 matrix at N = 16384 (the C2 size), flops
    N^3 / 3.

Each is timed with CUDA events over repeated calls after warm-up; the line printed per case
is JSON: {"case", "ms", "tflops", "frac" (of the 78.6 TFLOP/s fp64 matrix peak)}.

    python scripts/library_ref.py [--json out.json]
"""
import json
import sys

import torch

PEAK = 78.6e12


def timed(fn, reps):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    out = []

    def report(case, ms, flops, **kw):
        rec = {"case": case, "ms": ms, "tflops": flops / (ms * 1e-3) / 1e12,
               "frac": flops / (ms * 1e-3) / PEAK, **kw}
        out.append(rec)
        print(json.dumps(rec), flush=True)

    W = 640
    for m in (16384, 12288, 8192, 6144):
        a = torch.randn(m, W, dtype=torch.float64, device=dev, generator=g)
        b = torch.randn(W, m, dtype=torch.float64, device=dev, generator=g)
        c = torch.empty(m, m, dtype=torch.float64, device=dev)
        ms = timed(lambda: torch.matmul(a, b, out=c), 10)
        report(f"dgemm m={m} k={W}", ms, 2.0 * m * m * W)
        del a, b, c
    n = 8192
    a = torch.randn(n, n, dtype=torch.float64, device=dev, generator=g)
    b = torch.randn(n, n, dtype=torch.float64, device=dev, generator=g)
    ms = timed(lambda: torch.matmul(a, b), 5)
    report("dgemm 8192^3", ms, 2.0 * n ** 3)
    del a, b
    m = 16384
    a = torch.randn(m, W, dtype=torch.float64, device=dev, generator=g)
    c = torch.randn(m, m, dtype=torch.float64, device=dev, generator=g)
    ms = timed(lambda: c.addmm_(a, a.t(), beta=1.0, alpha=-1.0), 10)
    report(f"addmm C -= A A^T m={m} k={W} (full square)", ms, 2.0 * m * m * W,
           lower_triangle_tflops=(m * (m + 1) * W) / (ms * 1e-3) / 1e12)
    del a, c
    N = 16384
    x = torch.randn(N, 256, dtype=torch.float64, device=dev, generator=g)
    S = x @ x.t() / 256.0 + torch.eye(N, dtype=torch.float64, device=dev)
    L = torch.empty_like(S)
    ms = timed(lambda: torch.linalg.cholesky(S, out=L), 3)
    report(f"cholesky N={N}", ms, N ** 3 / 3.0, backend=str(torch.backends.cuda.preferred_linalg_library()))
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
