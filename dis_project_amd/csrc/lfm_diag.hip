// lfm_diag.hip — liblfm_diag.so, the diagnostics of include/lfm_diag.h, built apart from the
// product library (liblfm.so, which it links against and whose contexts it takes):
// (1) the lane maps of v_mfma_f64_16x16x4_f64 / 4x4x4_4b (checked against host products),
// (2) their sustained issue rates (TFLOP/s) with independent accumulators, (3) the pivot
// rsqrt, (4) the trailing-update kernel alone (through liblfm's launch hook), (5) phase stamps
// of the schedule-3 factorisation, (6) the schedule-3 tenancy state. No product call path
// loads this library.
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "lfm_math.h"

namespace lfm {

typedef double double4v __attribute__((ext_vector_type(4)));

// A: 16x4 row-major, B: 4x16 row-major, D: 16x16 row-major.
// Assumed maps: A[i=l&15][k=l>>4], B[k=l>>4][j=l&15], D[row=(l>>4)+4r][col=l&15].
__global__ void mfma_layout_kernel(const double* a, const double* b, double* d) {
  const int l = threadIdx.x;
  const double av = a[(l & 15) * 4 + (l >> 4)];
  const double bv = b[(l >> 4) * 16 + (l & 15)];
  double4v acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 4; ++r) d[((l >> 4) + 4 * r) * 16 + (l & 15)] = acc[r];
}

// v_mfma_f64_4x4x4_4b_f64 with every (CBSZ, ABID) broadcast setting used by the SYRK:
// one wave, a[64], b[64], c[64] per lane -> d[16][64] for (cbsz, abid) = (0,0), (2,0..3),
// and blgp = 0.
template <int CBSZ, int ABID>
__device__ __forceinline__ double mfma4(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, CBSZ, ABID, 0);
}
__global__ void mfma4_layout_kernel(const double* a, const double* b, const double* c, double* d) {
  const int l = threadIdx.x;
  const double av = a[l], bv = b[l], cv = c[l];
  d[0 * 64 + l] = mfma4<0, 0>(av, bv, cv);
  d[1 * 64 + l] = mfma4<2, 0>(av, bv, cv);
  d[2 * 64 + l] = mfma4<2, 1>(av, bv, cv);
  d[3 * 64 + l] = mfma4<2, 2>(av, bv, cv);
  d[4 * 64 + l] = mfma4<2, 3>(av, bv, cv);
}

int probe_mfma4_layout(lfm_ctx* ctx, const double* a, const double* b, const double* c,
                       double* d) {
  double* dv = nullptr;
  hipError_t e = hipMallocAsync((void**)&dv, (3 * 64 + 5 * 64) * sizeof(double), ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "probe alloc");
  hipMemcpyAsync(dv, a, 64 * 8, hipMemcpyHostToDevice, ctx->stream);
  hipMemcpyAsync(dv + 64, b, 64 * 8, hipMemcpyHostToDevice, ctx->stream);
  hipMemcpyAsync(dv + 128, c, 64 * 8, hipMemcpyHostToDevice, ctx->stream);
  hipLaunchKernelGGL(mfma4_layout_kernel, dim3(1), dim3(64), 0, ctx->stream, dv, dv + 64, dv + 128,
                     dv + 192);
  hipMemcpyAsync(d, dv + 192, 5 * 64 * 8, hipMemcpyDeviceToHost, ctx->stream);
  hipFreeAsync(dv, ctx->stream);
  return hip_fail(ctx, hipStreamSynchronize(ctx->stream), "probe mfma4 layout");
}

// 8 independent accumulator chains per wave; the result is kept live via a store.
// Block 0 / thread 0 stamps s_memtime (shader clock) and s_memrealtime (100 MHz) around
// the loop into out[gridDim.x .. +1].
__global__ __launch_bounds__(256) void mfma_rate_kernel(double* out, int iters, double seed) {
  const int l = threadIdx.x & 63;
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  double a = seed + l * 1e-3, b = seed - l * 1e-3;
  double4v acc[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) acc[u] = (double4v){0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[u], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int u = 0; u < 8; ++u) s += acc[u][0] + acc[u][1] + acc[u][2] + acc[u][3];
  if (s == 12345.678) out[blockIdx.x] = s;  // practically never taken; keeps the chain live
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    out[gridDim.x] = (double)(c1 - c0);
    out[gridDim.x + 1] = (double)(r1 - r0);
  }
}

// VALU fp64: 8 independent v_fma_f64 chains per lane.
__global__ __launch_bounds__(256) void valu_rate_kernel(double* out, int iters, double seed) {
  double a[8], b = 1.0000001, c = seed * 1e-9;
#pragma unroll
  for (int u = 0; u < 8; ++u) a[u] = seed + threadIdx.x * 1e-3 + u;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] = fma(a[u], b, c);
  }
  double s = 0;
#pragma unroll
  for (int u = 0; u < 8; ++u) s += a[u];
  if (s == 12345.678) out[blockIdx.x] = s;
}

// v_mfma_f64_4x4x4_4b_f64 (four 4x4x4 blocks per wave): 8 independent chains.
__global__ __launch_bounds__(256) void mfma4_rate_kernel(double* out, int iters, double seed) {
  const int l = threadIdx.x & 63;
  double a = seed + l * 1e-3, b = seed - l * 1e-3;
  double acc[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) acc[u] = 0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[u] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[u], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int u = 0; u < 8; ++u) s += acc[u];
  if (s == 12345.678) out[blockIdx.x] = s;
}

// Random-operand variants (which = 2: 16x16x4, 3: 4x4x4_4b): 16 pseudo-random operand
// pairs per lane cycled through, so the matrix cores see toggling data (power-limited rate).
__device__ __forceinline__ double hash_val(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return ((double)x * 2.3283064365386963e-10 - 0.5) * 0.0625;
}
template <bool BIG>
__global__ __launch_bounds__(256) void mfma_rand_kernel(double* out, int iters) {
  const unsigned l = threadIdx.x + 256u * blockIdx.x;
  double a[16], b[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    a[u] = hash_val(l * 32u + u);
    b[u] = hash_val(l * 32u + 16u + u);
  }
  double4v acc4[8];
  double acc1[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    acc4[u] = (double4v){0, 0, 0, 0};
    acc1[u] = 0;
  }
  for (int it = 0; it < iters; it += 2) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (BIG) acc4[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[8 * h + u], b[8 * h + u], acc4[u], 0, 0, 0);
        else acc1[u] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[8 * h + u], b[8 * h + u], acc1[u], 0, 0, 0);
      }
  }
  double s = 0;
#pragma unroll
  for (int u = 0; u < 8; ++u) s += BIG ? acc4[u][0] + acc4[u][1] + acc4[u][2] + acc4[u][3] : acc1[u];
  if (s == 12345.678) out[blockIdx.x] = s;
}

int probe_rates(lfm_ctx* ctx, int which, int nblocks, int iters, double* tflops) {
  double* dv = nullptr;
  hipError_t e = hipMallocAsync((void**)&dv, nblocks * sizeof(double), ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "probe alloc");
  auto go = [&](int it) {
    if (which == 0) hipLaunchKernelGGL(valu_rate_kernel, dim3(nblocks), dim3(256), 0, ctx->stream, dv, it, 1.0);
    else if (which == 1) hipLaunchKernelGGL(mfma4_rate_kernel, dim3(nblocks), dim3(256), 0, ctx->stream, dv, it, 1.0);
    else if (which == 2) hipLaunchKernelGGL(mfma_rand_kernel<true>, dim3(nblocks), dim3(256), 0, ctx->stream, dv, it);
    else hipLaunchKernelGGL(mfma_rand_kernel<false>, dim3(nblocks), dim3(256), 0, ctx->stream, dv, it);
  };
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  go(4);
  hipEventRecord(a, ctx->stream);
  go(iters);
  hipEventRecord(b, ctx->stream);
  e = hipStreamSynchronize(ctx->stream);
  float t = 0;
  hipEventElapsedTime(&t, a, b);
  hipEventDestroy(a);
  hipEventDestroy(b);
  hipFreeAsync(dv, ctx->stream);
  hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "probe rates");
  const double per = which == 0 ? 256.0 * 8 * 2
                     : which == 2 ? 4.0 * 8 * (16 * 16 * 4 * 2)
                                  : 4.0 * 8 * (4 * 4 * 4 * 4 * 2);
  *tflops = (double)nblocks * iters * per / (t * 1e-3) / 1e12;
  return LFM_OK;
}

int probe_mfma_f64_cycles(lfm_ctx* ctx, int nblocks, int iters, double* cyc_per_mfma,
                          double* mhz) {
  double* dv = nullptr;
  hipError_t e = hipMallocAsync((void**)&dv, (nblocks + 2) * sizeof(double), ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "probe alloc");
  hipLaunchKernelGGL(mfma_rate_kernel, dim3(nblocks), dim3(256), 0, ctx->stream, dv, iters, 1.0);
  double h[2];
  hipMemcpyAsync(h, dv + nblocks, 2 * sizeof(double), hipMemcpyDeviceToHost, ctx->stream);
  e = hipStreamSynchronize(ctx->stream);
  hipFreeAsync(dv, ctx->stream);
  hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "probe cycles");
  *cyc_per_mfma = h[0] / ((double)iters * 8);
  *mhz = h[0] / h[1] * 100.0;
  return LFM_OK;
}

int probe_mfma_f64_layout(lfm_ctx* ctx, const double* a, const double* b, double* d) {
  double* dv = nullptr;
  hipError_t e = hipMallocAsync((void**)&dv, (64 + 64 + 256) * sizeof(double), ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "probe alloc");
  hipMemcpyAsync(dv, a, 64 * sizeof(double), hipMemcpyHostToDevice, ctx->stream);
  hipMemcpyAsync(dv + 64, b, 64 * sizeof(double), hipMemcpyHostToDevice, ctx->stream);
  hipLaunchKernelGGL(mfma_layout_kernel, dim3(1), dim3(64), 0, ctx->stream, dv, dv + 64, dv + 128);
  hipMemcpyAsync(d, dv + 128, 256 * sizeof(double), hipMemcpyDeviceToHost, ctx->stream);
  hipFreeAsync(dv, ctx->stream);
  return hip_fail(ctx, hipStreamSynchronize(ctx->stream), "probe layout");
}

int probe_mfma_f64(lfm_ctx* ctx, int nblocks, int iters, double* tflops, double* ms) {
  double* dv = nullptr;
  hipError_t e = hipMallocAsync((void**)&dv, nblocks * sizeof(double), ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "probe alloc");
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(mfma_rate_kernel, dim3(nblocks), dim3(256), 0, ctx->stream, dv, 4, 1.0);
  hipEventRecord(a, ctx->stream);
  hipLaunchKernelGGL(mfma_rate_kernel, dim3(nblocks), dim3(256), 0, ctx->stream, dv, iters, 1.0);
  hipEventRecord(b, ctx->stream);
  e = hipStreamSynchronize(ctx->stream);
  float t = 0;
  hipEventElapsedTime(&t, a, b);
  hipEventDestroy(a);
  hipEventDestroy(b);
  hipFreeAsync(dv, ctx->stream);
  hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "probe rate");
  const double flops = (double)nblocks * 4 /*waves*/ * iters * 8 * (16.0 * 16 * 4 * 2);
  *ms = t;
  *tflops = flops / (t * 1e-3) / 1e12;
  return LFM_OK;
}

// Diagnostic: the pivot reciprocal square root of the diagonal factor (v_rsq_f64 + one
// Newton step) over host values x[n] -> y[n] (tests bound its relative error).
__global__ void rsq_probe_kernel(const double* x, double* y, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) y[i] = rsqrt_1nr(x[i]);
}

int probe_rsq(lfm_ctx* ctx, const double* x, int64_t n, double* y) {
  double* d = nullptr;
  hipError_t e = hipMalloc((void**)&d, 2 * n * sizeof(double));
  if (e != hipSuccess) return hip_fail(ctx, e, "probe rsq");
  hipMemcpyAsync(d, x, n * 8, hipMemcpyHostToDevice, ctx->stream);
  hipLaunchKernelGGL(rsq_probe_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream,
                     d, d + n, n);
  hipMemcpyAsync(y, d + n, n * 8, hipMemcpyDeviceToHost, ctx->stream);
  e = hipStreamSynchronize(ctx->stream);
  hipFree(d);
  return hip_fail(ctx, e, "probe rsq");
}

// kernel_ref and KxxTab's kxx_tab (small_mll_kernel's gene-gene pairs) on every pair of x, one
// workgroup: out[0, n^2) from kernel_ref, out[n^2, 2 n^2) from the tables (pairs with a latent
// row: kernel_ref in both halves, as the kernel does). The tables' claim is bit-identity.
__global__ void kxx_tab_probe_kernel(const double* __restrict__ x, int n, const double* hyp, int G,
                                     double* __restrict__ out) {
  extern __shared__ double tb[];
  double* gam = tb;
  double* egg = gam + G;
  double* erg = egg + G;
  double* e2 = erg + G;
  double* e1 = e2 + n;
  const HypDev h{hyp, hyp + G, hyp + 2 * G, G, hyp[3 * G]};
  const KxxTab t{gam, egg, erg, e1, e2, G};
  small_tables(h, x, n, t, gam, egg, erg, e1, e2);
  for (int q = threadIdx.x; q < n * n; q += 256) {
    const int i = q / n, c = q - i * n;
    const double* xa = x + 3 * i;
    const double* xb = x + 3 * c;
    out[q] = kernel_ref(h, xa[0], xa[1], xa[2], xb[0], xb[1], xb[2]);
    out[n * n + q] = flag_int(xa[2]) == 1 && flag_int(xb[2]) == 1
                         ? kxx_tab(h, t, xa[0], gene_index(xa[1], G), i, xb[0],
                                   gene_index(xb[1], G), c)
                         : kernel_ref(h, xa[0], xa[1], xa[2], xb[0], xb[1], xb[2]);
  }
}

int probe_kxx_tab(lfm_ctx* ctx, const double* x, int64_t n, const lfm_hyp* hyp, double* out) {
  const int G = (int)hyp->num_genes;
  const size_t nh = 3 * (size_t)G + 1, nx = 3 * (size_t)n, no = 2 * (size_t)n * n;
  double* d = nullptr;
  hipError_t e = hipMalloc((void**)&d, (nh + nx + no) * sizeof(double));
  if (e != hipSuccess) return hip_fail(ctx, e, "probe kxx tab");
  std::vector<double> hh(nh);
  std::memcpy(hh.data(), hyp->true_d, G * 8);
  std::memcpy(hh.data() + G, hyp->true_s, G * 8);
  std::memcpy(hh.data() + 2 * G, hyp->true_b, G * 8);
  hh[3 * G] = hyp->l;
  hipMemcpyAsync(d, hh.data(), nh * 8, hipMemcpyHostToDevice, ctx->stream);
  hipMemcpyAsync(d + nh, x, nx * 8, hipMemcpyHostToDevice, ctx->stream);
  const size_t lds = (3 * (size_t)G + n + (size_t)n * G) * sizeof(double);
  hipLaunchKernelGGL(kxx_tab_probe_kernel, dim3(1), dim3(256), lds, ctx->stream, d + nh, (int)n,
                     d, G, d + nh + nx);
  hipMemcpyAsync(out, d + nh + nx, no * 8, hipMemcpyDeviceToHost, ctx->stream);
  e = hipStreamSynchronize(ctx->stream);
  hipFree(d);
  return hip_fail(ctx, e, "probe kxx tab");
}

// Pseudo-random doubles in [-1/32, 1/32) (probe data: MFMA power, hence clocks, depends on it).
__global__ void fill_hash_kernel(double* a, int64_t cnt) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < cnt; i += (int64_t)gridDim.x * 256) {
    uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull;
    h ^= h >> 31;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 29;
    a[i] = ((double)(h >> 11) * 0x1.0p-53 - 0.5) * 0.0625;
  }
}

// Average duration (us) of one full-lower-triangle trailing-update launch over a T x T grid of
// 128-tiles with update depth kd (the launch itself: probe_update_launch in liblfm, whose
// comment lists the cio bits; bit 3 here: random operands, else zeros).
int probe_syrk(lfm_ctx* ctx, int T, int kd, int cio, int reps, double* us) {
  constexpr int64_t TILE = 128;
  const int64_t n = (int64_t)T * TILE + 512;
  const size_t xb = (cio & (512 | 256)) ? (size_t)n * 128 * 8 : 0;  // X_s / X_{s+1} slabs
  int r = ensure(ctx, (void**)&ctx->A, &ctx->A_bytes, (size_t)n * n * 8 + 2 * xb + 4096);
  if (r) return r;
  if (cio & 8)
    hipLaunchKernelGGL(fill_hash_kernel, dim3(4096), dim3(256), 0, ctx->stream, ctx->A,
                       n * n + 2 * (int64_t)(xb / 8));
  else
    hipMemsetAsync(ctx->A, 0, (size_t)n * n * 8 + 2 * xb, ctx->stream);
  hipMemsetAsync(ctx->A + (size_t)n * n + 2 * (xb / 8), 0, 4096, ctx->stream);
  hipStream_t st = (cio & 16) && ctx->m3 ? ctx->m3 : ctx->stream;
  if (st != ctx->stream) {
    hipEvent_t f;
    hipEventCreate(&f);
    hipEventRecord(f, ctx->stream);
    hipStreamWaitEvent(st, f, 0);
    hipEventDestroy(f);
  }
  r = probe_update_launch(ctx, st, T, kd, cio, n, xb);
  if (r) return r;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a, st);
  for (int i = 0; i < reps && !r; ++i) r = probe_update_launch(ctx, st, T, kd, cio, n, xb);
  hipEventRecord(b, st);
  hipError_t e = hipStreamSynchronize(st);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  hipEventDestroy(a);
  hipEventDestroy(b);
  if (r) return r;
  *us = ms * 1e3 / reps;
  return hip_fail(ctx, e, "probe_syrk");
}

}  // namespace lfm

using namespace lfm;

namespace {
struct DeviceGuard {
  DeviceGuard(int dev) { hipSetDevice(dev); }
};
}  // namespace

extern "C" {

int lfm_probe_rsq(lfm_ctx* ctx, const double* x, int64_t n, double* y) {
  if (!ctx || !x || !y || n < 1) return LFM_E_ARG;
  DeviceGuard g(ctx->device);
  return probe_rsq(ctx, x, n, y);
}

int lfm_probe_kxx_tab(lfm_ctx* ctx, const double* x, int64_t n, const lfm_hyp* hyp, double* out) {
  if (!ctx || !x || !hyp || !out || n < 1 || n > 63 || hyp->num_genes < 1 || hyp->num_genes > 63)
    return LFM_E_ARG;
  DeviceGuard g(ctx->device);
  return probe_kxx_tab(ctx, x, n, hyp, out);
}

// enable = 1 turns on s_memrealtime (100 MHz) stamps of the schedule-3 chain kernel's phases
// (16 per super-panel step, 256 steps) and of the step launches; enable = 0 copies them out
// and turns them off. The product kernels write them only while ctx->dbg_stamps is set.
int lfm_debug_stamps(lfm_ctx* ctx, int enable, unsigned long long* out, int max) {
  if (!ctx) return LFM_E_ARG;
  DeviceGuard g(ctx->device);
  const size_t cnt = 256 * 24;  // 256 chain rows of 16, then 256 step-launch rows of 8
  if (enable) {
    if (!ctx->dbg_stamps) {
      hipError_t e = hipMalloc((void**)&ctx->dbg_stamps, cnt * 8);
      if (e != hipSuccess) return hip_fail(ctx, e, "debug stamps");
    }
    hipError_t e = hipMemsetAsync(ctx->dbg_stamps, 0, cnt * 8, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    return hip_fail(ctx, e, "debug stamps");
  }
  if (!ctx->dbg_stamps) return LFM_OK;
  hipError_t e = hipStreamSynchronize(ctx->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(out, ctx->dbg_stamps, std::min<size_t>(cnt, (size_t)std::max(max, 0)) * 8,
                       hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  hipFree(ctx->dbg_stamps);
  ctx->dbg_stamps = nullptr;
  return hip_fail(ctx, e, "debug stamps");
}

// cap > 0 turns on the step-kernel unit trace for the next `cap` workgroups (4 words each:
// entry / exit s_memrealtime, HW_ID | XCC_ID << 32, launch tag << 40 | role << 32 | unit);
// cap = 0 copies out min(written, max) records, reports how many were written and turns it off.
int lfm_debug_trace(lfm_ctx* ctx, int64_t cap, unsigned long long* out, int64_t max,
                    int64_t* written) {
  if (!ctx || cap < 0) return LFM_E_ARG;
  DeviceGuard g(ctx->device);
  if (cap > 0) {
    if (ctx->dbg_trace) hipFree(ctx->dbg_trace);
    ctx->dbg_trace = nullptr;
    hipError_t e = hipMalloc((void**)&ctx->dbg_trace, (size_t)cap * 32);
    if (e == hipSuccess) e = hipMemsetAsync(ctx->dbg_trace, 0, (size_t)cap * 32, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) {
      hipFree(ctx->dbg_trace);
      ctx->dbg_trace = nullptr;
      return hip_fail(ctx, e, "debug trace");
    }
    ctx->dbg_trace_cap = cap;
    ctx->dbg_trace_cur = 0;
    ctx->dbg_trace_launch = 0;
    return LFM_OK;
  }
  if (written) *written = ctx->dbg_trace_cur;
  if (!ctx->dbg_trace) return LFM_OK;
  hipError_t e = hipDeviceSynchronize();
  const int64_t nrec = std::min<int64_t>(ctx->dbg_trace_cur, std::max<int64_t>(max, 0));
  if (e == hipSuccess && out && nrec > 0)
    e = hipMemcpy(out, ctx->dbg_trace, (size_t)nrec * 32, hipMemcpyDeviceToHost);
  hipFree(ctx->dbg_trace);
  ctx->dbg_trace = nullptr;
  ctx->dbg_trace_cap = ctx->dbg_trace_cur = 0;
  return hip_fail(ctx, e, "debug trace");
}

int lfm_debug_last_schedule(const lfm_ctx* ctx, int* out) {
  if (!ctx || !out) return LFM_E_ARG;
  *out = ctx->last_sched;
  return LFM_OK;
}

int lfm_debug_lock_path(const lfm_ctx* ctx, char* buf, int len) {
  if (!ctx || !buf || len < 1) return LFM_E_ARG;
  const std::string p = tenancy_lock_path(ctx->device);
  if ((int)p.size() + 1 > len) return LFM_E_ARG;
  std::memcpy(buf, p.c_str(), p.size() + 1);
  return LFM_OK;
}

int lfm_probe_mfma_f64(lfm_ctx* ctx, int nblocks, int iters, double* tflops, double* ms) {
  if (!ctx || !tflops || !ms || nblocks < 1 || iters < 1) return LFM_E_ARG;
  DeviceGuard g(ctx->device);
  return probe_mfma_f64(ctx, nblocks, iters, tflops, ms);
}

int lfm_probe_mfma_f64_cycles(lfm_ctx* ctx, int nblocks, int iters, double* cyc_per_mfma,
                              double* mhz) {
  if (!ctx || !cyc_per_mfma || !mhz || nblocks < 1 || iters < 1) return LFM_E_ARG;
  DeviceGuard g(ctx->device);
  return probe_mfma_f64_cycles(ctx, nblocks, iters, cyc_per_mfma, mhz);
}

int lfm_probe_mfma4_layout(lfm_ctx* ctx, const double* a, const double* b, const double* c,
                           double* d) {
  if (!ctx || !a || !b || !c || !d) return LFM_E_ARG;
  DeviceGuard g(ctx->device);
  return probe_mfma4_layout(ctx, a, b, c, d);
}

int lfm_probe_rate(lfm_ctx* ctx, int which, int nblocks, int iters, double* tflops) {
  if (!ctx || !tflops || nblocks < 1 || iters < 1) return LFM_E_ARG;
  DeviceGuard g(ctx->device);
  return probe_rates(ctx, which, nblocks, iters, tflops);
}

int lfm_probe_syrk(lfm_ctx* ctx, int T, int kd, int cio, int reps, double* us) {
  if (!ctx || !us || T < 1 || reps < 1 || kd < 16 || kd > 2048 || kd % 16) return LFM_E_ARG;
  DeviceGuard g(ctx->device);
  return probe_syrk(ctx, T, kd, cio, reps, us);
}

int lfm_probe_mfma_f64_layout(lfm_ctx* ctx, const double* a, const double* b, double* d) {
  if (!ctx || !a || !b || !d) return LFM_E_ARG;
  DeviceGuard g(ctx->device);
  return probe_mfma_f64_layout(ctx, a, b, d);
}

}  // extern "C"
