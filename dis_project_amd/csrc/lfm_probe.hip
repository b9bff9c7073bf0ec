// lfm_probe.hip — diagnostics for the fp64 matrix-core path used by the Cholesky:
// (1) the lane maps of v_mfma_f64_16x16x4_f64 (checked against a host product with an
//     asymmetric B), (2) its sustained issue rate (TFLOP/s) with independent accumulators.
#include "lfm_internal.h"

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

}  // namespace lfm
