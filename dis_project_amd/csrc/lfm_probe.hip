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

// 8 independent accumulator chains per wave; the result is kept live via a store.
__global__ __launch_bounds__(256) void mfma_rate_kernel(double* out, int iters, double seed) {
  const int l = threadIdx.x & 63;
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
