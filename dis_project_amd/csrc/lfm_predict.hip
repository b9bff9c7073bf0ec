// lfm_predict.hip — GP posterior at test inputs on gfx950.
//
// Reference: ExactLFM.latent_predict / multi_gene_predict, src/model.py:420-514:
//     mean = m(t) + K(t,x) S^{-1} (y - m(x)),   cov = K(t,t) - K(t,x) S^{-1} K(x,t),
//     S = K(x,x) + diag(v) + c I.
// Both are one Schur complement. The matrix
//     [ S        .      . ]   rows [0, n)
//     [ I        .      . ]   rows [n, Np)        identity padding, Np = round_up(n, 128)
//     [ K(t,x)   K(t,t) . ]   rows [Np, Np + m)
//     [ r^T      0      1 ]   row  Np + m         r = y - m(x)
// is factored through the block columns holding S (chol_factor_solve, CHOL_SCHUR): the
// panel solves turn K(t,x) into V = K(t,x) L^{-T} and r into z = L^{-1} r, and the trailing
// updates leave K(t,t) - V V^T (the covariance, lower triangle) in rows [Np, Np + m) and
// -V z (minus the mean correction) in row Np + m. Same three kernels as the MLL, no extra
// solve pass.
#include "lfm_math.h"

namespace lfm {

// Everything except the two gram blocks: the diagonal vector of S, identity padding, the
// zero gaps beside K(t,x), the residual row and the padding rows below it.
__global__ void posterior_fill_kernel(HypDev p, const double* __restrict__ x,
                                      const double* __restrict__ y,
                                      const double* __restrict__ dv, int64_t n, int64_t Np,
                                      int64_t m, double* __restrict__ A, int64_t lda,
                                      int64_t Mtot) {
  const int64_t row = blockIdx.y;
  const int64_t R = Np + m;
  const int64_t bs = n / p.G;
  double* a = A + row * lda;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c <= row;
       c += (int64_t)gridDim.x * blockDim.x) {
    if (row < n) {
      if (c == row && dv) a[c] += dv[row];  // S = K + c I (gram fill) + diag(v)
    } else if (row < Np) {
      a[c] = (c == row) ? 1.0 : 0.0;
    } else if (row < R) {
      if (c >= n && c < Np) a[c] = 0.0;
    } else if (row == R) {
      a[c] = c < n ? y[c] - mean_at(p, x, c, bs) : (c == R ? 1.0 : 0.0);
    } else {
      a[c] = (c == row) ? 1.0 : 0.0;
    }
  }
}

// mean[q] = m(t)[q] - A[R][Np + q];  cov = the lower triangle of rows [Np, Np + m), mirrored.
__global__ void posterior_extract_kernel(HypDev p, const double* __restrict__ t, int64_t m,
                                         const double* __restrict__ A, int64_t lda, int64_t Np,
                                         double* __restrict__ mean, double* __restrict__ cov) {
  const int64_t q = blockIdx.y;
  const double* a = A + (Np + q) * lda + Np;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < m;
       c += (int64_t)gridDim.x * blockDim.x) {
    const double v = c <= q ? a[c] : A[(Np + c) * lda + Np + q];
    cov[q * m + c] = v;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const int64_t bs = m / p.G;
    mean[q] = mean_at(p, t, q, bs) - A[(Np + m) * lda + Np + q];
  }
}

int posterior_blocked(lfm_ctx* ctx, const HypDev& h, const double* d_x, const double* d_y,
                      int64_t n, const double* d_dv, double diag_add, const double* d_t, int64_t m,
                      double* d_mean, double* d_cov) {
  const int64_t Np = (n + 127) / 128 * 128;
  const int64_t Mtot = (Np + m + 1 + 127) / 128 * 128;
  int r = ensure(ctx, (void**)&ctx->A, &ctx->A_bytes, (size_t)Mtot * Mtot * sizeof(double));
  if (r) return r;
  double* A = ctx->A;
  r = launch_gram_direct<double>(ctx, h, d_x, n, d_x, n, diag_add, 0.0, LFM_UPLO_LOWER, A, Mtot);
  if (r) return r;
  r = launch_gram_direct<double>(ctx, h, d_t, m, d_x, n, 0.0, 0.0, LFM_UPLO_FULL, A + Np * Mtot,
                                 Mtot);
  if (r) return r;
  r = launch_gram_direct<double>(ctx, h, d_t, m, d_t, m, 0.0, 0.0, LFM_UPLO_LOWER,
                                 A + Np * Mtot + Np, Mtot);
  if (r) return r;
  dim3 grid((unsigned)std::min<int64_t>((Mtot + 255) / 256, 64), (unsigned)Mtot);
  hipLaunchKernelGGL(posterior_fill_kernel, grid, dim3(256), 0, ctx->stream, h, d_x, d_y, d_dv,
                     n, Np, m, A, Mtot, Mtot);
  r = hip_fail(ctx, hipGetLastError(), "posterior_fill_kernel");
  if (r) return r;
  r = chol_factor_solve(ctx, A, Mtot, n, Mtot, 0, ctx->result, CHOL_SCHUR);
  if (r) return r;
  dim3 g2((unsigned)std::min<int64_t>((m + 255) / 256, 64), (unsigned)m);
  hipLaunchKernelGGL(posterior_extract_kernel, g2, dim3(256), 0, ctx->stream, h, d_t, m, A, Mtot,
                     Np, d_mean, d_cov);
  return hip_fail(ctx, hipGetLastError(), "posterior_extract_kernel");
}

}  // namespace lfm
