// lfm_chol.hip — blocked right-looking fp64 Cholesky + solve + logdet on gfx950.
//
// Replaces the arithmetic behind gpjax 0.8.2 GaussianDistribution.log_prob as called
// at src/objectives.py:76-78 (cola Cholesky -> jnp.linalg.cholesky -> LAPACK dpotrf,
// triangular solves, logdet = 2 sum log L_ii):
//     log N(y; m, S) = -1/2 ( n log 2pi + logdet S + r^T S^{-1} r ),  r = y - m.
//
// The factor is stored row-major, lower triangle, leading dimension lda = Mp
// (Mp = n+1 rounded up to 128). Row n holds r (written by augment_kernel), so the
// factorisation of the augmented matrix [[S, .], [r^T, 1]] yields z = L^{-1} r in
// row n: no separate triangular solve pass (quad = ||z||^2). Rows > n are identity.
//
// Per block column k (NB = 128):
//   potrf_diag_kernel  one workgroup: L_kk (in LDS) + L_kk^{-1} (transposed, to linvT),
//                      pivot check, logdet partial. Columns >= n take a unit pivot.
//   trsm_kernel        rows below the block: X = A_ik * L_kk^{-T} as a GEMM on
//                      v_mfma_f64_16x16x4_f64 against linvT.
//   syrk_kernel        trailing lower triangle, 128x128 tiles: C -= P P^T on
//                      v_mfma_f64_16x16x4_f64 (the only dense-flop kernel).
// finalize_kernel reduces logdet + ||z||^2 to the scalar MLL.
#include <climits>

#include "lfm_math.h"

namespace lfm {

typedef double double4v __attribute__((ext_vector_type(4)));

static constexpr int NB = 128;       // panel width (block column)
static constexpr int ST = 128;       // SYRK output tile edge
static constexpr int KB = 16;        // SYRK K-step staged through LDS
static constexpr int STATUS_NONE = INT_MAX;

__device__ __forceinline__ double4v mfma16(double a, double b, double4v c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------- potrf
// One 1024-thread workgroup factors the NB x NB diagonal block held in LDS.
// Right-looking, one barrier per column: in phase c every thread updates its
// trailing elements with the (unscaled) column c and scales column c-1, which no
// one reads in phase c.
__global__ __launch_bounds__(1024) void potrf_diag_kernel(double* __restrict__ A, int64_t lda,
                                                         int64_t kb, int64_t npiv,
                                                         double* __restrict__ linvT,
                                                         double* __restrict__ parts, int k,
                                                         int* __restrict__ status) {
  __shared__ double M[NB][NB + 1];
  __shared__ double xd[NB];  // unscaled pivots during the factorisation, then diag(L^{-1})
  const int tid = threadIdx.x;

  for (int idx = tid; idx < NB * NB; idx += 1024) {
    const int r = idx / NB, q = idx - r * NB;
    M[r][q] = (q <= r) ? A[(kb + r) * lda + kb + q] : 0.0;
  }
  // this thread's lower-triangle elements (row-major enumeration of q <= r)
  constexpr int NEL = NB * (NB + 1) / 2;
  constexpr int SLOTS = (NEL + 1023) / 1024;
  int er[SLOTS], eq[SLOTS];
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) {
    const int e = tid + 1024 * s;
    if (e < NEL) {
      int r = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
      while ((r + 1) * (r + 2) / 2 <= e) ++r;
      while (r * (r + 1) / 2 > e) --r;
      er[s] = r;
      eq[s] = e - r * (r + 1) / 2;
    } else {
      er[s] = -1;
      eq[s] = NB;  // never active
    }
  }
  __syncthreads();

  double logacc = 0.0;  // thread 0 only
  for (int c = 0; c <= NB; ++c) {
    // scale column c-1 (finished in phase c-1)
    if (c > 0) {
      const int cp = c - 1;
      const double dp = xd[cp];
      const double piv = sqrt(dp);
      const double inv = 1.0 / piv;
      for (int r = cp + 1 + tid; r < NB; r += 1024) M[r][cp] *= inv;
      if (tid == 0) {
        M[cp][cp] = piv;
        if (kb + cp < npiv) {
          if (!(dp > 0.0)) atomicMin(status, (int)(kb + cp));
          logacc += 0.5 * log(dp);
        }
      }
    }
    if (c < NB) {
      const double d = (kb + c >= npiv) ? 1.0 : M[c][c];
      if (tid == 0) xd[c] = d;  // read by everyone in phase c+1 only
      const double invd = 1.0 / d;
#pragma unroll
      for (int s = 0; s < SLOTS; ++s) {
        const int r = er[s], q = eq[s];
        if (q > c) M[r][q] -= M[r][c] * M[q][c] * invd;
      }
    }
    __syncthreads();
  }
  // write L (lower triangle incl. diagonal) back
  for (int idx = tid; idx < NB * NB; idx += 1024) {
    const int r = idx / NB, q = idx - r * NB;
    if (q <= r) A[(kb + r) * lda + kb + q] = M[r][q];
  }
  if (tid == 0) parts[k] = logacc;

  // X = L^{-1}: X^T is kept in the (zero) upper triangle of M, diag(X) in xd.
  if (tid < NB) xd[tid] = 1.0 / M[tid][tid];
  // clear the upper triangle (it held zeros already; keep explicit for clarity)
  __syncthreads();
  // row-by-row: X[i][j] = -(sum_{q=j}^{i-1} L[i][q] X[q][j]) / L[i][i], 8 lanes per j
  {
    const int j = tid >> 3, p = tid & 7;
    for (int i = 1; i < NB; ++i) {
      double sum = 0.0;
      if (j < i) {
        for (int q = j + p; q < i; q += 8) {
          const double xqj = (q == j) ? xd[j] : M[j][q];
          sum += M[i][q] * xqj;
        }
      }
      sum += __shfl_xor(sum, 1);
      sum += __shfl_xor(sum, 2);
      sum += __shfl_xor(sum, 4);
      if (j < i && p == 0) M[j][i] = -sum * xd[i];
      __syncthreads();
    }
  }
  // linvT[q][c] = X[c][q]: upper triangular, row-major NB x NB
  for (int idx = tid; idx < NB * NB; idx += 1024) {
    const int q = idx / NB, c = idx - q * NB;
    double v = 0.0;
    if (q < c) v = M[q][c];
    else if (q == c) v = xd[c];
    linvT[idx] = v;
  }
}

// ----------------------------------------------------------------- trsm
// Rows [s, Mp) of block column kb: X = A * L^{-T} = A * linvT (linvT upper triangular).
// 64 rows per 256-thread workgroup; wave w owns 16-column blocks w and 7-w (balanced
// because column block cb needs (cb+1)*4 MFMA k-steps).
__global__ __launch_bounds__(256) void trsm_kernel(double* __restrict__ A, int64_t lda, int64_t s,
                                                   int64_t kb, const double* __restrict__ linvT) {
  __shared__ double sA[64][NB + 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t r0 = s + (int64_t)blockIdx.x * 64;
  for (int idx = tid; idx < 64 * (NB / 2); idx += 256) {
    const int r = idx / (NB / 2), q2 = idx - r * (NB / 2);
    const double2 v = *reinterpret_cast<const double2*>(&A[(r0 + r) * lda + kb + 2 * q2]);
    sA[r][2 * q2] = v.x;
    sA[r][2 * q2 + 1] = v.y;
  }
  __syncthreads();
  const int li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int cb = half == 0 ? w : (NB / 16 - 1 - w);
    double4v acc[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) acc[m] = (double4v){0, 0, 0, 0};
    const int qend = (cb + 1) * 16;
    for (int q0 = 0; q0 < qend; q0 += 4) {
      const double b = linvT[(q0 + lk) * NB + cb * 16 + li];
#pragma unroll
      for (int m = 0; m < 4; ++m) acc[m] = mfma16(sA[m * 16 + li][q0 + lk], b, acc[m]);
    }
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m * 16 + lk + 4 * r;
        A[(r0 + row) * lda + kb + cb * 16 + li] = acc[m][r];
      }
  }
}

// ----------------------------------------------------------------- syrk
// Trailing update of the lower triangle: for 128x128 tiles (ti >= tj) of rows/cols
// starting at s:  C[i][j] -= sum_q P[i][q] P[j][q],  P = A[:, kb:kb+NB].
// 4 waves as 2x2, each 64x64 = 4x4 MFMA tiles of 16x16 accumulated in registers.
// The K dimension (NB) is staged KB columns at a time through LDS, the next stage
// prefetched into registers while the current one feeds the MFMAs.
__global__ __launch_bounds__(256, 2) void syrk_kernel(double* __restrict__ A, int64_t lda,
                                                      int64_t s, int64_t kb) {
  __shared__ double sP[2][ST][KB + 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 1, wc = w & 1;
  const int li = lane & 15, lk = lane >> 4;

  const int64_t b = blockIdx.x;
  int ti = (int)((sqrt(8.0 * (double)b + 1.0) - 1.0) * 0.5);
  while ((int64_t)(ti + 1) * (ti + 2) / 2 <= b) ++ti;
  while ((int64_t)ti * (ti + 1) / 2 > b) --ti;
  const int tj = (int)(b - (int64_t)ti * (ti + 1) / 2);
  const int64_t i0 = s + (int64_t)ti * ST, j0 = s + (int64_t)tj * ST;
  const bool diag = (ti == tj);

  double4v acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = i0 + wr * 64 + m * 16 + lk + 4 * r;
        const int64_t col = j0 + wc * 64 + n * 16 + li;
        acc[m][n][r] = A[row * lda + col];
      }

  // staging map: 2 panels x 128 rows x KB doubles = 8 double2 per thread
  constexpr int CH = KB / 2;  // double2 chunks per row
  double2 pre[8];
  auto gload = [&](int k0) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int idx = tid + 256 * u;  // 0..2047
      const int p = idx >> 10;        // panel
      const int rem = idx & 1023;
      const int row = rem / CH, ch = rem - row * CH;
      const int64_t grow = (p ? j0 : i0) + row;
      pre[u] = *reinterpret_cast<const double2*>(&A[grow * lda + kb + k0 + 2 * ch]);
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int idx = tid + 256 * u;
      const int p = idx >> 10;
      const int rem = idx & 1023;
      const int row = rem / CH, ch = rem - row * CH;
      sP[p][row][2 * ch] = pre[u].x;
      sP[p][row][2 * ch + 1] = pre[u].y;
    }
  };

  gload(0);
  for (int k0 = 0; k0 < NB; k0 += KB) {
    __syncthreads();
    lstore();
    __syncthreads();
    if (k0 + KB < NB) gload(k0 + KB);
#pragma unroll
    for (int kk = 0; kk < KB; kk += 4) {
      double a[4], bb[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) a[m] = -sP[0][wr * 64 + m * 16 + li][kk + lk];
#pragma unroll
      for (int n = 0; n < 4; ++n) bb[n] = sP[1][wc * 64 + n * 16 + li][kk + lk];
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = mfma16(a[m], bb[n], acc[m][n]);
    }
  }

#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = i0 + wr * 64 + m * 16 + lk + 4 * r;
        const int64_t col = j0 + wc * 64 + n * 16 + li;
        if (!diag || col <= row) A[row * lda + col] = acc[m][n][r];
      }
}

// ------------------------------------------------------------- finalize
__global__ __launch_bounds__(1024) void finalize_kernel(const double* __restrict__ A, int64_t lda,
                                                        int64_t n, const double* __restrict__ parts,
                                                        int nparts, const int* __restrict__ status,
                                                        int negative, double* __restrict__ out) {
  __shared__ double red[2][16];
  const int tid = threadIdx.x;
  double q = 0.0, ld = 0.0;
  for (int64_t c = tid; c < n; c += 1024) {
    const double z = A[n * lda + c];
    q += z * z;
  }
  for (int k = tid; k < nparts; k += 1024) ld += parts[k];
  for (int o = 32; o > 0; o >>= 1) {
    q += __shfl_xor(q, o);
    ld += __shfl_xor(ld, o);
  }
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = q;
    red[1][tid >> 6] = ld;
  }
  __syncthreads();
  if (tid == 0) {
    double Q = 0.0, LD = 0.0;
    for (int i = 0; i < 16; ++i) {
      Q += red[0][i];
      LD += red[1][i];
    }
    const double logdet = 2.0 * LD;
    const double two_pi = 6.283185307179586476925;
    double mll = -0.5 * ((double)n * log(two_pi) + logdet + Q);
    mll *= negative ? -1.0 : 1.0;
    if (status[0] != STATUS_NONE) mll = __builtin_nan("");
    out[0] = mll;
    out[1] = logdet;
    out[2] = Q;
    out[3] = (double)status[0];
  }
}

__global__ void status_init_kernel(int* st) { st[0] = STATUS_NONE; }

int chol_factor_solve(lfm_ctx* ctx, double* A, int64_t lda, int64_t n, int64_t Mp, int negative,
                      double* d_out) {
  const int64_t npb = (n + NB - 1) / NB;  // block columns that hold pivots
  int r = ensure(ctx, (void**)&ctx->parts, &ctx->parts_cap, (size_t)npb * sizeof(double));
  if (r) return r;
  hipStream_t st = ctx->stream;
  hipLaunchKernelGGL(status_init_kernel, dim3(1), dim3(1), 0, st, ctx->status);
  for (int64_t k = 0; k < npb; ++k) {
    const int64_t kb = k * NB;
    hipEvent_t ev;
    prof_begin(ctx, K_POTRF, &ev);
    hipLaunchKernelGGL(potrf_diag_kernel, dim3(1), dim3(1024), 0, st, A, lda, kb, n, ctx->linvT,
                       ctx->parts, (int)k, ctx->status);
    prof_end(ctx, K_POTRF, ev, (double)NB * NB * NB / 3.0 + (double)NB * NB * NB / 3.0, 0);
    const int64_t s = kb + NB;
    if (s < Mp) {
      const int64_t rows = Mp - s;
      prof_begin(ctx, K_TRSM, &ev);
      hipLaunchKernelGGL(trsm_kernel, dim3((unsigned)(rows / 64)), dim3(256), 0, st, A, lda, s, kb,
                         ctx->linvT);
      prof_end(ctx, K_TRSM, ev, (double)rows * NB * NB, 2.0 * rows * NB * 8);
    }
    if (k + 1 < npb) {
      const int64_t T = (Mp - s) / ST;
      const int64_t tiles = T * (T + 1) / 2;
      const double m = (double)(Mp - s);
      prof_begin(ctx, K_SYRK, &ev);
      hipLaunchKernelGGL(syrk_kernel, dim3((unsigned)tiles), dim3(256), 0, st, A, lda, s, kb);
      // algorithmic: lower triangle m(m+1)/2 outputs x NB FMAs; bytes: C read+write
      prof_end(ctx, K_SYRK, ev, m * (m + 1) * NB, m * (m + 1) / 2 * 16.0);
    }
    r = hip_fail(ctx, hipGetLastError(), "cholesky launch");
    if (r) return r;
  }
  hipEvent_t ev;
  prof_begin(ctx, K_FINALIZE, &ev);
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(1024), 0, st, A, lda, n, ctx->parts, (int)npb,
                     ctx->status, negative, d_out);
  prof_end(ctx, K_FINALIZE, ev, 0, (double)n * 8);
  return hip_fail(ctx, hipGetLastError(), "finalize_kernel");
}

// ------------------------------------------------------- small-N batch
// One workgroup per problem: Sigma (+ residual row) built and factored in LDS.
// Used for n <= SMALL_MAX (configs 1 and 5: N = 35, 28).

__global__ __launch_bounds__(256) void small_mll_kernel(const SmallProb* __restrict__ probs,
                                                        int negative, double* __restrict__ out,
                                                        int* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const SmallProb P = probs[blockIdx.x];
  const int n = P.n, M = n + 1, ld = n + 2;
  const int tid = threadIdx.x;
  HypDev h{P.D, P.S, P.B, P.G, P.l};
  double* red = sm + (size_t)M * ld;  // [8] reduction scratch + [1] flag
  for (int idx = tid; idx < n * n; idx += 256) {
    const int i = idx / n, c = idx - i * n;
    if (c <= i) {
      const double* xa = P.x + 3 * i;
      const double* xb = P.x + 3 * c;
      double v = kernel_ref(h, xa[0], xa[1], xa[2], xb[0], xb[1], xb[2]);
      if (i == c) v = (v + P.jitter) + P.noise;
      sm[i * ld + c] = v;
    }
  }
  const int64_t bs = n / P.G;
  for (int c = tid; c < n; c += 256) sm[n * ld + c] = P.y[c] - mean_at(h, P.x, c, bs);
  if (tid == 0) red[8] = 0.0;
  __syncthreads();
  for (int c = 0; c < n; ++c) {
    const double d = sm[c * ld + c];
    const double piv = sqrt(d);
    const double inv = 1.0 / piv;
    for (int r = c + 1 + tid; r < M; r += 256) sm[r * ld + c] *= inv;
    if (tid == 0) {
      sm[c * ld + c] = piv;
      if (!(d > 0.0) && red[8] == 0.0) red[8] = (double)(c + 1);
    }
    __syncthreads();
    const int w = M - c - 1;
    for (int idx = tid; idx < w * w; idx += 256) {
      const int r = c + 1 + idx / w, q = c + 1 + idx % w;
      if (q <= r) sm[r * ld + q] -= sm[r * ld + c] * sm[q * ld + c];
    }
    __syncthreads();
  }
  double ldp = 0.0, qp = 0.0;
  for (int c = tid; c < n; c += 256) {
    ldp += log(sm[c * ld + c]);
    const double z = sm[n * ld + c];
    qp += z * z;
  }
  for (int o = 32; o > 0; o >>= 1) {
    ldp += __shfl_xor(ldp, o);
    qp += __shfl_xor(qp, o);
  }
  if ((tid & 63) == 0) {
    red[tid >> 6] = ldp;
    red[4 + (tid >> 6)] = qp;
  }
  __syncthreads();
  if (tid == 0) {
    const double LD = 2.0 * (red[0] + red[1] + red[2] + red[3]);
    const double Q = red[4] + red[5] + red[6] + red[7];
    const double two_pi = 6.283185307179586476925;
    double mll = -0.5 * ((double)n * log(two_pi) + LD + Q);
    mll *= negative ? -1.0 : 1.0;
    int st = 0;
    if (red[8] != 0.0) {
      mll = __builtin_nan("");
      st = (int)red[8];  // 1-based failing pivot
    }
    out[blockIdx.x] = mll;
    if (status) status[blockIdx.x] = st;
  }
}

int launch_small_batch(lfm_ctx* ctx, const SmallProb* d_probs, int nprob, int maxn, int negative,
                       double* d_out, int* d_status) {
  const size_t lds = ((size_t)(maxn + 1) * (maxn + 2) + 16) * sizeof(double);
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&small_mll_kernel),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  hipEvent_t ev;
  prof_begin(ctx, K_SMALL, &ev);
  hipLaunchKernelGGL(small_mll_kernel, dim3(nprob), dim3(256), lds, ctx->stream,
                     d_probs, negative, d_out, d_status);
  prof_end(ctx, K_SMALL, ev, 0, 0);
  return hip_fail(ctx, hipGetLastError(), "small_mll_kernel");
}

}  // namespace lfm
