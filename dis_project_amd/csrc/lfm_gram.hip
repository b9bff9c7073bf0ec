// lfm_gram.hip — SIM multi-output covariance (gram / cross-covariance) on gfx950.
//
// Reference: ExactLFM.kernel / kernel_xx / kernel_xf / kernel_ff / h / gamma /
// cross_covariance / gram in wejpurvis/DIS_project src/model.py:152-414, and
// mean_function model.py:124-149.
//
// Two fill kernels:
//   gram_grid_kernel   — x in the dataset_3d block layout with a uniform time grid
//                        (the reference's linspace(0,12,T), dataset.py:108). Every
//                        transcendental of h() is separable per (gene, time) or
//                        depends on (gene, tau'-tau) only, so it is read from small
//                        per-gene tables built once per call (tables_kernel); the
//                        element itself costs ~10 FMAs and one coalesced store.
//                        Bound: HBM write bandwidth (8 B per fp64 element).
//   gram_direct_kernel — any x, any flags: evaluates the flag-switched kernel of
//                        model.py:152-195 per pair with erf/exp (only the branches
//                        whose switch is non-zero).
#include "lfm_math.h"

namespace lfm {

// ---------------------------------------------------------------- tables
// The two h() calls of kernel_xx (model.py:231, 343-363) separate into per-gene tables.
// Each erf sum of h is rewritten with exact complementary-error-function identities,
//   erf(a - g) + erf(b + g) = erfc(g - a) - erfc(b + g),
//   erf(t/l - g) + erf(g)   = erfc(g - t/l) - erfc(g),
// so no table entry is the difference of two numbers near +-1 scaled by e^{g^2 - D*delta}
// (the reference's own evaluation of those entries loses ~1e-16 * e^{g^2 + D*12}
// absolutely; these tables do not, which also makes the fp32 gram usable).
// Layout (doubles), W = 2T-1, d = tau' - tau in [-(T-1), T-1], delta = d * dt, g = D l / 2:
//   Wt[g][d]   = e^{g^2 - D delta} erfc(g - delta/l)      G*W
//   Xt[g][d]   = e^{g^2 - D delta}                        G*W
//   Pt[g][tau] = erfc(t_tau / l + g)                      G*T
//   Et[g][tau] = e^{-D t_tau}                             G*T
//   Qt[g][tau] = e^{g^2} (erfc(g - t_tau/l) - erfc(g))    G*T
//   Cm[j][k]   = S_j S_k l sqrt(pi)/2 / (D_j + D_k)       G*G
// kxx(j,tau; k,tau') = Cm[j][k] * ( Wt[k][d] - Xt[k][d] Pt[k][tau] + Wt[j][-d]
//        - Xt[j][-d] Pt[j][tau'] - Et[k][tau'] Et[j][tau] (Qt[k][tau'] + Qt[j][tau]) ).
size_t tables_doubles(int G, int T) {
  const size_t W = 2 * (size_t)T - 1;
  return 2 * (size_t)G * W + 3 * (size_t)G * T + (size_t)G * G;
}

__global__ void tables_kernel(HypDev p, int T, double dt, const double* __restrict__ times,
                              double* __restrict__ tab, float* __restrict__ tab32) {
  const int64_t W = 2 * (int64_t)T - 1;
  const int64_t total = 2 * (int64_t)p.G * W + 3 * (int64_t)p.G * T + (int64_t)p.G * p.G;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const double v = grid_table_entry(p, T, dt, times, idx);
    tab[idx] = v;
    if (tab32) tab32[idx] = (float)v;
  }
}

int launch_tables(lfm_ctx* ctx, const HypDev& h, const GridLayout& lay, const double* d_times,
                  double* tab) {
  const size_t total = tables_doubles(h.G, lay.T);
  float* t32 = nullptr;
  hipEvent_t ev;
  prof_begin(ctx, K_TABLES, &ev);
  int blocks = (int)std::min<size_t>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(tables_kernel, dim3(blocks), dim3(256), 0, ctx->stream, h, lay.T, lay.dt,
                     d_times, tab, t32);
  prof_end(ctx, K_TABLES, ev, 0, (double)total * 8);
  return hip_fail(ctx, hipGetLastError(), "tables_kernel");
}

// ------------------------------------------------------------ grid gram
// One workgroup = 256 consecutive columns x GR rows; a thread owns one column and
// walks the rows, so every row store is one fully coalesced 2 KiB (fp64) segment.
// Row quantities (block, tau, gene j) are wave-uniform; column quantities are per lane.
template <typename T, int GR>
__global__ __launch_bounds__(256) void gram_grid_kernel(
    const T* __restrict__ tab, int G, int Tn, const int* __restrict__ bg, int64_t n, T da1, T da2,
    int lower, T* __restrict__ out, int64_t ldo) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.y * GR;
  if (lower && (int64_t)blockIdx.x * 256 > r0 + GR - 1) return;  // tile entirely above diagonal
  if (c >= n) return;
  const int W = 2 * Tn - 1;
  const T* Wt = tab;
  const T* Xt = Wt + (int64_t)G * W;
  const T* Pt = Xt + (int64_t)G * W;
  const T* Et = Pt + (int64_t)G * Tn;
  const T* Qt = Et + (int64_t)G * Tn;
  const T* Cm = Qt + (int64_t)G * Tn;

  const int bc = (int)(c / Tn);
  const int tp = (int)(c - (int64_t)bc * Tn);
  const int k = bg[bc];
  const T* Wk = Wt + (int64_t)k * W + (Tn - 1);
  const T* Xk = Xt + (int64_t)k * W + (Tn - 1);
  const T* Pk = Pt + (int64_t)k * Tn;
  const T Ek = Et[(int64_t)k * Tn + tp];
  const T Qk = Qt[(int64_t)k * Tn + tp];

  int jprev = -1;
  T Cjk = 0, Pj_tp = 0;
  const T* Wj = Wt;
  const T* Xj = Xt;
  const int64_t rend = min(r0 + GR, n);
  for (int64_t i = r0; i < rend; ++i) {
    if (lower && c > i) continue;
    const int bi = (int)(i / Tn);
    const int tau = (int)(i - (int64_t)bi * Tn);
    const int j = bg[bi];
    if (j != jprev) {
      jprev = j;
      Cjk = Cm[(int64_t)j * G + k];
      Pj_tp = Pt[(int64_t)j * Tn + tp];
      Wj = Wt + (int64_t)j * W + (Tn - 1);
      Xj = Xt + (int64_t)j * W + (Tn - 1);
    }
    const T Ej = Et[(int64_t)j * Tn + tau];
    const T Qj = Qt[(int64_t)j * Tn + tau];
    const int d = tp - tau;
    T v = Wk[d] + Wj[-d];
    v = fma(-Xk[d], Pk[tau], v);
    v = fma(-Xj[-d], Pj_tp, v);
    v = fma(-(Ek * Ej), Qk + Qj, v);
    v = Cjk * v;
    if (i == c) v = (v + da1) + da2;
    out[i * ldo + c] = v;
  }
}

// Aligned variant: T % 256 == 0, so a 64-row x 256-column tile lies inside one (gene j,
// gene k) block. The tile's Toeplitz windows of Wt/Xt (d = tau' - tau spans 319 values)
// and its row tables are staged in LDS once; each element then costs 4 conflict-free LDS
// reads (consecutive d across lanes), 3 wave-uniform ones and one coalesced store.
template <typename T>
__global__ __launch_bounds__(256) void gram_grid_aligned_kernel(
    const T* __restrict__ tab, int G, int Tn, const int* __restrict__ bg, int64_t n, T da1, T da2,
    int lower, T* __restrict__ out, int64_t ldo) {
  constexpr int R = 64, C = 256, WIN = C + R - 1;
  __shared__ T sWk[WIN], sXk[WIN], sWj[WIN], sXj[WIN];
  __shared__ T sPk[R], sEj[R], sQj[R];
  int64_t c0, r0;
  if (lower) {
    // 1-D grid over the lower tiles only: 64-row tile row rb = 4 q + r holds q + 1 tiles of
    // 256 columns, so tile rows 4q .. 4q + 3 start at tile index 2 q (q + 1)
    const int64_t b = blockIdx.x;
    int64_t q = (int64_t)((sqrt(2.0 * (double)b + 1.0) - 1.0) * 0.5);
    while (2 * (q + 1) * (q + 2) <= b) ++q;
    while (2 * q * (q + 1) > b) --q;
    const int64_t off = b - 2 * q * (q + 1);
    r0 = (4 * q + off / (q + 1)) * R;
    c0 = (off % (q + 1)) * C;
  } else {
    c0 = (int64_t)blockIdx.x * C;
    r0 = (int64_t)blockIdx.y * R;
  }
  const int tid = threadIdx.x;
  const int W = 2 * Tn - 1;
  const T* Wt = tab;
  const T* Xt = Wt + (int64_t)G * W;
  const T* Pt = Xt + (int64_t)G * W;
  const T* Et = Pt + (int64_t)G * Tn;
  const T* Qt = Et + (int64_t)G * Tn;
  const T* Cm = Qt + (int64_t)G * Tn;
  const int j = bg[r0 / Tn], k = bg[c0 / Tn];
  const int tau0 = (int)(r0 % Tn), tp0 = (int)(c0 % Tn);
  const int dmin = tp0 - tau0 - (R - 1);  // window index e = d - dmin
  for (int e = tid; e < WIN; e += 256) {
    const int d = dmin + e;
    sWk[e] = Wt[(int64_t)k * W + (Tn - 1) + d];
    sXk[e] = Xt[(int64_t)k * W + (Tn - 1) + d];
    sWj[e] = Wt[(int64_t)j * W + (Tn - 1) - d];
    sXj[e] = Xt[(int64_t)j * W + (Tn - 1) - d];
  }
  if (tid < R) {
    sPk[tid] = Pt[(int64_t)k * Tn + tau0 + tid];
    sEj[tid] = Et[(int64_t)j * Tn + tau0 + tid];
    sQj[tid] = Qt[(int64_t)j * Tn + tau0 + tid];
  }
  const int tp = tp0 + tid;
  const T Ek = Et[(int64_t)k * Tn + tp];
  const T Qk = Qt[(int64_t)k * Tn + tp];
  const T Pj = Pt[(int64_t)j * Tn + tp];
  const T Cjk = Cm[(int64_t)j * G + k];
  __syncthreads();
  const int64_t c = c0 + tid;
  T* op = out + r0 * ldo + c;
#pragma unroll 4
  for (int i = 0; i < R; ++i) {
    const int64_t row = r0 + i;
    if (lower && c > row) continue;
    const int e = tid + (R - 1) - i;
    T v = sWk[e] + sWj[e];
    v = fma(-sXk[e], sPk[i], v);
    v = fma(-sXj[e], Pj, v);
    v = fma(-(Ek * sEj[i]), Qk + sQj[i], v);
    v = Cjk * v;
    if (row == c) v = (v + da1) + da2;
    op[(int64_t)i * ldo] = v;
  }
}

#ifdef LFM_GRAM_AB
#include "lfm_gram_ab.inc"  // A/B-only store-shape variants (make EXTRA=-DLFM_GRAM_AB)
#endif

__global__ void f64_to_f32_kernel(const double* __restrict__ a, float* __restrict__ b, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    b[i] = (float)a[i];
}

template <typename OutT>
int launch_gram_grid(lfm_ctx* ctx, const HypDev& h, const GridLayout& lay, const double* tab,
                     const int* bg, int64_t n, double da1, double da2, int uplo, OutT* out,
                     int64_t ldo) {
  constexpr int GR = 32;
  const OutT* tabT;
  if constexpr (sizeof(OutT) == 8) {
    tabT = tab;
  } else {
    const size_t nt = tables_doubles(h.G, lay.T);
    int r = ensure(ctx, (void**)&ctx->tab32, &ctx->tab32_bytes, nt * sizeof(float));
    if (r) return r;
    hipLaunchKernelGGL(f64_to_f32_kernel, dim3(256), dim3(256), 0, ctx->stream, tab, ctx->tab32,
                       (int64_t)nt);
    tabT = ctx->tab32;
  }
  const int lower = uplo == LFM_UPLO_LOWER;
  const double elems = lower ? (double)n * (n + 1) / 2 : (double)n * n;
  hipEvent_t ev;
  prof_begin(ctx, K_GRAM_GRID, &ev);
  if (lay.T % 256 == 0) {
    // lower: only the lower tiles are launched (2 Q (Q + 1) of them, Q = n / 256)
    const int64_t Q = n / 256;
    dim3 grid = lower ? dim3((unsigned)(2 * Q * (Q + 1))) : dim3((unsigned)(n / 256), (unsigned)(n / 64));
#ifdef LFM_GRAM_AB
    if (!gram_ab_launch<OutT>(ctx, grid, tabT, h, lay.T, bg, n, da1, da2, lower, out, ldo))
#endif
    hipLaunchKernelGGL((gram_grid_aligned_kernel<OutT>), grid, dim3(256), 0, ctx->stream, tabT,
                       h.G, lay.T, bg, n, (OutT)da1, (OutT)da2, lower, out, ldo);
  } else {
    dim3 grid((unsigned)((n + 255) / 256), (unsigned)((n + GR - 1) / GR));
    hipLaunchKernelGGL((gram_grid_kernel<OutT, GR>), grid, dim3(256), 0, ctx->stream, tabT, h.G,
                       lay.T, bg, n, (OutT)da1, (OutT)da2, lower, out, ldo);
  }
  prof_end(ctx, K_GRAM_GRID, ev, 0, elems * sizeof(OutT));
  return hip_fail(ctx, hipGetLastError(), "gram_grid_kernel");
}

// Lower elements (c <= r) of rows [r0, r1) x columns [c0, c1) of the aligned-grid gram, one
// thread per element from the tables in global memory, with gram_grid_aligned_kernel's
// arithmetic (bit-identical). The fused factorisation writes only these blocks.
__global__ __launch_bounds__(256) void gram_region_kernel(GramGen g, int64_t r0, int64_t c0,
                                                          int64_t nr, int64_t nc, double* out,
                                                          int64_t ldo) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= nr * nc) return;
  const int64_t r = r0 + idx / nc, c = c0 + idx % nc;
  if (c > r) return;
  const int Tn = g.Tn, G = g.G;
  const int64_t W = 2 * (int64_t)Tn - 1;
  const double* Wt = g.tab;
  const double* Xt = Wt + (int64_t)G * W;
  const double* Pt = Xt + (int64_t)G * W;
  const double* Et = Pt + (int64_t)G * Tn;
  const double* Qt = Et + (int64_t)G * Tn;
  const double* Cm = Qt + (int64_t)G * Tn;
  const int j = g.bg[r / Tn], k = g.bg[c / Tn];
  const int tau = (int)(r % Tn), tp = (int)(c % Tn), d = tp - tau;
  double v = Wt[k * W + (Tn - 1) + d] + Wt[j * W + (Tn - 1) - d];
  v = fma(-Xt[k * W + (Tn - 1) + d], Pt[(int64_t)k * Tn + tau], v);
  v = fma(-Xt[j * W + (Tn - 1) - d], Pt[(int64_t)j * Tn + tp], v);
  v = fma(-(Et[(int64_t)k * Tn + tp] * Et[(int64_t)j * Tn + tau]),
          Qt[(int64_t)k * Tn + tp] + Qt[(int64_t)j * Tn + tau], v);
  v = Cm[(int64_t)j * G + k] * v;
  if (r == c) v = (v + g.da1) + g.da2;
  out[r * ldo + c] = v;
}

int launch_gram_region(lfm_ctx* ctx, const GramGen& g, int64_t r0, int64_t r1, int64_t c0,
                       int64_t c1, double* out, int64_t ldo) {
  const int64_t nr = r1 - r0, nc = c1 - c0;
  if (nr <= 0 || nc <= 0) return LFM_OK;
  hipEvent_t ev;
  prof_begin(ctx, K_GRAM_GRID, &ev);
  hipLaunchKernelGGL(gram_region_kernel, dim3((unsigned)((nr * nc + 255) / 256)), dim3(256), 0,
                     ctx->stream, g, r0, c0, nr, nc, out, ldo);
  prof_end(ctx, K_GRAM_GRID, ev, 0, (double)nr * nc * 8);
  return hip_fail(ctx, hipGetLastError(), "gram_region_kernel");
}

template int launch_gram_grid<double>(lfm_ctx*, const HypDev&, const GridLayout&, const double*,
                                      const int*, int64_t, double, double, int, double*, int64_t);
template int launch_gram_grid<float>(lfm_ctx*, const HypDev&, const GridLayout&, const double*,
                                     const int*, int64_t, double, double, int, float*, int64_t);

// ----------------------------------------------------------- direct gram
// cross_covariance (model.py:372-394): out[i][c] = kernel(x[i], x2[c]).
template <typename T>
__global__ __launch_bounds__(256) void gram_direct_kernel(HypDev p, const double* __restrict__ x,
                                                          int64_t n, const double* __restrict__ x2,
                                                          int64_t m, double da1, double da2,
                                                          int lower, T* __restrict__ out,
                                                          int64_t ldo) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.y * 8;
  if (c >= m) return;
  const double tb = x2[c * 3 + 0], gb = x2[c * 3 + 1], fb = x2[c * 3 + 2];
  const int64_t rend = min(r0 + 8, n);
  for (int64_t i = r0; i < rend; ++i) {
    if (lower && c > i) continue;
    double v = kernel_ref(p, x[i * 3 + 0], x[i * 3 + 1], x[i * 3 + 2], tb, gb, fb);
    if (i == c) v = (v + da1) + da2;
    out[i * ldo + c] = (T)v;
  }
}

template <typename OutT>
int launch_gram_direct(lfm_ctx* ctx, const HypDev& h, const double* x, int64_t n,
                       const double* x2, int64_t m, double da1, double da2, int uplo,
                       OutT* out, int64_t ldo) {
  dim3 grid((unsigned)((m + 255) / 256), (unsigned)((n + 7) / 8));
  const int lower = uplo == LFM_UPLO_LOWER;
  hipEvent_t ev;
  prof_begin(ctx, K_GRAM_DIRECT, &ev);
  hipLaunchKernelGGL((gram_direct_kernel<OutT>), grid, dim3(256), 0, ctx->stream, h, x, n, x2, m,
                     da1, da2, lower, out, ldo);
  prof_end(ctx, K_GRAM_DIRECT, ev, 0, (double)n * m * sizeof(OutT));
  return hip_fail(ctx, hipGetLastError(), "gram_direct_kernel");
}

template int launch_gram_direct<double>(lfm_ctx*, const HypDev&, const double*, int64_t,
                                        const double*, int64_t, double, double, int, double*,
                                        int64_t);
template int launch_gram_direct<float>(lfm_ctx*, const HypDev&, const double*, int64_t,
                                       const double*, int64_t, double, double, int, float*,
                                       int64_t);

// ---------------------------------------------------------- h (element-wise)
__global__ void h_kernel(HypDev p, const int64_t* __restrict__ j, const int64_t* __restrict__ k,
                         const double* __restrict__ t1, const double* __restrict__ t2, int64_t n,
                         double* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = h_ref(p, gene_index((double)j[i], p.G), gene_index((double)k[i], p.G), t1[i], t2[i]);
}

int launch_h(lfm_ctx* ctx, const HypDev& h, const int64_t* j, const int64_t* k, const double* t1,
             const double* t2, int64_t n, double* out) {
  hipLaunchKernelGGL(h_kernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 1024)), dim3(256),
                     0, ctx->stream, h, j, k, t1, t2, n, out);
  return hip_fail(ctx, hipGetLastError(), "h_kernel");
}

// ------------------------------------------------------------------ mean
__global__ void mean_kernel(HypDev p, const double* __restrict__ x, int64_t n,
                            double* __restrict__ out) {
  const int64_t bs = n / p.G;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = mean_at(p, x, i, bs);
}

int launch_mean(lfm_ctx* ctx, const HypDev& h, const double* x, int64_t n, double* out) {
  hipLaunchKernelGGL(mean_kernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 1024)),
                     dim3(256), 0, ctx->stream, h, x, n, out);
  return hip_fail(ctx, hipGetLastError(), "mean_kernel");
}

// --------------------------------------------------------------- augment
// Row n of the augmented factor holds the residual r = y - m (objectives.py:67,76-78;
// or y - loc for log_prob), so the Cholesky of [[Sigma, .],[r^T, 1]] leaves
// z = L^{-1} r in that row. Rows n+1..Mp-1 are identity padding.
__global__ void augment_kernel(HypDev p, const double* __restrict__ x,
                               const double* __restrict__ y, const double* __restrict__ loc,
                               int64_t n, double* __restrict__ A, int64_t lda, int64_t Mp) {
  const int64_t row = n + blockIdx.y;
  if (row >= Mp) return;
  const int64_t bs = p.G > 0 ? n / p.G : 1;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c <= row;
       c += (int64_t)gridDim.x * blockDim.x) {
    double v;
    if (row == n) {
      if (c < n) v = y[c] - (loc ? loc[c] : mean_at(p, x, c, bs));
      else v = 1.0;
    } else {
      v = (c == row) ? 1.0 : 0.0;
    }
    A[row * lda + c] = v;
  }
}

int launch_augment(lfm_ctx* ctx, const HypDev& h, const double* x, const double* y,
                   const double* loc, int64_t n, double* A, int64_t lda, int64_t Mp) {
  dim3 grid((unsigned)std::min<int64_t>((Mp + 255) / 256, 256), (unsigned)(Mp - n));
  hipEvent_t ev;
  prof_begin(ctx, K_AUGMENT, &ev);
  hipLaunchKernelGGL(augment_kernel, grid, dim3(256), 0, ctx->stream, h, x, y, loc, n, A, lda, Mp);
  prof_end(ctx, K_AUGMENT, ev, 0, (double)(Mp - n) * Mp * 8);
  return hip_fail(ctx, hipGetLastError(), "augment_kernel");
}

}  // namespace lfm
