// oracle/lfm_cpu.cpp — TEST INFRASTRUCTURE ONLY: an independent C++ / OpenMP CPU
// restatement of the reference's MLL path, used (a) as the full-size parity check of the
// GPU path on the GPU box (tests/test_gpu_cpu_ref.py) and (b) as bench.py's timed
// `cpu_baseline` (kind "port"). The product library (dis_project_amd/liblfm.so) never links,
// loads or calls it. It shares no code with the HIP path or with oracle/lfm_oracle.py.
//
// What it restates (wejpurvis/DIS_project @ 2024-08-07), in the reference's term order:
//   h            src/model.py:315-365  (4 erf + 3 exp, the cancelling erf sums as written)
//   gamma        src/model.py:367-369
//   kernel_xx    src/model.py:197-235
//   kernel_xf    src/model.py:237-282
//   kernel_ff    src/model.py:284-312  (divides by 2 l, kept)
//   kernel       src/model.py:152-195  (every branch evaluated and multiplied by its integer
//                                      switch, as the reference does under vmap)
//   gram         src/model.py:372-414  (lower triangle only: K is exactly symmetric)
//   mean_function src/model.py:124-149 (block position i / (n / G), not x[:, 1])
//   Sigma        src/objectives.py:66-73 ((K + jitter I) + obs_stddev^2 I)
//   log_prob     gpjax 0.8.2 GaussianDistribution.log_prob as called at objectives.py:76-78:
//                -1/2 (n log 2 pi + 2 sum log L_ii + ||L^{-1} r||^2); a non-positive / NaN
//                pivot gives NaN (JAX semantics: no exception).
// The Cholesky is a blocked right-looking fp64 factorisation of its own (LAPACK dpotrf's
// algorithm, not its code): an unblocked diagonal factor, a row-parallel triangular solve
// of the panel and an OpenMP tile-parallel trailing update with an AVX2/FMA micro-kernel.
// Built with -ffp-contract=off so the kernel formulas round every product like XLA-CPU.
//
// The training step (lfm_cpu_mll_grad, lfm_cpu_fit): jax.value_and_grad of the MLL (trainer.py:126)
// with the kernel's derivatives in (D_row, D_col, l) by forward-mode duals of the same erf-form
// formulas (d erf(u) = 2/sqrt(pi) e^{-u^2} du), Sigma^{-1} explicitly from the Cholesky factor,
// 1/2 tr((a a^T - Sigma^{-1}) dSigma) + a^T dm; then JaxTrainer.fit's loop (trainer.py:162-228)
// with optax.adam as dis_project_amd/trainer.py restates it. The batched fit's CPU baseline
// (bench.py --workload c5fit).
#include <immintrin.h>
#include <omp.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

constexpr double kSqrtPi = 1.7724538509055160273;

// int(x[:, 1]) with JAX gather semantics: truncate, wrap negatives, clamp (model.py:231-232)
inline int64_t gene_index(double g, int64_t G) {
  double t = std::trunc(g);
  if (t < 0) t += (double)G;
  if (std::isnan(t)) t = 0;
  if (t < 0) t = 0;
  if (t > (double)(G - 1)) t = (double)(G - 1);
  return (int64_t)t;
}

inline int64_t flag_int(double f) {
  const double t = std::trunc(f);
  return std::isnan(t) ? 0 : (int64_t)t;
}

struct Hyp {
  const double* D;
  const double* S;
  int64_t G;
  double l;
};

// model.py:315-365
inline double h(const Hyp& p, int64_t j, int64_t k, double t1, double t2) {
  const double l = p.l;
  const double t_dist = t2 - t1;
  const double gk = (p.D[k] * l) / 2;
  const double multiplier = std::exp(gk * gk) / (p.D[j] + p.D[k]);
  const double first_multiplier = std::exp(-p.D[k] * t_dist);
  const double first_erf_terms = std::erf((t_dist / l) - gk) + std::erf(t1 / l + gk);
  const double second_multiplier = std::exp(-(p.D[k] * t2 + p.D[j] * t1));
  const double second_erf_terms = std::erf((t2 / l) - gk) + std::erf(gk);
  return multiplier * (first_multiplier * first_erf_terms - second_multiplier * second_erf_terms);
}

// model.py:197-235
inline double kernel_xx(const Hyp& p, double ta, int64_t ja, double tb, int64_t jb) {
  const double mult = p.S[ja] * p.S[jb] * p.l * kSqrtPi * 0.5;
  return mult * (h(p, jb, ja, tb, ta) + h(p, ja, jb, ta, tb));
}

// model.py:237-282 (the row whose flag is 0 is the latent one)
inline double kernel_xf(const Hyp& p, double ta, double ga, double fa, double tb, double gb) {
  const bool a_lat = fa == 0.0;
  const double t_gene = a_lat ? tb : ta, g_gene = a_lat ? gb : ga, t_lat = a_lat ? ta : tb;
  const int64_t j = gene_index(g_gene, p.G);
  const double t_dist = t_gene - t_lat;
  const double gj = (p.D[j] * p.l) / 2;
  const double first_term = 0.5 * p.l * kSqrtPi * p.S[j];
  const double first_expon_term = std::exp(gj * gj);
  const double second_expon_term = std::exp(-p.D[j] * t_dist);
  const double erf_terms = std::erf((t_dist / p.l) - gj) + std::erf(t_lat / p.l + gj);
  return first_term * first_expon_term * second_expon_term * erf_terms;
}

// model.py:284-312
inline double kernel_ff(const Hyp& p, double ta, double tb) {
  double sq = (ta - tb) * (ta - tb);
  sq = sq / (2 * p.l);
  return std::exp(-sq);
}

// model.py:152-195: all four branches, each times its integer switch
inline double kernel(const Hyp& p, const double* a, const double* b) {
  const int64_t f1 = flag_int(a[2]), f2 = flag_int(b[2]);
  const double s_xx = (double)(f1 * f2), s_ff = (double)((1 - f1) * (1 - f2));
  const double s_xf = (double)(f1 * (1 - f2)), s_fx = (double)((1 - f1) * f2);
  return s_xx * kernel_xx(p, a[0], gene_index(a[1], p.G), b[0], gene_index(b[1], p.G)) +
         s_ff * kernel_ff(p, a[0], b[0]) + s_xf * kernel_xf(p, a[0], a[1], a[2], b[0], b[1]) +
         s_fx * kernel_xf(p, b[0], b[1], b[2], a[0], a[1]);
}

double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

constexpr int NB = 192;  // Cholesky panel width
constexpr int TB = 96;   // trailing-update tile edge (rows and columns; 16 x 6, 12 x 8)

// Unblocked lower Cholesky of the nb x nb diagonal block at A (row-major, lda); returns the
// first failing column or -1.
int64_t potrf_unblocked(double* A, int64_t lda, int64_t nb) {
  for (int64_t c = 0; c < nb; ++c) {
    double d = A[c * lda + c];
    for (int64_t q = 0; q < c; ++q) d -= A[c * lda + q] * A[c * lda + q];
    if (!(d > 0.0)) return c;
    const double piv = std::sqrt(d);
    A[c * lda + c] = piv;
    const double inv = 1.0 / piv;
    for (int64_t r = c + 1; r < nb; ++r) {
      double v = A[r * lda + c];
      for (int64_t q = 0; q < c; ++q) v -= A[r * lda + q] * A[c * lda + q];
      A[r * lda + c] = v * inv;
    }
  }
  return -1;
}

// C[rows x cols tile] -= P_i P_j^T, both panels packed (BLIS-style micro-panels):
//   PA: the tile's rows in groups of 6, element (r, q) at PA[(r / 6) * 6 kd + 6 q + r % 6]
//   PT: P_j transposed, element (q, j) at PT[q * ldp + j]
// An AVX2 6 x 8 register-blocked micro-kernel (12 accumulators + 2 B vectors + 1 broadcast:
// the 16 ymm registers). Only elements with col <= row matter on diagonal tiles; the rest of
// such a tile is scratch above the diagonal.
void tile_update(double* C, int64_t ldc, const double* PA, const double* PT, int64_t ldp, int kd,
                 int rows, int cols) {
  for (int r = 0; r < rows; r += 6) {
    const int rr = std::min(6, rows - r);
    const double* pa0 = PA + (int64_t)(r / 6) * 6 * kd;
    for (int c = 0; c < cols; c += 8) {
      __m256d c00 = _mm256_setzero_pd(), c01 = c00, c10 = c00, c11 = c00, c20 = c00, c21 = c00;
      __m256d c30 = c00, c31 = c00, c40 = c00, c41 = c00, c50 = c00, c51 = c00;
      const double* bt = PT + c;
      const double* pa = pa0;
      for (int q = 0; q < kd; ++q, bt += ldp, pa += 6) {
        const __m256d b0 = _mm256_loadu_pd(bt), b1 = _mm256_loadu_pd(bt + 4);
        __m256d a = _mm256_broadcast_sd(pa);
        c00 = _mm256_fmadd_pd(a, b0, c00);
        c01 = _mm256_fmadd_pd(a, b1, c01);
        a = _mm256_broadcast_sd(pa + 1);
        c10 = _mm256_fmadd_pd(a, b0, c10);
        c11 = _mm256_fmadd_pd(a, b1, c11);
        a = _mm256_broadcast_sd(pa + 2);
        c20 = _mm256_fmadd_pd(a, b0, c20);
        c21 = _mm256_fmadd_pd(a, b1, c21);
        a = _mm256_broadcast_sd(pa + 3);
        c30 = _mm256_fmadd_pd(a, b0, c30);
        c31 = _mm256_fmadd_pd(a, b1, c31);
        a = _mm256_broadcast_sd(pa + 4);
        c40 = _mm256_fmadd_pd(a, b0, c40);
        c41 = _mm256_fmadd_pd(a, b1, c41);
        a = _mm256_broadcast_sd(pa + 5);
        c50 = _mm256_fmadd_pd(a, b0, c50);
        c51 = _mm256_fmadd_pd(a, b1, c51);
      }
      alignas(32) double t[6][8];
      _mm256_store_pd(t[0], c00); _mm256_store_pd(t[0] + 4, c01);
      _mm256_store_pd(t[1], c10); _mm256_store_pd(t[1] + 4, c11);
      _mm256_store_pd(t[2], c20); _mm256_store_pd(t[2] + 4, c21);
      _mm256_store_pd(t[3], c30); _mm256_store_pd(t[3] + 4, c31);
      _mm256_store_pd(t[4], c40); _mm256_store_pd(t[4] + 4, c41);
      _mm256_store_pd(t[5], c50); _mm256_store_pd(t[5] + 4, c51);
      const int cc = std::min(8, cols - c);
      for (int a = 0; a < rr; ++a) {
        double* cr = C + (int64_t)(r + a) * ldc + c;
        for (int e = 0; e < cc; ++e) cr[e] -= t[a][e];
      }
    }
  }
}

// Blocked right-looking Cholesky of the leading n x n of A (lower, row-major, lda >= n).
// Returns -1 or the first failing pivot.
int64_t potrf_blocked(double* A, int64_t n, int64_t lda) {
  std::vector<double> PT;
  for (int64_t k = 0; k < n; k += NB) {
    const int64_t nb = std::min<int64_t>(NB, n - k);
    const int64_t f = potrf_unblocked(A + k * lda + k, lda, nb);
    if (f >= 0) return k + f;
    const int64_t s = k + nb, m = n - s;
    if (m <= 0) break;
    // panel solve: A[i, k:k+nb] <- A[i, k:k+nb] L_kk^{-T} by forward substitution, 8 rows at
    // a time held transposed (column c of the 8 rows = 2 AVX2 vectors)
    const int64_t nchunk = (m + 7) / 8;
#pragma omp parallel for schedule(static)
    for (int64_t ch = 0; ch < nchunk; ++ch) {
      const int64_t i0 = s + 8 * ch;
      const int rows = (int)std::min<int64_t>(8, n - i0);
      alignas(32) double xt[NB][8];
      for (int r = 0; r < 8; ++r)
        for (int64_t c = 0; c < nb; ++c) xt[c][r] = r < rows ? A[(i0 + r) * lda + k + c] : 0.0;
      for (int64_t c = 0; c < nb; ++c) {
        const __m256d d = _mm256_set1_pd(A[(k + c) * lda + k + c]);
        const __m256d x0 = _mm256_div_pd(_mm256_load_pd(xt[c]), d);
        const __m256d x1 = _mm256_div_pd(_mm256_load_pd(xt[c] + 4), d);
        _mm256_store_pd(xt[c], x0);
        _mm256_store_pd(xt[c] + 4, x1);
        for (int64_t q = c + 1; q < nb; ++q) {
          const __m256d lq = _mm256_set1_pd(A[(k + q) * lda + k + c]);
          _mm256_store_pd(xt[q], _mm256_fnmadd_pd(x0, lq, _mm256_load_pd(xt[q])));
          _mm256_store_pd(xt[q] + 4, _mm256_fnmadd_pd(x1, lq, _mm256_load_pd(xt[q] + 4)));
        }
      }
      for (int r = 0; r < rows; ++r)
        for (int64_t c = 0; c < nb; ++c) A[(i0 + r) * lda + k + c] = xt[c][r];
    }
    // panel transposed: PT[q][j - s] = A[j, k + q] (row j read contiguously)
    PT.resize((size_t)nb * m + 16);  // the micro-kernel loads 16 columns past a short tile
#pragma omp parallel for schedule(static)
    for (int64_t j = s; j < n; ++j)
      for (int64_t q = 0; q < nb; ++q) PT[q * m + (j - s)] = A[j * lda + k + q];
    // trailing update of the lower triangle in TB x TB tiles
    const int64_t T = (m + TB - 1) / TB, ntile = T * (T + 1) / 2;
#pragma omp parallel
    {
      alignas(32) double PA[TB * NB];  // this thread's packed row panel
#pragma omp for schedule(dynamic, 1)
      for (int64_t t = 0; t < ntile; ++t) {
        int64_t ti = (int64_t)((std::sqrt(8.0 * (double)t + 1.0) - 1.0) / 2.0);
        while ((ti + 1) * (ti + 2) / 2 <= t) ++ti;
        while (ti * (ti + 1) / 2 > t) --ti;
        const int64_t tj = t - ti * (ti + 1) / 2;
        const int64_t i0 = s + ti * TB, j0 = s + tj * TB;
        const int rows = (int)std::min<int64_t>(TB, n - i0);
        const int cols = (int)std::min<int64_t>(TB, n - j0);
        for (int r = 0; r < (rows + 5) / 6 * 6; ++r) {
          const double* src = A + (i0 + std::min(r, rows - 1)) * lda + k;
          double* dst = PA + (r / 6) * 6 * nb + r % 6;
          for (int64_t q = 0; q < nb; ++q) dst[6 * q] = src[q];
        }
        tile_update(A + i0 * lda + j0, lda, PA, PT.data() + (j0 - s), m, (int)nb, rows, cols);
      }
    }
  }
  return -1;
}

// ---------------------------------------------------------------- gradient (duals)
// value and derivatives in (D_row, D_col, l)
struct Dd {
  double v, a, b, c;
};
inline Dd dc(double v) { return {v, 0, 0, 0}; }
inline Dd operator+(Dd x, Dd y) { return {x.v + y.v, x.a + y.a, x.b + y.b, x.c + y.c}; }
inline Dd operator-(Dd x, Dd y) { return {x.v - y.v, x.a - y.a, x.b - y.b, x.c - y.c}; }
inline Dd operator-(Dd x) { return {-x.v, -x.a, -x.b, -x.c}; }
inline Dd operator*(Dd x, Dd y) {
  return {x.v * y.v, x.a * y.v + x.v * y.a, x.b * y.v + x.v * y.b, x.c * y.v + x.v * y.c};
}
inline Dd operator/(Dd x, Dd y) {
  const double q = x.v / y.v;
  return {q, (x.a - q * y.a) / y.v, (x.b - q * y.b) / y.v, (x.c - q * y.c) / y.v};
}
inline Dd dexp(Dd x) {
  const double e = std::exp(x.v);
  return {e, e * x.a, e * x.b, e * x.c};
}
inline Dd derf(Dd x) {
  const double g = 1.1283791670955125739 * std::exp(-x.v * x.v);
  return {std::erf(x.v), g * x.a, g * x.b, g * x.c};
}

// h of model.py:315-365 on duals (Dj, Dk: the genes' decays as variables)
inline Dd h_d(Dd Dj, Dd Dk, Dd l, double t1, double t2) {
  const double t_dist = t2 - t1;
  const Dd gk = (Dk * l) / dc(2.0);
  const Dd multiplier = dexp(gk * gk) / (Dj + Dk);
  const Dd first_multiplier = dexp(-(Dk * dc(t_dist)));
  const Dd first_erf_terms = derf(dc(t_dist) / l - gk) + derf(dc(t1) / l + gk);
  const Dd second_multiplier = dexp(-(Dk * dc(t2) + Dj * dc(t1)));
  const Dd second_erf_terms = derf(dc(t2) / l - gk) + derf(gk);
  return multiplier * (first_multiplier * first_erf_terms - second_multiplier * second_erf_terms);
}

struct PairD {
  double dDr, dDc, dSr, dSc, dl;
};

// the flag-switched kernel (model.py:152-195) of rows a, b: derivatives into o (row / column
// gene accumulators), scaled by wgt
void kernel_grad_cpu(const Hyp& p, const double* a, const double* b, double wgt, PairD& o) {
  const int64_t f1 = flag_int(a[2]), f2 = flag_int(b[2]);
  const Dd L{p.l, 0, 0, 1};
  if (f1 * f2 != 0) {
    const int64_t ja = gene_index(a[1], p.G), jb = gene_index(b[1], p.G);
    const Dd Dr{p.D[ja], 1, 0, 0}, Dc{p.D[jb], 0, 1, 0};
    // kernel_xx: S_ja S_jb l sqrt(pi)/2 (h(jb, ja, tb, ta) + h(ja, jb, ta, tb))
    const Dd u = (L * dc(kSqrtPi * 0.5)) * (h_d(Dc, Dr, L, b[0], a[0]) + h_d(Dr, Dc, L, a[0], b[0]));
    const double w = wgt * (double)(f1 * f2), ss = p.S[ja] * p.S[jb];
    o.dDr += w * ss * u.a;
    o.dDc += w * ss * u.b;
    o.dl += w * ss * u.c;
    o.dSr += w * p.S[jb] * u.v;
    o.dSc += w * p.S[ja] * u.v;
  }
  if ((1 - f1) * (1 - f2) != 0) {  // kernel_ff: exp(-(d^2) / (2 l))
    const double d = a[0] - b[0];
    const double q = d * d / (2.0 * p.l);
    o.dl += wgt * (double)((1 - f1) * (1 - f2)) * std::exp(-q) * q / p.l;
  }
  auto kxf = [&](const double* ra, const double* rb, bool a_is_row, int64_t sw) {
    // kernel_xf(ra, rb): the row whose flag is 0 is the latent one (model.py:237-282)
    const bool a_lat = ra[2] == 0.0;
    const double tg = a_lat ? rb[0] : ra[0], gg = a_lat ? rb[1] : ra[1], tl = a_lat ? ra[0] : rb[0];
    const int64_t j = gene_index(gg, p.G);
    const bool gene_is_row = a_is_row != a_lat;  // the gene row is ra unless ra is latent
    const Dd Dg = gene_is_row ? Dd{p.D[j], 1, 0, 0} : Dd{p.D[j], 0, 1, 0};
    const double t_dist = tg - tl;
    const Dd gj = (Dg * L) / dc(2.0);
    const Dd u = (dc(0.5) * L * dc(kSqrtPi)) * dexp(gj * gj) * dexp(-(Dg * dc(t_dist))) *
                 (derf(dc(t_dist) / L - gj) + derf(dc(tl) / L + gj));
    const double w = wgt * (double)sw, s = p.S[j];
    if (gene_is_row) {
      o.dDr += w * s * u.a;
      o.dSr += w * u.v;
    } else {
      o.dDc += w * s * u.b;
      o.dSc += w * u.v;
    }
    o.dl += w * s * u.c;
  };
  if (f1 * (1 - f2) != 0) kxf(a, b, true, f1 * (1 - f2));
  if ((1 - f1) * f2 != 0) kxf(b, a, false, (1 - f1) * f2);
}

// value and gradient of CustomConjMLL(negative).step (constrained parameters); grad[3G + 2]:
// dD dS dB, dl, d obs_stddev. Work: 3 n^2 + 4 n doubles (allocated here if NULL). NaN if not PD.
double mll_grad_cpu(const double* x, const double* y, int64_t n, int64_t G, const double* D,
                    const double* S, const double* B, double l, double sd, double jitter,
                    int negative, double* grad, std::vector<double>& work) {
  const Hyp p{D, S, G, l};
  work.resize((size_t)3 * n * n + 4 * n);
  double* Sg = work.data();           // Sigma, then L (lower)
  double* Xi = Sg + n * n;            // X = L^{-1} (lower)
  double* Wm = Xi + n * n;            // W = a a^T - Sigma^{-1} (full)
  double* r = Wm + n * n;
  double* a = r + n;
  double* z = a + n;
  const double noise = sd * sd;
  for (int64_t i = 0; i < n; ++i)
    for (int64_t j = 0; j <= i; ++j) {
      double v = kernel(p, x + 3 * i, x + 3 * j);
      if (i == j) v = (v + jitter) + noise;
      Sg[i * n + j] = v;
    }
  const double nan = std::nan("");
  if (potrf_unblocked(Sg, n, n) >= 0) {
    for (int64_t k = 0; k < 3 * G + 2; ++k) grad[k] = nan;
    return nan;
  }
  const int64_t bs = n / G;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t g = std::min<int64_t>(i / bs, G - 1);
    r[i] = y[i] - (B[g] / D[g]) * (double)flag_int(x[3 * i + 2]);
  }
  double logdet = 0.0, quad = 0.0;
  for (int64_t i = 0; i < n; ++i) {
    double v = r[i];
    for (int64_t q = 0; q < i; ++q) v -= Sg[i * n + q] * z[q];
    z[i] = v / Sg[i * n + i];
    logdet += std::log(Sg[i * n + i]);
    quad += z[i] * z[i];
  }
  double mll = -0.5 * ((double)n * std::log(2.0 * M_PI) + 2.0 * logdet + quad);
  // X = L^{-1} column by column; a = X^T z; Sigma^{-1} = X^T X
  for (int64_t j = 0; j < n; ++j)
    for (int64_t i = 0; i < n; ++i) {
      if (i < j) {
        Xi[i * n + j] = 0.0;
        continue;
      }
      double v = i == j ? 1.0 : 0.0;
      for (int64_t q = j; q < i; ++q) v -= Sg[i * n + q] * Xi[q * n + j];
      Xi[i * n + j] = v / Sg[i * n + i];
    }
  for (int64_t i = 0; i < n; ++i) {
    double v = 0.0;
    for (int64_t k = i; k < n; ++k) v += Xi[k * n + i] * z[k];
    a[i] = v;
  }
  for (int64_t i = 0; i < n; ++i)
    for (int64_t j = 0; j <= i; ++j) {
      double s = 0.0;
      for (int64_t k = i; k < n; ++k) s += Xi[k * n + i] * Xi[k * n + j];
      Wm[i * n + j] = Wm[j * n + i] = a[i] * a[j] - s;
    }
  std::vector<double> acc((size_t)2 * G + 1, 0.0);
  double tr = 0.0;
  for (int64_t i = 0; i < n; ++i) {
    tr += Wm[i * n + i];
    const int64_t gi = gene_index(x[3 * i + 1], G);
    for (int64_t j = 0; j <= i; ++j) {
      PairD o{0, 0, 0, 0, 0};
      kernel_grad_cpu(p, x + 3 * i, x + 3 * j, i == j ? 0.5 * Wm[i * n + i] : Wm[i * n + j], o);
      const int64_t gj = gene_index(x[3 * j + 1], G);
      acc[gi] += o.dDr;
      acc[gj] += o.dDc;
      acc[G + gi] += o.dSr;
      acc[G + gj] += o.dSc;
      acc[2 * G] += o.dl;
    }
  }
  const double sign = negative ? -1.0 : 1.0;
  for (int64_t g = 0; g < G; ++g) {
    double af = 0.0;
    for (int64_t i = g * bs; i < (g + 1) * bs; ++i) af += a[i] * (double)flag_int(x[3 * i + 2]);
    grad[g] = sign * (acc[g] - B[g] / (D[g] * D[g]) * af);
    grad[G + g] = sign * acc[G + g];
    grad[2 * G + g] = sign * (af / D[g]);
  }
  grad[3 * G] = sign * acc[2 * G];
  grad[3 * G + 1] = sign * sd * tr;
  return sign * mll;
}

inline double softplus_c(double x) { return x >= 0.0 ? x + std::log1p(std::exp(-x)) : std::log1p(std::exp(x)); }
inline double sigmoid_c(double x) {
  const double e = std::exp(-std::fabs(x));
  return x >= 0.0 ? 1.0 / (1.0 + e) : e / (1.0 + e);
}

}  // namespace

extern "C" {

// Lower triangle (j <= i) of K(x, x) + diag_add I into K (row-major, ldk), OpenMP over rows.
int lfm_cpu_gram(const double* x, int64_t n, int64_t G, const double* D, const double* S,
                 double l, double diag_add, double* K, int64_t ldk, int threads) {
  if (!x || !D || !S || !K || n < 1 || G < 1 || ldk < n) return 1;
  if (threads > 0) omp_set_num_threads(threads);
  const Hyp p{D, S, G, l};
#pragma omp parallel for schedule(dynamic, 16)
  for (int64_t i = 0; i < n; ++i)
    for (int64_t j = 0; j <= i; ++j) {
      double v = kernel(p, x + 3 * i, x + 3 * j);
      if (i == j) v = v + diag_add;
      K[i * ldk + j] = v;
    }
  return 0;
}

// Sampled rows of the lower triangle: out[q * n + j] = K(x[rows[q]], x[j]) + diag_add [j ==
// rows[q]] for j <= rows[q] (fp64 arithmetic, stored as float: bench.py's C4 CPU baseline,
// the reference formula on a bounded sample of the fp32 fill's rows); j > rows[q] untouched.
int lfm_cpu_gram_rows_f32(const double* x, int64_t n, int64_t G, const double* D, const double* S,
                          double l, double diag_add, const int64_t* rows, int64_t nrows,
                          float* out, int threads) {
  if (!x || !D || !S || !rows || !out || n < 1 || G < 1 || nrows < 0) return 1;
  for (int64_t q = 0; q < nrows; ++q)
    if (rows[q] < 0 || rows[q] >= n) return 1;
  if (threads > 0) omp_set_num_threads(threads);
  const Hyp p{D, S, G, l};
#pragma omp parallel for schedule(dynamic, 4)
  for (int64_t q = 0; q < nrows; ++q) {
    const int64_t i = rows[q];
    float* o = out + q * n;
    for (int64_t j = 0; j <= i; ++j) {
      double v = kernel(p, x + 3 * i, x + 3 * j);
      if (i == j) v = v + diag_add;
      o[j] = (float)v;
    }
  }
  return 0;
}

// In-place lower Cholesky of the leading n x n of A; returns -1 or the first failing pivot.
int64_t lfm_cpu_potrf(double* A, int64_t n, int64_t lda, int threads) {
  if (threads > 0) omp_set_num_threads(threads);
  return potrf_blocked(A, n, lda);
}

// CustomConjMLL(negative).step (objectives.py:21-78). info (optional, [8]): mll, logdet,
// quad, gram seconds, Cholesky seconds, solve seconds, failing pivot (-1: none), threads.
// work: caller-provided n x n scratch (NULL: allocated here). Returns the MLL (NaN if not PD).
double lfm_cpu_mll(const double* x, const double* y, int64_t n, int64_t G, const double* D,
                   const double* S, const double* B, double l, double obs_stddev, double jitter,
                   int negative, int threads, double* work, double* info) {
  if (threads > 0) omp_set_num_threads(threads);
  std::vector<double> own;
  double* A = work;
  if (!A) {
    own.resize((size_t)n * n);
    A = own.data();
  }
  const double t0 = now();
  // (K + jitter I) + obs_stddev^2 I on the diagonal (objectives.py:71-73)
  const Hyp p{D, S, G, l};
  const double noise = obs_stddev * obs_stddev;
#pragma omp parallel for schedule(dynamic, 16)
  for (int64_t i = 0; i < n; ++i)
    for (int64_t j = 0; j <= i; ++j) {
      double v = kernel(p, x + 3 * i, x + 3 * j);
      if (i == j) v = (v + jitter) + noise;
      A[i * n + j] = v;
    }
  const double t1 = now();
  const int64_t fail = potrf_blocked(A, n, n);
  const double t2 = now();
  double mll = std::nan(""), logdet = std::nan(""), quad = std::nan("");
  if (fail < 0) {
    // r = y - m, m_i = (B/D)[i / (n / G)] * int(flag_i) (model.py:143-149); z = L^{-1} r
    const int64_t bs = n / G;
    std::vector<double> z((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
      const int64_t g = std::min<int64_t>(i / bs, G - 1);
      z[i] = y[i] - (B[g] / D[g]) * (double)flag_int(x[3 * i + 2]);
    }
    for (int64_t i = 0; i < n; ++i) {
      double v = z[i];
      const double* li = A + i * n;
      for (int64_t q = 0; q < i; ++q) v -= li[q] * z[q];
      z[i] = v / li[i];
    }
    logdet = 0.0;
    quad = 0.0;
    for (int64_t i = 0; i < n; ++i) {
      logdet += std::log(A[i * n + i]);
      quad += z[i] * z[i];
    }
    logdet *= 2.0;
    mll = -0.5 * ((double)n * std::log(2.0 * M_PI) + logdet + quad);
    if (negative) mll = -mll;
  }
  const double t3 = now();
  if (info) {
    info[0] = mll;
    info[1] = logdet;
    info[2] = quad;
    info[3] = t1 - t0;
    info[4] = t2 - t1;
    info[5] = t3 - t2;
    info[6] = (double)fail;
    info[7] = (double)omp_get_max_threads();
  }
  return mll;
}


// Value and gradient of CustomConjMLL(negative).step at the constrained parameters (trainer.py:126
// before the chain rule); grad[3G + 2] = dD dS dB, dl, d obs_stddev. Returns the value (NaN and a
// NaN gradient when Sigma is not PD).
double lfm_cpu_mll_grad(const double* x, const double* y, int64_t n, int64_t G, const double* D,
                        const double* S, const double* B, double l, double obs_stddev,
                        double jitter, int negative, double* grad) {
  std::vector<double> work;
  return mll_grad_cpu(x, y, n, G, D, S, B, l, obs_stddev, jitter, negative, grad, work);
}

// JaxTrainer.fit of ONE problem (trainer.py:162-228; dis_project_amd/trainer.py's loop):
// raw[3G + 3] in/out, the unconstrained parameters (d s b, l, obs_stddev) and the static jitter;
// iters Adam steps (step0 = 0, fresh moments) with after_epoch every spe steps when fix; the loss
// history[iters]. Returns the number of steps whose factorisation failed.
int lfm_cpu_fit(const double* x, const double* y, int64_t n, int64_t G, double* raw, int64_t iters,
                double lr, double b1, double b2, double eps, double eps_root, int64_t spe, int fix,
                int negative, double* history) {
  const int64_t np = 3 * G + 2;
  std::vector<double> mu((size_t)np, 0.0), nu((size_t)np, 0.0), hyp((size_t)np), g((size_t)np), work;
  int failed = 0;
  for (int64_t s = 0; s < iters; ++s) {
    for (int64_t i = 0; i < np; ++i)
      hyp[i] = i == 3 * G ? 0.5 + 3.0 * sigmoid_c(raw[i]) : softplus_c(raw[i]);
    const double v = mll_grad_cpu(x, y, n, G, hyp.data(), hyp.data() + G, hyp.data() + 2 * G,
                                  hyp[3 * G], hyp[3 * G + 1], raw[3 * G + 2], negative, g.data(),
                                  work);
    if (std::isnan(v)) ++failed;
    history[s] = v;
    const double count = (double)(s + 1);
    const double c1 = 1.0 - std::pow(b1, count), c2 = 1.0 - std::pow(b2, count);
    for (int64_t i = 0; i < np; ++i) {
      const double sg = sigmoid_c(raw[i]);
      const double gr = i == 3 * G ? g[i] * 3.0 * sg * (1.0 - sg) : g[i] * sg;
      mu[i] = b1 * mu[i] + (1.0 - b1) * gr;
      nu[i] = b2 * nu[i] + (1.0 - b2) * (gr * gr);
      raw[i] = raw[i] + -lr * ((mu[i] / c1) / (std::sqrt(nu[i] / c2 + eps_root) + eps));  // optax's order
    }
    if (fix && s % spe == 0 && G > 3) {
      raw[G + 3] = 1.0;
      raw[3] = 0.8;
    }
  }
  return failed;
}

// The CPU baselines across cores (bench.py's c5 / c5fit cpu_baseline "threads" variants): nprob
// independent problems, one per OpenMP thread at a time (dynamic, 1), each evaluated or fitted
// serially (nested regions inactive). x / y / n / G per problem; hyp in lfm_batch_mll_f64's
// packed layout (each problem's D S B, then each problem's l, obs_stddev, jitter).
// reps > 1: the nprob problems evaluated reps times over (a timing sample), out from any rep.
// Inside a team of several threads the problem's own parallel regions are nested, so inactive
// (serial); a team of one passes threads = 1 so that they do not spread over the cores.
int lfm_cpu_mll_batch(int64_t nprob, const double* const* x, const double* const* y,
                      const int64_t* n, const int64_t* G, const double* hyp, int negative,
                      int threads, int64_t reps, double* out) {
  if (nprob < 1 || reps < 1) return 1;
  std::vector<int64_t> off((size_t)nprob), nvec(1, 0);
  for (int64_t q = 0; q < nprob; ++q) {
    off[q] = nvec[0];
    nvec[0] += 3 * G[q];
  }
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads > 0 ? threads : omp_get_max_threads())
  for (int64_t t = 0; t < nprob * reps; ++t) {
    const int64_t q = t % nprob;
    const double* v = hyp + off[q];
    const double* sc = hyp + nvec[0] + 3 * q;
    out[q] = lfm_cpu_mll(x[q], y[q], n[q], G[q], v, v + G[q], v + 2 * G[q], sc[0], sc[1], sc[2],
                         negative, omp_get_num_threads() > 1 ? 0 : 1, nullptr, nullptr);
  }
  return 0;
}

// raw[q]: problem q's [3G + 3] unconstrained parameters (in / out); history [nprob][iters].
// Returns the number of failed steps over all problems.
int lfm_cpu_fit_batch(int64_t nprob, const double* const* x, const double* const* y,
                      const int64_t* n, const int64_t* G, double* const* raw, int64_t iters,
                      double lr, double b1, double b2, double eps, double eps_root, int64_t spe,
                      int fix, int negative, int threads, double* history) {
  int failed = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : failed) num_threads(threads > 0 ? threads : omp_get_max_threads())
  for (int64_t q = 0; q < nprob; ++q)
    failed += lfm_cpu_fit(x[q], y[q], n[q], G[q], raw[q], iters, lr, b1, b2, eps, eps_root, spe,
                          fix, negative, history + q * iters);
  return failed;
}

}  // extern "C"
