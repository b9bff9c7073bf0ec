// lfm_math.h — per-pair SIM kernel math (device), shared by the gram and small-N kernels.
// Each function restates the reference expression it cites, in the same operation order,
// with floating-point contraction off (no fused multiply-add): the reference's XLA-CPU
// elementwise code rounds every product, and exact identities of the formula — e.g. the
// t = 0 rows of h vanishing because erf is odd (SURVEY.md §4 KAT) — depend on it.
#pragma once
#include "lfm_internal.h"


namespace lfm {

static constexpr double kSqrtPi = 1.7724538509055160273;

// ------------------------------------------------------------- per-pair math
// h(j,k,t1,t2), model.py:315-365.
__device__ __forceinline__ double h_ref(const HypDev& p, int j, int k, double t1, double t2) {
  #pragma clang fp contract(off)
  const double l = p.l;
  const double gk = p.D[k] * l / 2.0;                           // gamma(k), model.py:367-369
  const double tdist = t2 - t1;
  const double multiplier = exp(gk * gk) / (p.D[j] + p.D[k]);
  const double first_multiplier = exp(-p.D[k] * tdist);
  const double first_erf = erf((tdist / l) - gk) + erf(t1 / l + gk);
  const double second_multiplier = exp(-(p.D[k] * t2 + p.D[j] * t1));
  const double second_erf = erf((t2 / l) - gk) + erf(gk);
  return multiplier * (first_multiplier * first_erf - second_multiplier * second_erf);
}

// kernel_xx, model.py:197-235.
__device__ __forceinline__ double kxx_ref(const HypDev& p, double ta, int j, double tb, int k) {
  #pragma clang fp contract(off)
  const double mult = p.S[j] * p.S[k] * p.l * kSqrtPi * 0.5;
  return mult * (h_ref(p, k, j, tb, ta) + h_ref(p, j, k, ta, tb));
}

// kernel_xf, model.py:237-282 (the row whose flag is non-zero is the gene row).
__device__ __forceinline__ double kxf_ref(const HypDev& p, double ta, double ga, double fa,
                                          double tb, double gb) {
  #pragma clang fp contract(off)
  const bool a_is_latent = (fa == 0.0);
  const double tg = a_is_latent ? tb : ta;
  const double gg = a_is_latent ? gb : ga;
  const double tl = a_is_latent ? ta : tb;
  const int j = gene_index(gg, p.G);
  const double l = p.l;
  const double gj = p.D[j] * l / 2.0;
  const double t_dist = tg - tl;
  const double first_term = 0.5 * l * kSqrtPi * p.S[j];
  const double e1 = exp(gj * gj);
  const double e2 = exp(-p.D[j] * t_dist);
  const double erfs = erf((t_dist / l) - gj) + erf(tl / l + gj);
  return first_term * e1 * e2 * erfs;
}

// kernel_ff, model.py:284-312 (divides by 2*l, not l^2: kept for parity).
__device__ __forceinline__ double kff_ref(const HypDev& p, double ta, double tb) {
  #pragma clang fp contract(off)
  const double d = ta - tb;
  return exp(-((d * d) / (2.0 * p.l)));
}

// Flag-switched kernel, model.py:152-195. Branches whose integer switch is zero
// are not evaluated (the reference evaluates them and multiplies by 0).
__device__ __forceinline__ double kernel_ref(const HypDev& p, double ta, double ga, double fa,
                                             double tb, double gb, double fb) {
  #pragma clang fp contract(off)
  const long long f1 = flag_int(fa), f2 = flag_int(fb);
  const long long s_xx = f1 * f2, s_ff = (1 - f1) * (1 - f2);
  const long long s_xf = f1 * (1 - f2), s_fx = (1 - f1) * f2;
  double v = 0.0;
  if (s_xx) v += (double)s_xx * kxx_ref(p, ta, gene_index(ga, p.G), tb, gene_index(gb, p.G));
  if (s_ff) v += (double)s_ff * kff_ref(p, ta, tb);
  if (s_xf) v += (double)s_xf * kxf_ref(p, ta, ga, fa, tb, gb);
  if (s_fx) v += (double)s_fx * kxf_ref(p, tb, gb, fb, ta, ga);
  return v;
}

// kernel_xx from per-problem tables (small_mll_kernel): the same operations on the same
// operands as kxx_ref / h_ref, so the same bits, with every factor that depends on one row or
// one gene only evaluated once per row / gene instead of once per pair:
//   gam[g] = D_g l / 2, egg[g] = exp(gam^2), erg[g] = erf(gam)            (per gene)
//   e2[i] = erf(t_i / l - gam[g_i]), e1[i G + g] = erf(t_i / l + gam[g])    (per row)
// and exp(-(D_k t2 + D_j t1)), which both h terms of a pair share (the sum is the same two
// products in the other order, and IEEE addition commutes). Left per pair: one erf and one exp
// per h, the shared exp and the two divisions. a, b: row indices; j = g_a, k = g_b.
struct KxxTab {
  const double* gam;
  const double* egg;
  const double* erg;
  const double* e1;
  const double* e2;
  int G;
};
__device__ __forceinline__ double h_tab(const HypDev& p, const KxxTab& t, int j, int k,
                                        double t1, double t2, int r1, int r2, double se) {
  #pragma clang fp contract(off)
  const double l = p.l;
  const double tdist = t2 - t1;
  const double multiplier = t.egg[k] / (p.D[j] + p.D[k]);
  const double first_multiplier = exp(-p.D[k] * tdist);
  const double first_erf = erf((tdist / l) - t.gam[k]) + t.e1[r1 * t.G + k];
  const double second_erf = t.e2[r2] + t.erg[k];
  return multiplier * (first_multiplier * first_erf - se * second_erf);
}
__device__ __forceinline__ double kxx_tab(const HypDev& p, const KxxTab& t, double ta, int j,
                                          int a, double tb, int k, int b) {
  #pragma clang fp contract(off)
  const double mult = p.S[j] * p.S[k] * p.l * kSqrtPi * 0.5;
  const double se = exp(-(p.D[k] * tb + p.D[j] * ta));
  return mult * (h_tab(p, t, k, j, tb, ta, b, a, se) + h_tab(p, t, j, k, ta, tb, a, b, se));
}

// KxxTab's per-gene and per-row factors of one problem, into the shared memory t points to
// (one 256-thread workgroup; two workgroup barriers).
__device__ __forceinline__ void small_tables(const HypDev& h, const double* __restrict__ x, int n,
                                             const KxxTab& t, double* gam, double* egg,
                                             double* erg, double* e1, double* e2) {
  #pragma clang fp contract(off)
  const int tid = threadIdx.x, G = h.G;
  const double l = h.l;
  for (int g = tid; g < G; g += 256) {
    const double gk = h.D[g] * l / 2.0;  // gamma(k), model.py:367-369
    gam[g] = gk;
    egg[g] = exp(gk * gk);
    erg[g] = erf(gk);
  }
  __syncthreads();
  for (int i = tid; i < n; i += 256) e2[i] = erf((x[3 * i] / l) - gam[gene_index(x[3 * i + 1], G)]);
  for (int q = tid; q < n * G; q += 256) {
    const int i = q / G, g = q - i * G;
    e1[q] = erf(x[3 * i] / l + gam[g]);
  }
  __syncthreads();
}

// e^{A} erfc(z) without overflow: erfcx(z) e^{A - z^2} once erfc(z) underflows towards 0.
__device__ __forceinline__ double exp_erfc(double A, double z) {
  return z > 0.0 ? erfcx(z) * exp(A - z * z) : exp(A) * erfc(z);
}

// Entry idx of the grid-layout tables (layout and identities: lfm_gram.hip, tables_kernel),
// shared by tables_kernel and small_mll_kernel's grid path.
__device__ __forceinline__ double grid_table_entry(const HypDev& p, int T, double dt,
                                                   const double* __restrict__ times,
                                                   int64_t idx) {
  const int G = p.G;
  const int64_t W = 2 * (int64_t)T - 1;
  const int64_t nW = (int64_t)G * W, nT = (int64_t)G * T;
  const double l = p.l;
  if (idx < 2 * nW) {
    const int64_t q = idx < nW ? idx : idx - nW;
    const int g = (int)(q / W);
    const int d = (int)(q - (int64_t)g * W) - (T - 1);
    const double gam = p.D[g] * l / 2.0;
    const double delta = (double)d * dt;
    const double A = gam * gam - p.D[g] * delta;
    return idx < nW ? exp_erfc(A, gam - delta / l) : exp(A);
  }
  if (idx < 2 * nW + 3 * nT) {
    const int64_t q0 = idx - 2 * nW;
    const int which = (int)(q0 / nT);
    const int64_t q = q0 - which * nT;
    const int g = (int)(q / T);
    const double t = times[q - (int64_t)g * T];
    const double gam = p.D[g] * l / 2.0;
    if (which == 0) return erfc(t / l + gam);
    if (which == 1) return exp(-p.D[g] * t);
    return exp_erfc(gam * gam, gam - t / l) - erfcx(gam);
  }
  const int64_t q = idx - 2 * nW - 3 * nT;
  const int j = (int)(q / G), k = (int)(q - (int64_t)j * G);
  return p.S[j] * p.S[k] * l * kSqrtPi * 0.5 / (p.D[j] + p.D[k]);
}

// mean_function, model.py:143-149: m[i] = (B/D)[i / (n/G)] * int(x[i,2]).
__device__ __forceinline__ double mean_at(const HypDev& p, const double* x, int64_t i,
                                          int64_t bs) {
  #pragma clang fp contract(off)
  const int g = (int)(i / bs);
  return (p.B[g] / p.D[g]) * (double)flag_int(x[i * 3 + 2]);
}

// 1/sqrt(x): v_rsq_f64 estimate + one Newton step (a pivot and its inverse come from one
// estimate instead of a correctly rounded sqrt followed by a divide). The pivot's relative
// error stays far below the 1e-9 MLL tolerance (a perturbation of the pivot by a factor
// (1 + e) is a backward error e in that column); tests/test_gpu_parity.py bounds it.
__device__ __forceinline__ double rsqrt_1nr(double x) {
  const double h = -0.5 * x;
  const double y = __builtin_amdgcn_rsq(x);
  return y * fma(h * y, y, 1.5);
}

// Value of v held by `lane` (wave-uniform lane index), broadcast to the wave.
__device__ __forceinline__ double rdl(double v, int lane) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b & 0xffffffffu), lane);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), lane);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

}  // namespace lfm
