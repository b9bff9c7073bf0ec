// lfm_dual.h — device math of the MLL gradient, shared by the large-N
// reduction kernels (lfm_grad.hip) and the small-N batched gradient / fit (lfm_small.hip):
// forward-mode duals of the SIM kernel in (D_row, D_col, l) on the cancellation-free erfc form
// of h (model.py:315-365), and the per-gene grid tables of its derivatives.
#pragma once
#include "lfm_math.h"

namespace lfm {

// e^{A} erfc(z) without overflow: erfcx(z) e^{A - z^2} once erfc(z) underflows towards 0.
__device__ __forceinline__ double exp_erfc_g(double A, double z) {
  return z > 0.0 ? erfcx(z) * exp(A - z * z) : exp(A) * erfc(z);
}

// ---------------------------------------------------------------- duals
// Value and derivatives with respect to (D_row_gene, D_col_gene, l).
struct Dual3 {
  double v, a, b, c;
};
__device__ __forceinline__ Dual3 dconst(double v) { return {v, 0.0, 0.0, 0.0}; }
__device__ __forceinline__ Dual3 operator+(Dual3 x, Dual3 y) {
  return {x.v + y.v, x.a + y.a, x.b + y.b, x.c + y.c};
}
__device__ __forceinline__ Dual3 operator-(Dual3 x, Dual3 y) {
  return {x.v - y.v, x.a - y.a, x.b - y.b, x.c - y.c};
}
__device__ __forceinline__ Dual3 operator*(Dual3 x, Dual3 y) {
  return {x.v * y.v, x.a * y.v + x.v * y.a, x.b * y.v + x.v * y.b, x.c * y.v + x.v * y.c};
}
__device__ __forceinline__ Dual3 operator*(double s, Dual3 x) {
  return {s * x.v, s * x.a, s * x.b, s * x.c};
}
__device__ __forceinline__ Dual3 operator/(Dual3 x, Dual3 y) {
  const double iv = 1.0 / y.v, q = x.v * iv;
  return {q, (x.a - q * y.a) * iv, (x.b - q * y.b) * iv, (x.c - q * y.c) * iv};
}
__device__ __forceinline__ Dual3 dexp(Dual3 x) {
  const double e = exp(x.v);
  return {e, e * x.a, e * x.b, e * x.c};
}
// e^{A} erfc(z) and its derivative e^{A} erfc(z) dA - (2/sqrt(pi)) e^{A - z^2} dz.
__device__ __forceinline__ Dual3 dexp_erfc(Dual3 A, Dual3 z) {
  const double ez = exp(A.v - z.v * z.v);
  const double f = z.v > 0.0 ? erfcx(z.v) * ez : exp(A.v) * erfc(z.v);
  const double g = 1.1283791670955125739 * ez;  // 2 / sqrt(pi)
  return {f, f * A.a - g * z.a, f * A.b - g * z.b, f * A.c - g * z.c};
}

// (D_j + D_k) h(j, k, t1, t2) of model.py:343-363 in the erfc form:
//   e^{g^2 - Dk d} (erfc(g - d/l) - erfc(t1/l + g))
//   - e^{-(Dk t2 + Dj t1)} e^{g^2} (erfc(g - t2/l) - erfc(g)),   g = Dk l / 2, d = t2 - t1.
__device__ __forceinline__ Dual3 h_bracket(Dual3 Dj, Dual3 Dk, Dual3 l, double t1, double t2) {
  const Dual3 g = 0.5 * (Dk * l);
  const Dual3 g2 = g * g;
  const double d = t2 - t1;
  const Dual3 il = dconst(1.0) / l;
  const Dual3 A1 = g2 - d * Dk;
  const Dual3 first = dexp_erfc(A1, g - d * il) - dexp_erfc(A1, t1 * il + g);
  const Dual3 E = dexp(dconst(0.0) - (t2 * Dk + t1 * Dj));
  const Dual3 Q = dexp_erfc(g2, g - t2 * il) - dexp_erfc(g2, g);
  return first - E * Q;
}

// Derivative contributions of one pair: K and dK/d{D_row, D_col, l}, dK/dS_row, dK/dS_col.
struct PairGrad {
  double dDr, dDc, dl, dSr, dSc;
};

// kernel_xx (model.py:197-235): K = S_j S_k l sqrt(pi)/2 (h(k,j,tb,ta) + h(j,k,ta,tb)).
__device__ __forceinline__ void kxx_grad(const HypDev& p, double ta, int j, double tb, int k,
                                         double wgt, PairGrad& o) {
  const Dual3 Dj{p.D[j], 1.0, 0.0, 0.0}, Dk{p.D[k], 0.0, 1.0, 0.0}, L{p.l, 0.0, 0.0, 1.0};
  const Dual3 hs = h_bracket(Dj, Dk, L, ta, tb) + h_bracket(Dk, Dj, L, tb, ta);
  const Dual3 u = (0.5 * kSqrtPi) * (L * hs / (Dj + Dk));
  const double ss = p.S[j] * p.S[k];
  o.dDr += wgt * ss * u.a;
  o.dDc += wgt * ss * u.b;
  o.dl += wgt * ss * u.c;
  o.dSr += wgt * p.S[k] * u.v;
  o.dSc += wgt * p.S[j] * u.v;
}

// kernel_xf (model.py:237-282) with the gene row's time tg, gene gg and the latent time tl:
//   K = l sqrt(pi)/2 S_g e^{g^2 - D delta} (erfc(g - delta/l) - erfc(tl/l + g)).
// gene_is_row selects which accumulator (row or column gene) receives dD and dS.
__device__ __forceinline__ void kxf_grad(const HypDev& p, double tg, int g, double tl,
                                         bool gene_is_row, double wgt, PairGrad& o) {
  const Dual3 Dg{p.D[g], 1.0, 0.0, 0.0}, L{p.l, 0.0, 0.0, 1.0};
  const Dual3 gm = 0.5 * (Dg * L);
  const double d = tg - tl;
  const Dual3 il = dconst(1.0) / L;
  const Dual3 A = gm * gm - d * Dg;
  const Dual3 br = dexp_erfc(A, gm - d * il) - dexp_erfc(A, tl * il + gm);
  const Dual3 u = (0.5 * kSqrtPi) * (L * br);
  const double s = p.S[g];
  if (gene_is_row) {
    o.dDr += wgt * s * u.a;
    o.dSr += wgt * u.v;
  } else {
    o.dDc += wgt * s * u.a;
    o.dSc += wgt * u.v;
  }
  o.dl += wgt * s * u.c;
}

// Flag-switched kernel derivatives (model.py:152-195), same branch selection as kernel_ref.
__device__ __forceinline__ void kernel_grad(const HypDev& p, double ta, double ga, double fa,
                                            double tb, double gb, double fb, double wgt,
                                            PairGrad& o) {
  const long long f1 = flag_int(fa), f2 = flag_int(fb);
  const long long s_xx = f1 * f2, s_ff = (1 - f1) * (1 - f2);
  const long long s_xf = f1 * (1 - f2), s_fx = (1 - f1) * f2;
  const int j = gene_index(ga, p.G), k = gene_index(gb, p.G);
  if (s_xx) kxx_grad(p, ta, j, tb, k, wgt * (double)s_xx, o);
  if (s_ff) {
    const double d = ta - tb;
    const double q = (d * d) / (2.0 * p.l);
    o.dl += wgt * (double)s_ff * exp(-q) * q / p.l;
  }
  // kxf_ref(p, ta, ga, fa, tb, gb): the row whose flag is 0.0 is the latent one
  if (s_xf) {
    const bool a_lat = (fa == 0.0);
    kxf_grad(p, a_lat ? tb : ta, a_lat ? k : j, a_lat ? ta : tb, !a_lat, wgt * (double)s_xf, o);
  }
  if (s_fx) {
    const bool b_lat = (fb == 0.0);
    kxf_grad(p, b_lat ? ta : tb, b_lat ? j : k, b_lat ? tb : ta, b_lat, wgt * (double)s_fx, o);
  }
}

__device__ __forceinline__ double wave_sum(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// The same sum without LDS round trips (the small kernels' reductions are latency-bound): an
// inclusive scan by DPP row shifts (1, 2, 4, 8) within each 16-lane row, row_bcast15 /
// row_bcast31 across the rows, then lane 63's total read back to every lane. 32-bit DPP moves on
// the two halves; lanes without a source read 0. Another summation order than wave_sum's.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ double dpp_step(double x) {
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, ROW_MASK, 0xf, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROW_MASK, 0xf, true);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double wave_sum_dpp(double v) {
  v += dpp_step<0x111, 0xf>(v);  // row_shr:1
  v += dpp_step<0x112, 0xf>(v);  // row_shr:2
  v += dpp_step<0x114, 0xf>(v);  // row_shr:4
  v += dpp_step<0x118, 0xf>(v);  // row_shr:8
  v += dpp_step<0x142, 0xa>(v);  // row_bcast:15 into rows 1 and 3
  v += dpp_step<0x143, 0xc>(v);  // row_bcast:31 into rows 2 and 3
  return rdl(v, 63);
}

// ------------------------------------------------------- grid (table) path
// On the dataset_3d grid every transcendental of kernel_xx and of its derivatives in
// (D_j, D_k, l) separates per (gene, tau) or per (gene, d = tau' - tau), as in the gram's
// tables (lfm_gram.hip): with g = D l / 2, delta = d dt, A = g^2 - D delta, z = g - delta/l,
// y = t/l + g, u = g - t/l (and A - z^2 = -delta^2/l^2, g^2 - u^2 = D t - t^2/l^2):
//   Wt = e^A erfc(z)  dW/dD = Wt (g l - delta) - c e^{-delta^2/l^2} l/2
//                     dW/dl = Wt g D - c e^{-delta^2/l^2} (D/2 + delta/l^2)
//   Xt = e^A          dX/dD = Xt (g l - delta),  dX/dl = Xt g D
//   Pt = erfc(y)      dP/dD = -c e^{-y^2} l/2,   dP/dl = -c e^{-y^2} (D/2 - t/l^2)
//   Et = e^{-D t}     dE/dD = -t Et
//   Qt = e^{g^2}(erfc(u) - erfc(g))
//                     dQ/dD = g l Qt - c (l/2) (e^{D t - t^2/l^2} - 1)
//                     dQ/dl = g D Qt - c ((D/2 + t/l^2) e^{D t - t^2/l^2} - D/2)
// with c = 2/sqrt(pi). Layout (doubles), W = 2T - 1: the six Toeplitz rows
// Wt Xt WtD XtD Wtl Xtl (G x W each), then the eight time rows Pt PtD Ptl Et EtD Qt QtD Qtl
// (G x T each).
__host__ __device__ inline size_t grad_tables_doubles(int G, int T) {
  return 6 * (size_t)G * (2 * (size_t)T - 1) + 8 * (size_t)G * T;
}

__device__ __forceinline__ double grad_table_entry(const HypDev& p, int T, double dt,
                                                 const double* __restrict__ times, int64_t idx) {
  const int G = p.G;
  const int64_t W = 2 * (int64_t)T - 1, nW = (int64_t)G * W, nT = (int64_t)G * T;
  const double l = p.l, c2 = 1.1283791670955125739;  // 2 / sqrt(pi)
  double v;
  if (idx < 6 * nW) {
    const int which = (int)(idx / nW);
    const int64_t q = idx - which * nW;
    const int g = (int)(q / W);
    const int d = (int)(q - (int64_t)g * W) - (T - 1);
    const double D = p.D[g], gam = D * l / 2.0, delta = (double)d * dt;
    const double A = gam * gam - D * delta;
    const double X = exp(A);
    const double Wv = exp_erfc_g(A, gam - delta / l);
    const double ez = c2 * exp(-(delta / l) * (delta / l));
    switch (which) {
      case 0: v = Wv; break;
      case 1: v = X; break;
      case 2: v = Wv * (gam * l - delta) - ez * (l / 2.0); break;
      case 3: v = X * (gam * l - delta); break;
      case 4: v = Wv * gam * D - ez * (D / 2.0 + delta / (l * l)); break;
      default: v = X * gam * D; break;
    }
  } else {
    const int64_t q0 = idx - 6 * nW;
    const int which = (int)(q0 / nT);
    const int64_t q = q0 - which * nT;
    const int g = (int)(q / T);
    const double t = times[q - (int64_t)g * T];
    const double D = p.D[g], gam = D * l / 2.0;
    if (which < 3) {
      const double y = t / l + gam, ey = c2 * exp(-y * y);
      v = which == 0 ? erfc(y) : which == 1 ? -ey * (l / 2.0) : -ey * (D / 2.0 - t / (l * l));
    } else if (which < 5) {
      const double E = exp(-D * t);
      v = which == 3 ? E : -t * E;
    } else {
      const double Q = exp_erfc_g(gam * gam, gam - t / l) - erfcx(gam);
      const double eq = exp(D * t - t * t / (l * l));
      v = which == 5 ? Q
          : which == 6 ? gam * l * Q - c2 * (l / 2.0) * (eq - 1.0)
                       : gam * D * Q - c2 * ((D / 2.0 + t / (l * l)) * eq - D / 2.0);
    }
  }
  return v;
}

}  // namespace lfm
