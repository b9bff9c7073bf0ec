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
//   potrf_diag_kernel  one workgroup factors the 128x128 diagonal block in LDS, 16 columns
//                      at a time: the 16x16 diagonal sub-block is factored and inverted
//                      in registers by every wave (cross-lane v_readlane broadcasts), the
//                      rows below are solved against that inverse, and the rank-16 update
//                      of the rest runs on v_mfma_f64_16x16x4_f64. It also writes the eight
//                      16x16 diagonal inverses (dinv) for the panel solve, the logdet
//                      partial and the first failing pivot. Columns >= n take a unit pivot.
//   trsm_kernel        rows below the block: X = A_ik L_kk^{-T} by blocked substitution,
//                      16 columns at a time, on fp64 MFMA (L_kk from L2, dinv blocks).
//   syrk_kernel        trailing lower triangle, 128x128 tiles: C -= P P^T on fp64 MFMA —
//                      the only O(n^3) kernel.
// Look-ahead: the SYRK of block column k is split into the next block column (k+1) and
// the rest. A high-priority side stream runs syrk(next) -> potrf(k+1) -> trsm(k+1) while
// the main stream runs syrk(rest) of step k, so the latency-bound panel work of step k+1
// hides behind the bulk of step k's trailing update.
// finalize_kernel reduces logdet + ||z||^2 to the scalar MLL.
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <utility>

#include "lfm_math.h"

namespace lfm {

typedef double double4v __attribute__((ext_vector_type(4)));

static constexpr int NB = 128;       // panel width (block column)
static constexpr int IB = 16;        // inner block of the diagonal factor / panel solve
static constexpr int ST = 128;       // SYRK output tile edge
static constexpr int KB = 16;        // SYRK K-step staged through LDS
#ifndef LFM_LDS_PAD
#define LFM_LDS_PAD 2
#endif
// LDS row stride of a staged K stage: KS + LDP doubles. ds_read_b64 banks by (a / 4) mod 64
// per 32-lane half: the MFMA fragment reads (16 rows x 4 k, and 4 rows x 4 k) are conflict-free
// at a stride of 18 (and 66 for the chain's 64-deep stages); at 17 the 16-row reads were 2-way
// conflicted. Measured: -0.57 ms per C2 evaluation (scripts/ab_lib.py, 5 rounds), same bits.
static constexpr int LDP = LFM_LDS_PAD;
static constexpr int STATUS_NONE = INT_MAX;
constexpr int PANEL_TIMEOUT = STATUS_TIMEOUT;  // status: a bounded device-side wait ran out
// Which wait ran out first (status[1], reported in LFM_E_TIMEOUT's message): 1 tall unit on the
// chain, 2 tall unit on its ahead units, 5 chain input wait, 6 chain grid barrier, 7 fused panel
// wait (3 and 4 are unused).
__device__ __forceinline__ void timeout_at(int* status, int why) {
  atomicMin(status, PANEL_TIMEOUT);
  atomicCAS(status + 1, 0, why);
}

__device__ __forceinline__ double4v mfma16(double a, double b, double4v c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// v_mfma_f64_4x4x4_4b_f64: four independent 4x4x4 blocks, g = (lane >> 2) & 3; lane maps
// (scripts/probe_mfma4_layout.py): A_g[i][k] at lane 16k + 4g + i, B_g[k][j] at lane
// 16k + 4g + j, D_g[i][j] at lane 16i + 4g + j.
__device__ __forceinline__ double mfma4(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}

// Value of v held by lane `src` (0..15, compile-time) of each 16-lane row, broadcast to the
// row: DPP row_newbcast (VGPR to VGPR; no SGPR round trip as with v_readlane).
template <int SRC>
__device__ __forceinline__ double row_bcast_t(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, 0x150 + SRC, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), 0x150 + SRC, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// src folds to a constant in the fully unrolled callers
__device__ __forceinline__ double row_bcast(double v, int src) {
  switch (src) {
    case 0: return row_bcast_t<0>(v);
    case 1: return row_bcast_t<1>(v);
    case 2: return row_bcast_t<2>(v);
    case 3: return row_bcast_t<3>(v);
    case 4: return row_bcast_t<4>(v);
    case 5: return row_bcast_t<5>(v);
    case 6: return row_bcast_t<6>(v);
    case 7: return row_bcast_t<7>(v);
    case 8: return row_bcast_t<8>(v);
    case 9: return row_bcast_t<9>(v);
    case 10: return row_bcast_t<10>(v);
    case 11: return row_bcast_t<11>(v);
    case 12: return row_bcast_t<12>(v);
    case 13: return row_bcast_t<13>(v);
    case 14: return row_bcast_t<14>(v);
    default: return row_bcast_t<15>(v);
  }
}

// As row_bcast with one v_mov_b64_dpp (gfx90a+ 64-bit DPP, row_newbcast) instead of two
// 32-bit moves; the compiler keeps the DPP hazards.
template <int SRC>
__device__ __forceinline__ double row_bcast64_t(double v) {
  return __builtin_amdgcn_mov_dpp(v, 0x150 + SRC, 0xf, 0xf, false);
}
__device__ __forceinline__ double row_bcast64(double v, int src) {
  switch (src) {
    case 0: return row_bcast64_t<0>(v);
    case 1: return row_bcast64_t<1>(v);
    case 2: return row_bcast64_t<2>(v);
    case 3: return row_bcast64_t<3>(v);
    case 4: return row_bcast64_t<4>(v);
    case 5: return row_bcast64_t<5>(v);
    case 6: return row_bcast64_t<6>(v);
    case 7: return row_bcast64_t<7>(v);
    case 8: return row_bcast64_t<8>(v);
    case 9: return row_bcast64_t<9>(v);
    case 10: return row_bcast64_t<10>(v);
    case 11: return row_bcast64_t<11>(v);
    case 12: return row_bcast64_t<12>(v);
    case 13: return row_bcast64_t<13>(v);
    case 14: return row_bcast64_t<14>(v);
    default: return row_bcast64_t<15>(v);
  }
}

// Orders one wave's LDS writes before its following LDS reads (and vice versa): LDS
// operations of a wave complete in order; the asm keeps the compiler from reordering.
__device__ __forceinline__ void wave_lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Pins 16 register values at this point of the instruction stream (no instructions): the
// updates before it are issued before the ones after it. Keeps a right-looking sweep
// right-looking (the scheduler otherwise regroups the FMAs per element, a dependent chain of
// c FMAs for element c).
__device__ __forceinline__ void pin16(double (&p)[16]) {
  asm volatile("" : "+v"(p[0]), "+v"(p[1]), "+v"(p[2]), "+v"(p[3]), "+v"(p[4]), "+v"(p[5]),
               "+v"(p[6]), "+v"(p[7]), "+v"(p[8]), "+v"(p[9]), "+v"(p[10]), "+v"(p[11]),
               "+v"(p[12]), "+v"(p[13]), "+v"(p[14]), "+v"(p[15]));
}

// ---------------------------------------------------------------- potrf
// Two doubles; COH: device-coherent loads that bypass the CU's vector L1, which may hold stale
// lines of data another CU wrote (write-through) in the same launch. LFM_COH_NT (default):
// one 16-B nontemporal load (global_load_dwordx4 nt, L2-served like sc1); else two 8-B
// agent-scope relaxed atomic loads (sc1).
#ifndef LFM_COH_NT
#define LFM_COH_NT 1
#endif
#ifndef LFM_LEAF_SHARE
#define LFM_LEAF_SHARE 1
#endif
#ifndef LFM_KK_UNROLL
#define LFM_KK_UNROLL 1
#endif
typedef double double2v __attribute__((ext_vector_type(2)));
template <bool COH>
__device__ __forceinline__ double2 ld2(const double* p) {
  if (COH) {
    double2 v;
#if LFM_COH_NT
    const double2v t = __builtin_nontemporal_load(reinterpret_cast<const double2v*>(p));
    v.x = t.x;
    v.y = t.y;
#else
    v.x = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    v.y = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
    return v;
  }
  return *reinterpret_cast<const double2*>(p);
}
// One double, write-through (COH) or plain.
template <bool COH>
__device__ __forceinline__ void st1(double* p, double v) {
  if (COH) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}
// Two doubles at base + off (bytes, 16-B aligned) in one 16-B write-through (sc1) vector store:
// the wide form of st1<true> (an 8-B sc1 store is one fabric write, ≈2.7x the 16-B time per
// byte, MI355X_MICROARCH.md). base must be wave-uniform (a kernel argument or derived from one):
// it becomes the buffer resource. Range: off + 16 <= 2^31 - 1 (num_records); a store past it is
// dropped without a fault, so the helper serves the per-block workspaces only (the inverse,
// X_D, the chain workspace: at most 4 W^2 doubles = 13 MB at W = 640), never the matrix.
typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st2_wt(double* base, unsigned off, double a, double b) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
  const double2v v = {a, b};
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, v), r, off, 0, 16 /* sc1 */);
}
template <bool COH>
__device__ __forceinline__ double ld1(const double* p) {
  if (COH) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return *p;
}

__device__ __forceinline__ double rsqrt_nr(double x) {
  double y = __builtin_amdgcn_rsq(x);
  y = y * fma(-0.5 * x * y, y, 1.5);
  y = y * fma(-0.5 * x * y, y, 1.5);
  return y;
}

// One 256-thread workgroup, the 128x128 diagonal block in LDS, 16 columns per step:
//  (1) wave 0 factors the 16x16 diagonal sub-block in registers (lane = row);
//  (2) every wave solves rows below against it by substitution (lane = row; the L_D
//      entries are wave-uniform LDS reads);
//  (3) the rank-16 update of the trailing lower triangle on fp64 MFMA.
// After the loop the eight 16x16 diagonal inverses (dinv, for trsm_kernel) are built by
// the four waves, and logdet / the first failing pivot are reduced.
// PH: bit 0 = phase 1, bit 1 = phase 2, bit 2 = phase 3, bit 3 = global load / store of
// the block. The product path always runs PH = 15, in the
// chain kernel with bit 5 (the block load in one batch) and bit 7 (64-bit DPP broadcasts in
// the leaf), in its light mode also bit 4 (device-coherent block loads) and bit 6 (no block
// store: nothing reads it but row n).
// only the 36 lower 16x16 blocks of the 128x128 block, each 16 x 17 (padded) doubles:
// 78 KB, so the kernel fits on a CU beside one SYRK workgroup (look-ahead overlap)
constexpr int MB_DOUBLES = (NB / IB) * (NB / IB + 1) / 2 * IB * (IB + 1);

template <int PH>
__device__ __forceinline__ void potrf_block(double* __restrict__ Mb, double* __restrict__ A,
                                            int64_t lda, int64_t kb, int64_t npiv,
                                            double* __restrict__ dinv,
                                            double* __restrict__ parts, int k,
                                            int* __restrict__ status,
                                            double* __restrict__ Li = nullptr,
                                            unsigned long long* __restrict__ pst = nullptr) {
  // pst (diagnostics, NULL: off): s_memrealtime after the load (0), panel iterations 0, 3, 6
  // (1-3), the loop (4), inverse block row 6 (5) and 7 (6), the block store (7)
  auto pstamp = [&](int p) {
#ifndef LFM_PSTAMP_LEAF
    if (pst && threadIdx.x == 0) pst[p] = __builtin_amdgcn_s_memrealtime();
#endif
  };
  // diagnostics build (-DLFM_PSTAMP_LEAF): panel iteration 3 by phase and wave instead
  auto lstamp = [&](int ib, int p, int wv) {
#ifdef LFM_PSTAMP_LEAF
    if (pst && ib == 3 && threadIdx.x == 64 * wv) pst[p] = __builtin_amdgcn_s_memrealtime();
#endif
  };
  __shared__ double pvs[NB];  // unscaled pivots
  __shared__ double ipv[NB];  // 1 / L_cc
  __shared__ double red[4];
  __shared__ int redi[4];
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));  // opaque: the callers' loops do not hoist and hold its index math
  const int lane = tid & 63, w = tid >> 6;
  const int li = lane & 15, lk = lane >> 4;
#define MS(r, q) Mb[((((r) >> 4) * (((r) >> 4) + 1) / 2) + ((q) >> 4)) * (IB * (IB + 1)) + \
                    ((r) & 15) * (IB + 1) + ((q) & 15)]

  // block load: row r, 16-B chunks of the lower 16x16 blocks; two batches of 16 loads per
  // thread in flight (64 VGPRs), so the kernel fits in one bulk-SYRK workgroup's registers
  // (PH bit 5, the chain kernel with one workgroup per CU: all 32 at once)
  constexpr int LB = (PH & 32) ? 32 : 16;
#pragma unroll
  for (int hb = 0; hb < 32 / LB; ++hb) {
    double2 v[LB];
#pragma unroll
    for (int u = 0; u < LB; ++u) {
      const int idx = tid + 256 * (u + LB * hb), r = idx >> 6, c2 = idx & 63;
      if ((2 * c2) >> 4 <= r >> 4)
        v[u] = (PH & 8) ? ld2<(PH & 16) != 0>(&A[(kb + r) * lda + kb + 2 * c2])
                        : double2{(r == 2 * c2) ? 2.0 : 0.0, (r == 2 * c2 + 1) ? 2.0 : 0.0};
    }
#pragma unroll
    for (int u = 0; u < LB; ++u) {
      const int idx = tid + 256 * (u + LB * hb), r = idx >> 6, c2 = idx & 63;
      if ((2 * c2) >> 4 <= r >> 4) {
        MS(r, 2 * c2) = v[u].x;
        MS(r, 2 * c2 + 1) = v[u].y;
      }
    }
  }
  __syncthreads();

  // Look-ahead over the eight 16-column panels: after the rows below panel ib are solved,
  // wave 0 applies panel ib to the next diagonal 16x16 block alone and factors it (the serial
  // leaf) while waves 1-3 apply panel ib to the rest of the trailing triangle.
  // leaf: wave 0 factors diagonal block cb in registers (lane = row)
  auto leaf = [&](int cb) {
    const int c0 = cb * IB;
    double d[IB], pv[IB], yv[IB];
#pragma unroll
    for (int q = 0; q < IB; ++q) d[q] = (lane < IB && q <= lane) ? MS(c0 + li, c0 + q) : 0.0;
    // PH bit 7: 64-bit DPP moves (v_mov_b64_dpp, one instruction per broadcast) instead of
    // two 32-bit ones
    if constexpr ((PH & 128) != 0) {
      // pipelined: column c's update of column c + 1 first, then the pivot chain of c + 1
      // (broadcast, rsqrt, Newton) is issued ahead of c's remaining updates, whose latency it
      // hides; the same operations per element in the same order (bit-identical)
      double dc = row_bcast64(d[0], 0);
      if (kb + c0 >= npiv) dc = 1.0;
      double y = rsqrt_1nr(dc);
#pragma unroll
      for (int c = 0; c < IB; ++c) {
        pv[c] = dc;
        yv[c] = y;
        d[c] = (lane == c) ? dc * y : d[c] * y;
        if (c + 1 < IB) {
          d[c + 1] = fma(-d[c], row_bcast64(d[c], c + 1), d[c + 1]);
          double dn = row_bcast64(d[c + 1], c + 1);
          if (kb + c0 + c + 1 >= npiv) dn = 1.0;
          // rsqrt_1nr(dn) = r * fma(-0.5 dn * r, r, 1.5), its dependent steps spread over the
          // remaining updates in four chunks (scheduling fences keep the interleave: the wave
          // issues in order, so a dependent step stalls it unless independent work sits between)
          const double r = __builtin_amdgcn_rsq(dn);
          const double hh = -0.5 * dn;
          const int REM = IB - c - 2, K = (REM + 3) / 4;
          double t1 = 0.0, t2 = 0.0, yn = 0.0;
#pragma unroll
          for (int part = 0; part < 4; ++part) {
            // a chunk's broadcasts first, then its FMAs (each FMA would otherwise wait on the
            // broadcast issued just before it)
            double bq[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {  // K <= 4 (REM <= 14)
              const int q = c + 2 + part * K + i;
              if (i < K && q < IB) bq[i] = row_bcast64(d[c], q);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int q = c + 2 + part * K + i;
              if (i < K && q < IB) d[q] = fma(-d[c], bq[i], d[q]);
            }
            if (part == 0) t1 = hh * r;
            if (part == 1) t2 = fma(t1, r, 1.5);
            if (part == 2) yn = r * t2;
            __builtin_amdgcn_sched_barrier(0);
          }
          dc = dn;
          y = yn;
        }
      }
    } else {
#pragma unroll
      for (int c = 0; c < IB; ++c) {
        double dc = row_bcast(d[c], c);
        if (kb + c0 + c >= npiv) dc = 1.0;
        const double y = rsqrt_1nr(dc);
        pv[c] = dc;
        yv[c] = y;
        d[c] = (lane == c) ? dc * y : d[c] * y;
#pragma unroll
        for (int q = c + 1; q < IB; ++q) d[q] = fma(-d[c], row_bcast(d[c], q), d[q]);
      }
    }
    if (lane < IB) {
#pragma unroll
      for (int q = 0; q < IB; ++q)
        if (q <= lane) MS(c0 + lane, c0 + q) = d[q];
    }
    // the pivots are wave-uniform after the broadcasts: lane c keeps pivot c
    double pvl = 0.0, yvl = 0.0;
#pragma unroll
    for (int c = 0; c < IB; ++c) {
      pvl = (lane == c) ? pv[c] : pvl;
      yvl = (lane == c) ? yv[c] : yvl;
    }
    if (lane < IB) {
      pvs[c0 + lane] = pvl;
      ipv[c0 + lane] = yvl;
    }
  };
  // one 16x16 tile (i0, j0) -= panel c0 rows i0 x rows j0 (fp64 MFMA), in LDS
  // (block offsets from wave-uniform block indices: scalar address math; the lane parts
  // (lk + 4 r) * 17 + li and li * 17 + 4 ks + lk are fixed per lane)
  auto tile_update = [&](int i0, int j0, int c0) {
    const int bi = __builtin_amdgcn_readfirstlane(i0 >> 4);
    const int bj = __builtin_amdgcn_readfirstlane(j0 >> 4);
    const int bc = __builtin_amdgcn_readfirstlane(c0 >> 4);
    double* C = Mb + (bi * (bi + 1) / 2 + bj) * (IB * (IB + 1));
    const double* Pa = Mb + (bi * (bi + 1) / 2 + bc) * (IB * (IB + 1));
    const double* Pb = Mb + (bj * (bj + 1) / 2 + bc) * (IB * (IB + 1));
    double4v acc;
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = C[(lk + 4 * r) * (IB + 1) + li];
#pragma unroll
    for (int ks = 0; ks < IB / 4; ++ks)
      acc = mfma16(-Pa[li * (IB + 1) + ks * 4 + lk], Pb[li * (IB + 1) + ks * 4 + lk], acc);
#pragma unroll
    for (int r = 0; r < 4; ++r) C[(lk + 4 * r) * (IB + 1) + li] = acc[r];
  };
  // lower 16x16 tiles of a triangle of side nrb, enumerated row by row: tile t -> (row, column)
  auto tri_tile = [](int t, int* ti, int* tj) {
    int r = 0;
    while ((r + 1) * (r + 2) / 2 <= t) ++r;
    *ti = r;
    *tj = t - r * (r + 1) / 2;
  };
  // With Li (the full inverse is wanted), waves 1-3 build it in the time the look-ahead leaves
  // them: Dinv_I (16x16 inverse of L_II, forward substitution, lane = column) and the blocks
  // Linv_IJ = -Dinv_I sum_{K=J}^{I-1} L_IK Linv_KJ of block row I (fp64 MFMA; the 16x16
  // accumulator layout is the B-operand layout of the next product).
#define LI(r, q) Li[((((r) >> 4) * (((r) >> 4) + 1) / 2) + ((q) >> 4)) * (IB * (IB + 1)) + \
                    ((r) & 15) * (IB + 1) + ((q) & 15)]
  // PH bit 9: p <- p L^-T (16 columns, right-looking), pinned column by column, column c + 1
  // of L (and its 1 / L_cc) loaded while column c is applied (the pins are scheduling
  // boundaries). Ld: the 16x16 block (row stride 17), y: 1 / L_cc.
  auto sweep_pinned = [](double (&p)[IB], const double* Ld, const double* y) {
    double lc[IB], ln[IB], yc = y[0], yn = 0.0;
#pragma unroll
    for (int q = 1; q < IB; ++q) lc[q] = Ld[q * (IB + 1)];
#pragma unroll
    for (int c = 0; c < IB; ++c) {
      if (c + 1 < IB) {
        yn = y[c + 1];
#pragma unroll
        for (int q = c + 2; q < IB; ++q) ln[q] = Ld[q * (IB + 1) + c + 1];
      }
      p[c] = p[c] * yc;
#pragma unroll
      for (int q = c + 1; q < IB; ++q) p[q] = fma(-p[c], lc[q], p[q]);
      pin16(p);
      yc = yn;
#pragma unroll
      for (int q = c + 2; q < IB; ++q) lc[q] = ln[q];
    }
  };
  auto dinv_block = [&](int I) {
    const int c0 = I * IB;
    const int bd = __builtin_amdgcn_readfirstlane(I);
    const double* Ld = Mb + (bd * (bd + 1) / 2 + bd) * (IB * (IB + 1));
    double x[IB];
#pragma unroll
    for (int r = 0; r < IB; ++r) x[r] = (li == r) ? 1.0 : 0.0;
    // right-looking (the same terms in the same order per element as the left-looking sum,
    // one dependent FMA + multiply per step instead of r)
    if constexpr ((PH & 512) != 0) {
      sweep_pinned(x, Ld, ipv + c0);
    } else {
#pragma unroll
      for (int r = 0; r < IB; ++r) {
        x[r] = x[r] * ipv[c0 + r];
#pragma unroll
        for (int q = r + 1; q < IB; ++q) x[q] = fma(-Ld[q * (IB + 1) + r], x[r], x[q]);
      }
    }
    if (lane < IB) {
#pragma unroll
      for (int r = 0; r < IB; ++r) LI(c0 + r, c0 + lane) = x[r];
    }
  };
  auto linv_block = [&](int I, int J) {
    I = __builtin_amdgcn_readfirstlane(I);  // wave-uniform block indices: scalar offsets
    J = __builtin_amdgcn_readfirstlane(J);
    auto blk = [&](int bi, int bj) { return (bi * (bi + 1) / 2 + bj) * (IB * (IB + 1)); };
    double4v sacc = {0, 0, 0, 0};
    for (int K = J; K < I; ++K) {
      const double* a = Mb + blk(I, K);
      const double* b = Li + blk(K, J);
#pragma unroll
      for (int ks = 0; ks < IB / 4; ++ks)
        sacc = mfma16(a[li * (IB + 1) + 4 * ks + lk], b[(4 * ks + lk) * (IB + 1) + li], sacc);
    }
    const double* d = Li + blk(I, I);
    double4v o = {0, 0, 0, 0};
#pragma unroll
    for (int ks = 0; ks < IB / 4; ++ks) o = mfma16(d[li * (IB + 1) + 4 * ks + lk], sacc[ks], o);
    double* out = Li + blk(I, J);
#pragma unroll
    for (int r = 0; r < 4; ++r) out[(lk + 4 * r) * (IB + 1) + li] = -o[r];
  };
  if ((PH & 1) && w == 0) leaf(0);
  __syncthreads();
  pstamp(0);
#pragma unroll 1
  for (int ib = 0; ib < NB / IB; ++ib) {
    const int c0 = ib * IB;
    lstamp(ib, 0, 0);
    // (2) rows below: x_c = (p_c - sum_{q<c} x_q L[c][q]) / L_cc, swept right-looking: once
    // x_c is known it is subtracted from every later p_q at once. Each p_q still accumulates
    // its terms in increasing c (bit-identical to the left-looking sum), but the dependent
    // chain per column is one FMA and one multiply instead of c FMAs.
    const int nr = NB - c0 - IB;
    if ((PH & 2) && w * 64 < nr) {
      const bool act = tid < nr;
      const int row = c0 + IB + (act ? tid : 0);
      double p[IB];
#pragma unroll
      for (int q = 0; q < IB; ++q) p[q] = MS(row, c0 + q);
      const int bd = __builtin_amdgcn_readfirstlane(c0 >> 4);
      const double* Ld = Mb + (bd * (bd + 1) / 2 + bd) * (IB * (IB + 1));  // L[c0.., c0..]
      if constexpr ((PH & 512) != 0) {
        sweep_pinned(p, Ld, ipv + c0);
      } else {
#pragma unroll
        for (int c = 0; c < IB; ++c) {
          p[c] = p[c] * ipv[c0 + c];
#pragma unroll
          for (int q = c + 1; q < IB; ++q) p[q] = fma(-p[c], Ld[q * (IB + 1) + c], p[q]);
        }
      }
      if (act) {
#pragma unroll
        for (int q = 0; q < IB; ++q) MS(row, c0 + q) = p[q];
      }
    }
    lstamp(ib, 1, 0);
    __syncthreads();
    lstamp(ib, 2, 0);
    if (nr == 0) break;
    // (3) wave 0: next diagonal block, then its leaf; waves 1-3: the other trailing tiles
    const int nrb = nr / IB;
    // the early panels' wide trailing triangles: wave 0 takes its last k0 tiles after the leaf
    // (28 tiles -> 4, 21 -> 2, 15 -> 1), so the four waves reach the barrier together
    const int ntiles = nrb * (nrb + 1) / 2;
    const int k0 = LFM_LEAF_SHARE ? max(0, (ntiles - 11) / 4) : 0;
    if (w == 0) {
      if (PH & 4) {
        tile_update(c0 + IB, c0 + IB, c0);
        wave_lds_fence();
      }
      lstamp(ib, 3, 0);
      if (PH & 1) leaf(ib + 1);
      lstamp(ib, 4, 0);
      if (PH & 4) {
        for (int tc = ntiles - k0; tc < ntiles; ++tc) {
          int ti, tj;
          tri_tile(tc, &ti, &tj);
          tile_update(c0 + IB + ti * IB, c0 + IB + tj * IB, c0);
        }
      }
    } else if (PH & 4) {
      const int wu = __builtin_amdgcn_readfirstlane(w);  // wave-uniform: scalar tile walk
      for (int t = wu; t < ntiles - k0; t += 6) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int tc = t + 3 * u;
          if (tc >= ntiles - k0) break;
          int ti, tj;
          tri_tile(tc, &ti, &tj);
          tile_update(c0 + IB + ti * IB, c0 + IB + tj * IB, c0);
        }
      }
    }
    if (Li && w > 0) {
      // Dinv_ib (L_ib,ib final since leaf(ib)); block row ib - 1 (Dinv_{ib-1} from last pass)
      if (w == 1) dinv_block(ib);
      else
        for (int J = w - 2; J < ib - 1; J += 2) linv_block(ib - 1, J);
    }
    lstamp(ib, 5, 1);
    lstamp(ib, 6, 3);
    __syncthreads();
    lstamp(ib, 7, 0);
    if (ib == 0 || ib == 3 || ib == 6) pstamp(ib == 0 ? 1 : ib == 3 ? 2 : 3);
  }
  pstamp(4);
  if (Li) {
    // remaining: Dinv_7 with block row 6, then block row 7
    constexpr int L7 = NB / IB - 1;
    if (w == 0) dinv_block(L7);
    else
      for (int J = w - 1; J < L7 - 1; J += 3) linv_block(L7 - 1, J);
    __syncthreads();
    pstamp(5);
    for (int J = w; J < L7; J += 4) linv_block(L7, J);
    pstamp(6);
  }
#undef LI
  // inverses of the eight 16x16 diagonal blocks: wave w builds blocks w and w + 4,
  // lane c (< 16) column c by forward substitution; dinv[ib][r][c] = X[r][c]
  // (not needed with Li: the caller uses the full inverse)
#pragma unroll
  for (int h = 0; h < (Li ? 0 : 2); ++h) {
    const int ib = w + 4 * h, c0 = ib * IB;
    double x[IB];
#pragma unroll
    for (int r = 0; r < IB; ++r) {
      double sacc = (li == r) ? 1.0 : 0.0;
#pragma unroll
      for (int q = 0; q < r; ++q) sacc = fma(-MS(c0 + r, c0 + q), x[q], sacc);
      x[r] = sacc * ipv[c0 + r];
    }
    if (lane < IB) {
#pragma unroll
      for (int r = 0; r < IB; ++r) {
        dinv[(ib * IB + r) * IB + lane] = x[r];
      }
    }
  }
  // block store (lower triangle incl. diagonal)
  if ((PH & 8) && !(PH & 64)) {
#pragma unroll 8
    for (int u = 0; u < 32; ++u) {
      const int idx = tid + 256 * u, r = idx >> 6, c2 = idx & 63;
      if (2 * c2 <= r) {
        double2 v;
        v.x = MS(r, 2 * c2);
        v.y = MS(r, 2 * c2 + 1);  // past the diagonal: scratch (the upper triangle is unused)
        *reinterpret_cast<double2*>(&A[(kb + r) * lda + kb + 2 * c2]) = v;
      }
    }
  }
  pstamp(7);
  // logdet partial = 1/2 sum log(pivot) over real pivots; first non-positive pivot
  double lg = 0.0;
  int bad = STATUS_NONE;
  if (tid < NB && kb + tid < npiv) {
    const double dp = pvs[tid];
    lg = 0.5 * log(dp);
    if (!(dp > 0.0)) bad = (int)(kb + tid);
  }
  for (int o = 32; o > 0; o >>= 1) {
    lg += __shfl_xor(lg, o);
    bad = min(bad, __shfl_xor(bad, o));
  }
  if (lane == 0) {
    red[w] = lg;
    redi[w] = bad;
  }
  __syncthreads();
  if (tid == 0) {
    parts[k] = red[0] + red[1] + red[2] + red[3];
    const int b = min(min(redi[0], redi[1]), min(redi[2], redi[3]));
    if (b != STATUS_NONE) atomicMin(status, b);
  }
#undef MS
}

// out[k][j] = Linv[j][k] (the transposed inverse of the factored block: upper triangular,
// zeros below the diagonal), ld ldo, from Li (packed 16x16 blocks, built by potrf_block).
template <bool COH = false>
__device__ __forceinline__ void store_inverse_t(const double* __restrict__ Li,
                                                double* __restrict__ out, int64_t ldo) {
#define LI(r, q) Li[((((r) >> 4) * (((r) >> 4) + 1) / 2) + ((q) >> 4)) * (IB * (IB + 1)) + \
                    ((r) & 15) * (IB + 1) + ((q) & 15)]
  __syncthreads();
#pragma unroll 8
  for (int u = 0; u < NB * (NB / 2) / 256; ++u) {
    const int idx = threadIdx.x + 256 * u;
    const int k = idx / (NB / 2), j = 2 * (idx % (NB / 2));
    double2 v;
    v.x = j >= k ? LI(j, k) : 0.0;
    v.y = j + 1 >= k ? LI(j + 1, k) : 0.0;
    if (COH) {
      st2_wt(out, (unsigned)((k * ldo + j) * 8), v.x, v.y);
    } else {
      *reinterpret_cast<double2*>(&out[k * ldo + j]) = v;
    }
  }
#undef LI
}

// (256, 4): at most 128 VGPRs, so the factor fits in the registers one bulk-SYRK workgroup frees
// The block lives in dynamic LDS (MB_DOUBLES doubles, set at launch) so the occupancy target
// (4 waves / SIMD) holds at compile time and caps the kernel at 128 VGPRs.
template <int PH>
__global__ __launch_bounds__(256, 4) void potrf_diag_kernel(double* __restrict__ A, int64_t lda,
                                                           int64_t kb, int64_t npiv,
                                                           double* __restrict__ dinv,
                                                           double* __restrict__ parts, int k,
                                                           int* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) double Mb[];
  __builtin_amdgcn_s_setprio(3);  // critical path: win issue slots over co-resident SYRK waves
  potrf_block<PH>(Mb, A, lda, kb, npiv, dinv, parts, k, status);
}

// ------------------------------------------------------------ trsm (v2)
// Rows [s, Mp) of block column kb, 64 rows per workgroup, 16 rows per wave:
//   X_cb = (A_cb - sum_{q < cb} X_q L_{cb,q}^T) * Dinv_cb^T,  cb = 0..7 (16 columns each).
// The wave's rows live in LDS; the L_{cb,q} fragments (the factored diagonal block, shared
// by every workgroup, L2-resident) for column block cb+1 are loaded while cb computes,
// and the K chain is split over two accumulators.
// The solve proper on 64 rows already in LDS (sA, visible to every wave of the workgroup).
__device__ __forceinline__ void trsm_rows(double (*__restrict__ sA)[NB + 1],
                                          double* __restrict__ A, int64_t lda, int64_t r0,
                                          int64_t kb, const double* __restrict__ dinv) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const int wr = w * IB;
  const double* Lrow = A + (kb + li) * lda + kb + lk;  // L[li][lk]
  constexpr int NCB = NB / IB;
  double bf[2][NB / 4];
  double dv[2][IB / 4];
#pragma unroll
  for (int ks = 0; ks < IB / 4; ++ks) dv[0][ks] = dinv[li * IB + ks * 4 + lk];
  __syncthreads();
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
    const int cur = cb & 1, nxt = cur ^ 1;
    if (cb + 1 < NCB) {
#pragma unroll
      for (int st = 0; st < (cb + 1) * 4; ++st)
        bf[nxt][st] = Lrow[(int64_t)(cb + 1) * IB * lda + st * 4];
#pragma unroll
      for (int ks = 0; ks < IB / 4; ++ks)
        dv[nxt][ks] = dinv[(cb + 1) * IB * IB + li * IB + ks * 4 + lk];
    }
    double4v acc0, acc1 = {0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < 4; ++r) acc0[r] = sA[wr + lk + 4 * r][cb * IB + li];
#pragma unroll
    for (int st = 0; st < cb * 4; ++st) {
      if (st & 1) acc1 = mfma16(-sA[wr + li][st * 4 + lk], bf[cur][st], acc1);
      else acc0 = mfma16(-sA[wr + li][st * 4 + lk], bf[cur][st], acc0);
    }
    acc0 += acc1;
#pragma unroll
    for (int r = 0; r < 4; ++r) sA[wr + lk + 4 * r][cb * IB + li] = acc0[r];
    wave_lds_fence();
    double4v z = {0, 0, 0, 0};
#pragma unroll
    for (int ks = 0; ks < IB / 4; ++ks) z = mfma16(sA[wr + li][cb * IB + ks * 4 + lk], dv[cur][ks], z);
    wave_lds_fence();
#pragma unroll
    for (int r = 0; r < 4; ++r) sA[wr + lk + 4 * r][cb * IB + li] = z[r];
    wave_lds_fence();
  }
  // the wave's 16 rows back to HBM
  for (int idx = lane; idx < IB * (NB / 2); idx += 64) {
    const int r = idx / (NB / 2), q2 = idx - r * (NB / 2);
    double2 v;
    v.x = sA[wr + r][2 * q2];
    v.y = sA[wr + r][2 * q2 + 1];
    *reinterpret_cast<double2*>(&A[(r0 + wr + r) * lda + kb + 2 * q2]) = v;
  }
}

__global__ __launch_bounds__(256) void trsm_kernel_v2(double* __restrict__ A, int64_t lda, int64_t s,
                                                   int64_t kb, const double* __restrict__ dinv) {
  __shared__ double sA[64][NB + 1];
  __builtin_amdgcn_s_setprio(3);
  const int tid = threadIdx.x;
  const int64_t r0 = s + (int64_t)blockIdx.x * 64;
  for (int idx = tid; idx < 64 * (NB / 2); idx += 256) {
    const int r = idx / (NB / 2), q2 = idx - r * (NB / 2);
    const double2 v = *reinterpret_cast<const double2*>(&A[(r0 + r) * lda + kb + 2 * q2]);
    sA[r][2 * q2] = v.x;
    sA[r][2 * q2 + 1] = v.y;
  }
  trsm_rows(sA, A, lda, r0, kb, dinv);
}

// ----------------------------------------------------------------- syrk
// Trailing update of the lower triangle: for 128x128 tiles (ti >= tj) of rows/cols
// starting at s:  C[i][j] -= sum_q P[i][q] P[j][q],  P = A[:, kb:kb+NB].
// 4 waves as 2x2, each a 64x64 block of C held in registers. The product runs on
// v_mfma_f64_4x4x4_4b_f64 (72.7 TFLOP/s measured on MI355X, against 49 for
// v_mfma_f64_16x16x4_f64; scripts/probe_mfma.py). Lane maps (scripts/probe_mfma4_layout.py),
// with g = (lane >> 2) & 3 the block: A_g[i][k] at lane 16k + 4g + i, B_g[k][j] at lane
// 16k + 4g + j, D_g[i][j] at lane 16i + 4g + j. A is replicated over the four blocks
// (rows ir*4 + i) and each block owns 4 of 16 columns (jr*16 + 4g + j), so accumulator
// acc[ir][jr] holds C[ir*4 + (lane >> 4)][jr*16 + (lane & 15)]: 16 consecutive columns per
// 16 lanes, as the 16x16 layout. Per K step of 4: 16 A + 4 B fragments, 64 MFMAs.
// The K dimension (NB) is staged KB columns at a time through LDS, the next stage
// prefetched into registers while the current one feeds the MFMAs.
// mode 0: every lower tile; 1: only tile column 0 (the next block column, look-ahead);
// 2: every lower tile with tile column >= 1 (the rest).
// KD: depth of the update (columns kb .. kb+KD of A). CIO = false (diagnostics only) skips
// the C tile's HBM read and write.
// Lower tiles (tile row ti >= tile column tj, 128-wide tile columns) of the trailing matrix
// starting at row/column s, restricted to tile columns [tj_lo, tj_hi); T tile rows in all.
// Bands of at most 8 columns (look-ahead / in-panel updates) are enumerated column by
// column; otherwise tj_hi must be T and the band is a triangle. Update depth kd (multiple
// of KB): columns kb .. kb + kd of A. TR = tile rows (128, or 64 for latency-critical bands).
// DB: double-buffered LDS stages (one barrier per K step instead of two).
// acc[ir][jr] (C[wr + ir*4 + (lane>>4)][wc + jr*16 + (lane&15)] of a TR x 128 block; waves
// as 2 x 2) += sum_k Pi[i][k] Pj[j][k], k < kd. pi: row i0 of the i panel (k contiguous,
// row stride ldi). pj: BT = false, row j0 of the j panel (k contiguous, row stride ldj);
// BT = true, a K-major panel: element (k, j) at pj[k * ldj + j]. The SYRK callers hold -C in
// acc (negated once at load / store instead of per fragment). sP: LDS staging, (TR + ST) rows
// of KB + LDP doubles: rows [0, TR) panel i, rows [TR, TR + ST) panel j (j-major).
// Every thread of the (256-thread) workgroup must call it.

// KS: depth of one LDS stage (16 in the bulk kernels; 64 where one workgroup per CU has no
// neighbours to hide the global-load latency behind — the side stream's chain kernel).
template <int TR, bool BT = false, bool COH = false, int KS = KB>
__device__ __forceinline__ void gemm_accumulate(const double* __restrict__ pi, int64_t ldi,
                                                const double* __restrict__ pj, int64_t ldj,
                                                int kd, double (&acc)[TR / 8][4],
                                                double (*__restrict__ sP)[KS + LDP]) {
  constexpr int IRN = TR / 8;
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));  // opaque: lane offsets are recomputed, not held live
  const int lane = tid & 63, w = tid >> 6;
  const int wr = (w >> 1) * (TR / 2), wc = (w & 1) * 64;
  const int li = lane & 15, lk = lane >> 4, l3 = lane & 3;
  // staging: TR rows of panel i and 128 rows of panel j, KS doubles each; a row is CH double2
  // chunks, thread tid moves chunk (tid % CH) of rows tid / CH + RP u. K-major j panel:
  // thread tid moves the double2 (k = idx >> 6, j = 2 (idx & 63)) of idx = tid + 256u and
  // stores it transposed.
  static_assert(KS % 16 == 0 && KS <= 64, "stage depth");
  constexpr int CH = KS / 2, RP = 256 / CH;
  constexpr int NUI = TR / RP, NUJ = ST / RP, NU = NUI + NUJ;
  const int srow = tid / CH, sch = tid % CH;
  const double* gi = pi + srow * ldi + 2 * sch;
  const double* gj = BT ? pj + (tid >> 6) * ldj + 2 * (tid & 63) : pj + srow * ldj + 2 * sch;
  const int li32 = (int)(RP * ldi);
  const int lj32 = BT ? (int)(4 * ldj) : (int)(RP * ldj);
  double2 pre[NU];
  auto gload = [&](int k0) {
    // row offsets recomputed per call (opaque stride) rather than held as live 64-bit pointers
    int l32 = li32, m32 = lj32;
    asm volatile("" : "+v"(l32), "+v"(m32));
#pragma unroll
    for (int u = 0; u < NUI; ++u) pre[u] = ld2<COH>(gi + u * l32 + k0);
    const double* gjk = BT ? gj + (int64_t)k0 * ldj : gj + k0;
#pragma unroll
    for (int u = 0; u < NUJ; ++u) pre[NUI + u] = ld2<COH>(gjk + u * m32);
  };
  gload(0);
  for (int k0 = 0; k0 < kd; k0 += KS) {
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NUI; ++u) {
      double* d = &sP[srow + RP * u][2 * sch];
      d[0] = pre[u].x;
      d[1] = pre[u].y;
    }
#pragma unroll
    for (int u = 0; u < NUJ; ++u) {
      if (BT) {
        const int kr = (tid >> 6) + 4 * u, jc = 2 * (tid & 63);
        sP[TR + jc][kr] = pre[NUI + u].x;
        sP[TR + jc + 1][kr] = pre[NUI + u].y;
      } else {
        double* d = &sP[TR + srow + RP * u][2 * sch];
        d[0] = pre[NUI + u].x;
        d[1] = pre[NUI + u].y;
      }
    }
    __syncthreads();
    if (k0 + KS < kd) gload(k0 + KS);
    {
#pragma unroll LFM_KK_UNROLL
      for (int kk = 0; kk < KS; kk += 4) {
        double bb[4];
#pragma unroll
        for (int jr = 0; jr < 4; ++jr) bb[jr] = sP[TR + wc + jr * 16 + li][kk + lk];
#pragma unroll
        for (int h = 0; h < IRN / 8; ++h) {
          double a[8];
#pragma unroll
          for (int ir = 0; ir < 8; ++ir) a[ir] = sP[wr + (h * 8 + ir) * 4 + l3][kk + lk];
#pragma unroll
          for (int ir = 0; ir < 8; ++ir)
#pragma unroll
            for (int jr = 0; jr < 4; ++jr)
              acc[h * 8 + ir][jr] = mfma4(a[ir], bb[jr], acc[h * 8 + ir][jr]);
        }
      }
    }
  }
}

// gemm_accumulate on v_mfma_f64_16x16x4_f64: the same staging and the same products, acc as
// TR / 32 x 4 blocks of 16 x 16 (acc[rb][jr][r] = C[wr + 16 rb + 4 r + (lane >> 4)][wc + 16 jr
// + (lane & 15)] — element for element the map of gemm_accumulate's acc[4 rb + r][jr]). Per
// 4-deep k step a wave issues 2 TR / 64 A and 4 B fragment reads and 2 TR / 16 MFMAs of 2048
// flops (against 12 reads and 32 MFMAs of 512 flops on the 4x4x4 blocks).
template <int TR, bool BT = false, bool COH = false, int KS = KB, int CW = ST>
__device__ __forceinline__ void gemm_accumulate16(const double* __restrict__ pi, int64_t ldi,
                                                  const double* __restrict__ pj, int64_t ldj,
                                                  int kd, double4v (&acc)[TR / 32][CW / 32],
                                                  double (*__restrict__ sP)[KS + LDP]) {
  constexpr int RB = TR / 32, JB = CW / 32;  // 16 x 16 blocks per wave: RB rows, JB columns
  constexpr int CPR = CW / 2;                 // K-major j panel: double2 chunks per k row
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));  // opaque: lane offsets are recomputed, not held live
  const int lane = tid & 63, w = tid >> 6;
  const int wr = (w >> 1) * (TR / 2), wc = (w & 1) * (CW / 2);
  const int li = lane & 15, lk = lane >> 4;
  static_assert(KS % 16 == 0 && KS <= 64, "stage depth");
  constexpr int CH = KS / 2, RP = 256 / CH;
  constexpr int NUI = TR / RP, NUJ = CW / RP, NU = NUI + NUJ;
  static_assert(BT ? KS * CPR == 256 * NUJ : true, "K-major staging");
  const int srow = tid / CH, sch = tid % CH;
  const double* gi = pi + srow * ldi + 2 * sch;
  const double* gj = BT ? pj + (tid / CPR) * ldj + 2 * (tid % CPR) : pj + srow * ldj + 2 * sch;
  const int li32 = (int)(RP * ldi);
  const int lj32 = BT ? (int)((256 / CPR) * ldj) : (int)(RP * ldj);
  double2 pre[NU];
  auto gload = [&](int k0) {
    int l32 = li32, m32 = lj32;
    asm volatile("" : "+v"(l32), "+v"(m32));
#pragma unroll
    for (int u = 0; u < NUI; ++u) pre[u] = ld2<COH>(gi + u * l32 + k0);
    const double* gjk = BT ? gj + (int64_t)k0 * ldj : gj + k0;
#pragma unroll
    for (int u = 0; u < NUJ; ++u) pre[NUI + u] = ld2<COH>(gjk + u * m32);
  };
  gload(0);
  for (int k0 = 0; k0 < kd; k0 += KS) {
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NUI; ++u) {
      double* d = &sP[srow + RP * u][2 * sch];
      d[0] = pre[u].x;
      d[1] = pre[u].y;
    }
#pragma unroll
    for (int u = 0; u < NUJ; ++u) {
      if (BT) {
        const int kr = tid / CPR + (256 / CPR) * u, jc = 2 * (tid % CPR);
        sP[TR + jc][kr] = pre[NUI + u].x;
        sP[TR + jc + 1][kr] = pre[NUI + u].y;
      } else {
        double* d = &sP[TR + srow + RP * u][2 * sch];
        d[0] = pre[NUI + u].x;
        d[1] = pre[NUI + u].y;
      }
    }
    __syncthreads();
    if (k0 + KS < kd) gload(k0 + KS);
#pragma unroll LFM_KK_UNROLL
    for (int kk = 0; kk < KS; kk += 4) {
      double bb[JB], a[RB];
#pragma unroll
      for (int jr = 0; jr < JB; ++jr) bb[jr] = sP[TR + wc + jr * 16 + li][kk + lk];
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) a[rb] = sP[wr + rb * 16 + li][kk + lk];
#pragma unroll
      for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int jr = 0; jr < JB; ++jr) acc[rb][jr] = mfma16(a[rb], bb[jr], acc[rb][jr]);
    }
  }
}

// Source of a trailing update's panel rows: matrix row r (k = 0 at the panel's first column)
// starts at p + (r - r0) * ld. The factor's own block column: {A + kb, lda, 0}; a separate
// panel buffer holding rows r0 .. : {X, ldx, r0}.
struct Panel {
  const double* p;
  int64_t ld, r0;
};

// schedule 1's 64-row SYRK (syrk_kernel<., 64>): workgroups per CU in its launch bounds
#ifndef LFM_SLAB_WGS
#define LFM_SLAB_WGS 3
#endif
// schedule-3 MLL bulk super-panel width in block columns
#ifndef LFM_WBULK
#define LFM_WBULK 5
#endif
// the same for the gradient's bordered factorisation (its window keeps every step full width)
#ifndef LFM_WBORD
#define LFM_WBORD 4
#endif
// rest-triangle enumeration: tile rows in groups of Q, Q x Q supertiles within a group (1: row
// by row)
#ifndef LFM_SUPERTILE
#define LFM_SUPERTILE 6
#endif
// rectangular bands (the step kernel's next-super-panel columns) enumerated row by row (0:
// column by column)
#ifndef LFM_BAND_ROWS
#define LFM_BAND_ROWS 1
#endif
// Bulk trailing update (step_kernel's update units): K depth of one LDS stage (32: 130 VGPRs +
// 64 AGPRs, 2 waves / SIMD)
#ifndef LFM_STEP_KS
#define LFM_STEP_KS 16
#endif
// trailing-update tile body on v_mfma_f64_16x16x4_f64 (1) or the 4x4x4_4b blocks (0)
#ifndef LFM_MFMA16
#define LFM_MFMA16 1
#endif
// tall units (X_{s+1} = A21 Bd) in 64 x (128 / LFM_TALL_SPLIT) pieces
#ifndef LFM_TALL_SPLIT
#define LFM_TALL_SPLIT 2
#endif
// the chain's 32 x 32 products (gemm32) on v_mfma_f64_16x16x4_f64 (1) or 4x4x4_4b (0)
#ifndef LFM_G32_M16
#define LFM_G32_M16 1
#endif
// tall units dealt round-robin to the XCDs (1) or in contiguous ranges like the other roles (0)
#ifndef LFM_TALL_RR
#define LFM_TALL_RR 1
#endif
// round-robin deal in groups of the LFM_TALL_SPLIT pieces of one row block (1): the pieces that
// read the same A21 rows go to the same XCD back to back, so the second reads them from that
// XCD's L2; else (0) piece by piece, consecutive pieces on different XCDs (round 3)
#ifndef LFM_TALL_GROUP
#define LFM_TALL_GROUP 1
#endif
// workgroups of the tall segment: a multiple of 8 (XCDs), of 8 LFM_TALL_SPLIT when grouped
__host__ __device__ constexpr int64_t tall_grid(int64_t nt) {
  return (LFM_TALL_RR && LFM_TALL_GROUP) ? (nt + 8 * LFM_TALL_SPLIT - 1) / (8 * LFM_TALL_SPLIT) *
                                               (8 * LFM_TALL_SPLIT)
                                         : (nt + 7) / 8 * 8;
}
// C tile loads of the trailing update: device-coherent, or plain / nontemporal (LFM_C_NT bit 0;
// bit 1: nontemporal C stores)
#ifndef LFM_C_NT
#define LFM_C_NT 3
#endif
template <bool COH>
__device__ __forceinline__ double ldc(const double* p) {
  if (COH) return ld1<true>(p);
  if (LFM_C_NT & 1) return __builtin_nontemporal_load(p);
  return *p;
}

// The tile body of syrk_unit: C (TR x 128 at row i0, column j0) -= panel rows i0.. x rows j0..
// over depth kd; CLOAD = false: C starts from zero (not read).
// GEN: C is not read but generated from the gram tables (GramGen, a tile inside one gene pair
// of an aligned grid layout): the tile's Toeplitz windows and row / column tables staged in
// sP first, then gram_grid_aligned_kernel's arithmetic per element (bit-identical Sigma).
template <bool CIO, int TR, int KS, bool LDCOH, bool CLOAD, bool GEN = false>
__device__ __forceinline__ void syrk_tile(double* __restrict__ A, int64_t lda, Panel P, int kd,
                                          int64_t i0, int64_t j0, bool diag, bool coh,
                                          double (*__restrict__ sP)[KS + LDP],
                                          const GramGen* gen = nullptr) {
  constexpr int IRN = TR / 8;  // 4-row groups per wave (2 x 2 waves, TR/2 rows each)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = (w >> 1) * (TR / 2), wc = (w & 1) * 64;
  const int li = lane & 15, lk = lane >> 4;
  double* Cb = A + (i0 + wr + lk) * lda + j0 + wc + li;  // C[wr + lk][wc + li]
  const int ld4 = (int)(4 * lda);  // row-group stride (elements); 60 * ld4 < 2^31 for lda < 2^23

#if LFM_MFMA16
  double4v acc4[IRN / 4][4];
#define ACC(ir, jr) acc4[(ir) >> 2][jr][(ir) & 3]
#else
  double acc[IRN][4];
#define ACC(ir, jr) acc[ir][jr]
#endif
  if constexpr (GEN) {
    constexpr int WIN = ST + TR - 1;
    static_assert(4 * WIN + 3 * TR + 3 * ST <= (TR + ST) * (KS + LDP), "gram windows in sP");
    double* sWk = &sP[0][0];
    double* sXk = sWk + WIN;
    double* sWj = sXk + WIN;
    double* sXj = sWj + WIN;
    double* sPk = sXj + WIN;  // rows: Pt[k][tau], Et[j][tau], Qt[j][tau]
    double* sEj = sPk + TR;
    double* sQj = sEj + TR;
    double* sPj = sQj + TR;   // columns: Pt[j][tau'], Et[k][tau'], Qt[k][tau']
    double* sEk = sPj + ST;
    double* sQk = sEk + ST;
    const int Tn = gen->Tn, G = gen->G;
    const int64_t Wd = 2 * (int64_t)Tn - 1;
    const double* Wt = gen->tab;
    const double* Xt = Wt + (int64_t)G * Wd;
    const double* Pt = Xt + (int64_t)G * Wd;
    const double* Et = Pt + (int64_t)G * Tn;
    const double* Qt = Et + (int64_t)G * Tn;
    const double* Cm = Qt + (int64_t)G * Tn;
    const int j = gen->bg[i0 / Tn], k = gen->bg[j0 / Tn];
    const int tau0 = (int)(i0 % Tn), tp0 = (int)(j0 % Tn);
    const int dmin = tp0 - tau0 - (TR - 1);
    for (int e = tid; e < WIN; e += 256) {
      const int64_t d = dmin + e;
      sWk[e] = Wt[(int64_t)k * Wd + (Tn - 1) + d];
      sXk[e] = Xt[(int64_t)k * Wd + (Tn - 1) + d];
      sWj[e] = Wt[(int64_t)j * Wd + (Tn - 1) - d];
      sXj[e] = Xt[(int64_t)j * Wd + (Tn - 1) - d];
    }
    if (tid < TR) {
      sPk[tid] = Pt[(int64_t)k * Tn + tau0 + tid];
      sEj[tid] = Et[(int64_t)j * Tn + tau0 + tid];
      sQj[tid] = Qt[(int64_t)j * Tn + tau0 + tid];
    }
    if (tid < ST) {
      sPj[tid] = Pt[(int64_t)j * Tn + tp0 + tid];
      sEk[tid] = Et[(int64_t)k * Tn + tp0 + tid];
      sQk[tid] = Qt[(int64_t)k * Tn + tp0 + tid];
    }
    const double Cjk = Cm[(int64_t)j * G + k];
    __syncthreads();
#pragma unroll
    for (int ir = 0; ir < IRN; ++ir)
#pragma unroll
      for (int jr = 0; jr < 4; ++jr) {
        const int rl = wr + ir * 4 + lk, cl = wc + jr * 16 + li, e = cl - rl + (TR - 1);
        double v = sWk[e] + sWj[e];
        v = fma(-sXk[e], sPk[rl], v);
        v = fma(-sXj[e], sPj[cl], v);
        v = fma(-(sEk[cl] * sEj[rl]), sQk[cl] + sQj[rl], v);
        v = Cjk * v;
        if (i0 + rl == j0 + cl) v = (v + gen->da1) + gen->da2;
        ACC(ir, jr) = -v;
        if (jr == 3) __builtin_amdgcn_sched_barrier(0);  // one row group's reads at a time
      }
    __syncthreads();  // the windows are read: sP is the K stages' again
  } else {
#pragma unroll
    for (int ir = 0; ir < IRN; ++ir)
#pragma unroll
      for (int jr = 0; jr < 4; ++jr)
        ACC(ir, jr) = (CIO && CLOAD) ? -ldc<LDCOH>(&Cb[ir * ld4 + jr * 16]) : 0.0;
  }
#if LFM_MFMA16
  gemm_accumulate16<TR, false, LDCOH, KS>(P.p + (i0 - P.r0) * P.ld, P.ld,
                                          P.p + (j0 - P.r0) * P.ld, P.ld, kd, acc4, sP);
#else
  gemm_accumulate<TR, false, LDCOH, KS>(P.p + (i0 - P.r0) * P.ld, P.ld, P.p + (j0 - P.r0) * P.ld,
                                        P.ld, kd, acc, sP);
#endif

  int ld4s = ld4;
  asm volatile("" : "+v"(ld4s));  // recompute store addresses instead of keeping 64 pointers live
#pragma unroll
  for (int ir = 0; ir < IRN; ++ir)
#pragma unroll
    for (int jr = 0; jr < 4; ++jr) {
      const int64_t row = i0 + wr + ir * 4 + lk, col = j0 + wc + jr * 16 + li;
      if (CIO && (!diag || col <= row)) {
        // coh: device-coherent (write-through) stores, read by another XCD in flight
        if (coh)
          __hip_atomic_store(&Cb[ir * ld4s + jr * 16], -ACC(ir, jr), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        else if (LFM_C_NT & 2)
          __builtin_nontemporal_store(-ACC(ir, jr), &Cb[ir * ld4s + jr * 16]);
        else
          Cb[ir * ld4s + jr * 16] = -ACC(ir, jr);
      }
      if (!CIO && ACC(ir, jr) == 1.2345e300) Cb[0] = 0.0;  // keep the MFMAs live
    }
#undef ACC
}

// Unit b of a band / triangle enumeration -> (TR-row slab ti, 128-column tile tj), relative
// to the trailing matrix: tile columns [tj_lo, tj_hi), tile rows from ti0 (bands) / the
// triangle over tile columns [tj_lo, T). Host mirror of the triangle: rest_unit_tile
// (lfm_host.cpp).
template <int TR>
__device__ __forceinline__ void unit_tile(int T, int tj_lo, int tj_hi, int64_t b, int ti0,
                                          int* ti_out, int* tj_out) {
  constexpr int SUB = ST / TR;  // row tiles per 128 rows
  int ti, tj;  // ti in TR-row units
  if (LFM_BAND_ROWS && tj_hi - tj_lo <= kBandMaxCols && ti0 >= tj_hi) {
    // rectangular band (every row below the band's columns): row by row, so consecutive units
    // share a row panel and the band's few column panels stay in L2
    const int nb = tj_hi - tj_lo;
    const int64_t r = b / (nb * SUB);
    const int rem = (int)(b - r * nb * SUB);
    tj = tj_lo + rem / SUB;
    ti = SUB * (ti0 + (int)r) + rem % SUB;
  } else if (tj_hi - tj_lo <= kBandMaxCols) {
    // band: tile columns [tj_lo, tj_hi), tile rows max(tj, ti0) .. T - 1
    tj = tj_lo;
    while (b >= (int64_t)SUB * max(0, T - max(tj, ti0))) {
      b -= (int64_t)SUB * max(0, T - max(tj, ti0));
      ++tj;
    }
    ti = SUB * max(tj, ti0) + (int)b;
  } else {
    // triangle of 128-tiles over tile columns [tj_lo, T), SUB row slabs of TR rows per tile;
    // groups of LFM_SUPERTILE tile rows are enumerated in order (so a launch can skip the first
    // ones: b offset), within a group Q x Q supertiles in turn, tiles row by row within those:
    // consecutive units (one XCD's co-resident workgroups) then share row and column panels
    const int sub = (int)(b % SUB);
    b /= SUB;
    int a = (int)((sqrt(8.0 * (double)b + 1.0) - 1.0) * 0.5);
    while ((int64_t)(a + 1) * (a + 2) / 2 <= b) ++a;
    while ((int64_t)a * (a + 1) / 2 > b) --a;
    constexpr int Q = LFM_SUPERTILE;
    if constexpr (Q > 1) {
      const int R = a / Q, r0 = R * Q, qr = min(Q, T - tj_lo - r0);
      const int64_t off = b - (int64_t)r0 * (r0 + 1) / 2;
      const int64_t full = (int64_t)R * qr * Q;
      int lr, lc;
      if (off < full) {
        const int C = (int)(off / (qr * Q)), t = (int)(off % (qr * Q));
        lr = t / Q;
        lc = C * Q + t % Q;
      } else {
        const int d = (int)(off - full);
        lr = (int)((sqrt(8.0 * (double)d + 1.0) - 1.0) * 0.5);
        while ((lr + 1) * (lr + 2) / 2 <= d) ++lr;
        while (lr * (lr + 1) / 2 > d) --lr;
        lc = r0 + d - lr * (lr + 1) / 2;
      }
      tj = lc + tj_lo;
      ti = SUB * (r0 + lr + tj_lo) + sub;
    } else {
      tj = (int)(b - (int64_t)a * (a + 1) / 2) + tj_lo;
      ti = SUB * (a + tj_lo) + sub;
    }
  }
  *ti_out = ti;
  *tj_out = tj;
}

// One TR x 128 work unit of a band / triangle launch: C -= P_i P_j^T over panel depth kd,
// C the lower part of the trailing matrix of A starting at row / column s. b = the unit's
// index in the enumeration (unit_tile).
// Returns whether the unit's tile lies in the leading coh_lim x coh_lim tiles of the trailing
// matrix (stores then write through to memory: device-coherent, for an in-flight reader).
// LDCOH: C and panel loads device-coherent too (a reader of data written in the same launch).
template <bool CIO, int TR, bool COH = false, int KS = KB, bool LDCOH = false>
__device__ __forceinline__ bool syrk_unit(double* __restrict__ A, int64_t lda, int64_t s, Panel P,
                                          int kd, int T, int tj_lo, int tj_hi, int64_t b, int ti0,
                                          double (*__restrict__ sP)[KS + LDP], int coh_lim = 0,
                                          int64_t pad_after = INT64_MAX,
                                          int64_t pad_end = INT64_MAX,
                                          int64_t zero_from = INT64_MAX,
                                          const GramGen* gen = nullptr) {
  int ti, tj;  // ti in TR-row units
  unit_tile<TR>(T, tj_lo, tj_hi, b, ti0, &ti, &tj);

  const int64_t i0 = s + (int64_t)ti * TR, j0 = s + (int64_t)tj * ST;
  const bool diag = i0 < j0 + ST;  // the tile reaches the diagonal: keep col <= row only
  const bool in_lead = (i0 - s) / ST < coh_lim && (j0 - s) / ST < coh_lim;
  // rows in (pad_after, pad_end) are identity padding of the augmented matrix (their panel
  // entries are zero): nothing reads their update
  if (i0 > pad_after && i0 < pad_end && !in_lead) return false;
  const bool coh = COH || in_lead;
  // rows >= zero_from are zeros no update has written yet (the bordered matrix's border rows
  // entering the window; never initialised in memory): a tile body that does not load C. (A
  // per-element load-or-zero choice makes hipcc branch around every load and wait on each, +7 %
  // per evaluation; a selected base pointer costs 2 VGPRs, occupancy 4 -> 3 waves / SIMD.)
  if (i0 >= zero_from)
    syrk_tile<CIO, TR, KS, LDCOH, false>(A, lda, P, kd, i0, j0, diag, coh, sP);
  else if (gen && i0 + TR <= gen->n)
    syrk_tile<CIO, TR, KS, LDCOH, false, true>(A, lda, P, kd, i0, j0, diag, coh, sP, gen);
  else
    syrk_tile<CIO, TR, KS, LDCOH, true>(A, lda, P, kd, i0, j0, diag, coh, sP);
  return in_lead;
}

// XCD-aware order: workgroups are dealt round-robin to the 8 XCDs (each with its own L2), so
// XCD x is given the contiguous range [lo_x, hi_x) of the enumeration: the workgroups resident
// on one XCD then share panel rows instead of striding over them.
__device__ __forceinline__ void xcd_range(int64_t nunits, int x, int64_t* lo, int64_t* hi) {
  const int64_t q = nunits / 8, r = nunits % 8;
  *lo = x * q + min((int64_t)x, r);
  *hi = *lo + q + (x < r ? 1 : 0);
}

// Trailing update (mode by tile-column range, see syrk_unit); skip: units of the triangle
// enumeration left out at its start (tile rows already updated elsewhere).
template <bool CIO, int TR>
__global__ __launch_bounds__(256, TR == 64 ? LFM_SLAB_WGS : 2) void syrk_kernel(
    double* __restrict__ A, int64_t lda, int64_t s, Panel P, int kd, int T, int tj_lo, int tj_hi,
    int prio, int xcd_remap, int ti0, int64_t skip) {
  __shared__ double sP[TR + ST][KB + LDP];
  if (prio) __builtin_amdgcn_s_setprio(2);  // look-ahead bands: ahead of the bulk update
  int64_t b = blockIdx.x;
  if (xcd_remap && tj_hi - tj_lo > 8) {
    int64_t lo, hi;
    xcd_range(gridDim.x, (int)(b % 8), &lo, &hi);
    b = lo + b / 8;
  }
  syrk_unit<CIO, TR>(A, lda, s, P, kd, T, tj_lo, tj_hi, b + skip, ti0, sP);
}

// Device-side waits are bounded in TIME, on the 100 MHz constant clock (s_memrealtime), not
// in polls: `limit` ticks (ctx->wait_ticks, LFM_DEVICE_WAIT_MS; 2 s by default), so a wait
// starved by another tenant of the GPU ends after a known time whatever the poll rate, and the
// call re-runs on schedule 1 (lfm_api.hip). limit = 0 fails at once (the LFM_DEBUG_SPIN_LIMIT
// test knob). A wait also ends as soon as another wait of the call has recorded a timeout
// (`status`), so one stall drains the whole factorisation within one bound.
__device__ __forceinline__ unsigned long long wall_ticks() { return __builtin_amdgcn_s_memrealtime(); }

// Bounded relaxed / acquire spin on a device counter: true once *p >= target, false after
// `limit` ticks or once *status records a timeout (the caller records PANEL_TIMEOUT).
template <bool ACQ = true, int SLEEP = 2>
__device__ __forceinline__ bool spin_until(const unsigned* p, unsigned target, unsigned limit,
                                           const int* status = nullptr) {
  auto ready = [&] {
    return __hip_atomic_load(p, ACQ ? __ATOMIC_ACQUIRE : __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT) >= target;
  };
  if (ready()) return true;
  if (limit == 0) return false;
  const unsigned long long t0 = wall_ticks();
  for (unsigned it = 1; !ready(); ++it) {
    if ((it & 15) == 0) {
      if (wall_ticks() - t0 > limit) return false;
      if (status &&
          __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == PANEL_TIMEOUT)
        return false;
    }
    __builtin_amdgcn_s_sleep(SLEEP);
  }
  return true;
}

// One main-stream launch per super-panel step s (schedule 3): step s's trailing update from
// X_s (the next diagonal block excluded: chain_kernel applies it), then X_{s+1}. Roles of
// 64 x 128 units in blockIdx order (each segment padded to a multiple of 8 workgroups,
// XCD-contiguous within it):
//   ahead the next super-panel's columns below its diagonal block; each unit bumps
//         a_done[tile row]
//   rest  the remaining trailing triangle (optionally split around the tall units)
//   tall  X_{s+1} = A21 Bd_{s+1} for the rows below the next diagonal block: a unit waits for
//         the side stream's factor (chain_done) and for its rows' `ahead` units.
// Workgroups are dispatched in order per XCD, so a waiting `tall` unit never holds a slot an
// unfinished `ahead` unit of its XCD still needs; waits are bounded (status PANEL_TIMEOUT).
struct StepArgs {
  double* A;
  int64_t lda;
  int64_t s0;     // trailing matrix of step s starts at row / column s0 = K1
  Panel px;       // X_s (rows from s0)
  int kd, T, wn;  // depth W_s, trailing 128-tiles, next width in tiles
  int na, nr, nt;  // units per role
  int64_t tr0;    // tall: first row (K1 of step s + 1), W_{s+1} = tw * 128, K0_{s+1} = tk0
  int64_t tk0;
  int tw;
  const double* Bd;
  double* X;      // X_{s+1}, ld tw * 128, row tr0 first
  int64_t n;
  double* zvec;
  unsigned* a_done;  // [T] per tile row of step s (NULL: no wait)
  const unsigned* chain_done;  // NULL: no wait
  int* status;
  // inputs of chain(s + 2), which starts while this launch runs: the rest units of its block
  // (lead x lead leading tiles of the rest triangle) and the ahead units of its rows (tile
  // rows < wn + lead) write through to memory and bump *xready when done
  unsigned* xready;  // NULL: no chain waits on this launch
  int lead;
  unsigned spin;     // time bound of every device-side wait, ticks (PANEL_TIMEOUT past it)
  unsigned long long* stamps;  // diagnostics (NULL: off): [8] launch stamps, lfm_diag.h
  int64_t pad_end;   // rows in (n, pad_end) are skipped identity padding (INT64_MAX: every
                     // row past n; n + 1: none)
  // bordered matrix (the gradient's inverse): border row Mp + i is e_i in the first Mp columns
  // and zero after until the window reaches it, so it is never initialised in memory —
  // update units of rows >= zero_from start from C = 0, and the tall units of rows >=
  // copy_from (= Mp + K0: A21 is the identity there) copy Bd's row (row - copy_from)
  int64_t zero_from;
  int64_t copy_from;
  GramGen gen;       // gen.tab != NULL: the first step's update units generate Sigma (fused gram)
  int64_t rest_off;  // rest units of this launch are [rest_off, rest_off + nr) of the step's
                     // enumeration (the side-CU helper launch takes the tail of it)
  unsigned long long* trace;  // diagnostics (NULL: off): 4 words per workgroup (lfm_debug_trace)
  unsigned long long trace_tag;  // launch tag, bits 40+ of each record's last word
};

// Diagnostics: atomic max of the 100 MHz clock (or of its bitwise NOT: the earliest start)
__device__ __forceinline__ void stamp_max(unsigned long long* p, bool negate = false) {
  if (p && threadIdx.x == 0) {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    __hip_atomic_fetch_max(p, negate ? ~t : t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Unit of workgroup b (offset within its role's segment) of a step launch: *u, and *end (u >=
// *end: padding). Ahead and rest units are dealt to the XCDs in contiguous ranges (panel
// sharing in each XCD's L2); the tall units round-robin, so every XCD gets the same mix of
// depths, deepest first (contiguous ranges gave one XCD all the deepest column block and made
// it the launch's last by a whole unit: profiles/r03_unit_trace_*).
__device__ __forceinline__ void tall_or_xcd_range(int seg, int64_t cnt, int64_t b, int64_t* u,
                                                  int64_t* end) {
  if (seg == 2 && LFM_TALL_RR) {
    if (LFM_TALL_GROUP) {
      // workgroup b runs on XCD x = b % 8 at position p = b / 8 of its queue: group j = (p / S)
      // 8 + x, piece p % S (the segment is padded to 8 S workgroups: tall_grid)
      constexpr int S = LFM_TALL_SPLIT;
      const int64_t p = b / 8;
      *u = S * ((p / S) * 8 + b % 8) + p % S;
    } else {
      *u = b;
    }
    *end = cnt;
    return;
  }
  int64_t lo, hi;
  xcd_range(cnt, (int)(b % 8), &lo, &hi);
  *u = lo + b / 8;
  *end = hi;
}

// workgroups of a step launch's rest segment (a multiple of 8: one queue per XCD)
__host__ __device__ inline int64_t rest_wgs(const StepArgs& g) { return (int64_t)(g.nr + 7) / 8 * 8; }

__device__ __forceinline__ void bump_after_stores(unsigned* ctr) {
  __builtin_amdgcn_s_waitcnt(0);  // this thread's write-through stores have completed
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}


// tall unit u (row slab rb, column block cb, its part hf of LFM_TALL_SPLIT) of step s + 1:
// deepest column blocks first (longest units), so the launch ends on short ones; the split
// halves a unit's width so the launch's last round drains in shorter pieces
// Returns false when its device-side wait ran out (the workgroup then stops claiming units).
__device__ __forceinline__ bool tall_unit(const StepArgs& g, int64_t u, double (*sP)[KB + LDP],
                                          unsigned long long* const st,
                                          unsigned long long t_unit) {
  auto add_dur = [&](int slot) {
    if (threadIdx.x == 0)
      __hip_atomic_fetch_add(st + slot, __builtin_amdgcn_s_memrealtime() - t_unit,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  constexpr int TCW = NB / LFM_TALL_SPLIT;  // output columns per tall unit
  const int64_t nrb = g.nt / (g.tw * LFM_TALL_SPLIT);
  const int cb = g.tw - 1 - (int)(u / (nrb * LFM_TALL_SPLIT));
  const int64_t rq = u % (nrb * LFM_TALL_SPLIT);
  const int64_t rb = rq / LFM_TALL_SPLIT;
  const int c0 = cb * NB + (int)(rq % LFM_TALL_SPLIT) * TCW;  // first output column in X_{s+1}
  const int64_t i0 = g.tr0 + rb * 64;
  if (i0 > g.n && i0 < g.pad_end) return true;  // identity padding rows: their X is never read
  {
    __shared__ int ok;
    // relaxed polling and device-coherent operand loads below instead of an acquire fence:
    // an agent-scope acquire invalidates this XCD's L2 under the running bulk units
    if (threadIdx.x == 0) {
      int why = 0;
      bool good = !g.chain_done || spin_until<false>(g.chain_done, 1u, g.spin, g.status);
      if (!good) why = 1;
      // rows past step s's update (bordered: the border rows that entered the window with
      // super-panel s + 1, zero in every earlier panel column) have no ahead unit to wait for
      if (good && g.a_done && (i0 - g.s0) / ST < g.T) {
        good = spin_until<false>(&g.a_done[(i0 - g.s0) / ST], (unsigned)(2 * g.wn), g.spin,
                                 g.status);
        if (!good) why = 2;
      }
      if (!good) timeout_at(g.status, why);
      ok = good;
    }
    __syncthreads();
    if (!ok) return false;
    if (st) stamp_max(st + 2);
  }
  const int W = g.tw * NB;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (i0 >= g.copy_from) {
    // border rows: X = e_{row - copy_from} Bd, the row of Bd (written through by the chain)
    const double* src = g.Bd + (i0 - g.copy_from) * W + c0;
    double* dst = g.X + (i0 - g.tr0) * W + c0;
#pragma unroll 4
    for (int u = 0; u < 64 * TCW / 2 / 256; ++u) {
      const int idx = tid + 256 * u, r = idx / (TCW / 2), c2 = 2 * (idx % (TCW / 2));
      *reinterpret_cast<double2*>(&dst[r * W + c2]) = ld2<true>(&src[(int64_t)r * W + c2]);
    }
    if (st) {
      __syncthreads();
      stamp_max(st + 3);
      add_dur(6);
    }
    return true;
  }
  const int wr = (wv >> 1) * 32, wc = (wv & 1) * (TCW / 2);
  const int li = lane & 15, lk = lane >> 4;
  constexpr int JR = TCW / 32;  // 16-column blocks per wave
#if LFM_MFMA16
  double4v acc4[2][JR];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int jr = 0; jr < JR; ++jr) acc4[rb][jr] = (double4v){0.0, 0.0, 0.0, 0.0};
  gemm_accumulate16<64, true, true, KB, TCW>(g.A + i0 * g.lda + g.tk0, g.lda, g.Bd + c0, W,
                                             NB * (cb + 1), acc4, sP);
#define ACC(ir, jr) acc4[(ir) >> 2][jr][(ir) & 3]
#else
  static_assert(TCW == NB, "the 4x4x4 tile body has no split tall units");
  double acc[8][4];
#pragma unroll
  for (int ir = 0; ir < 8; ++ir)
#pragma unroll
    for (int jr = 0; jr < 4; ++jr) acc[ir][jr] = 0.0;
  gemm_accumulate<64, true, true>(g.A + i0 * g.lda + g.tk0, g.lda, g.Bd + cb * NB, W,
                                  NB * (cb + 1), acc, sP);
#define ACC(ir, jr) acc[ir][jr]
#endif
  double* Xb = g.X + (i0 - g.tr0 + wr + lk) * W + c0 + wc + li;
#pragma unroll
  for (int ir = 0; ir < 8; ++ir)
#pragma unroll
    for (int jr = 0; jr < JR; ++jr) {
      Xb[(ir * 4) * W + jr * 16] = ACC(ir, jr);
      if (i0 + wr + ir * 4 + lk == g.n) g.zvec[g.tk0 + c0 + wc + jr * 16 + li] = ACC(ir, jr);
    }
#undef ACC
  if (st) {
    __syncthreads();
    stamp_max(st + 3);
    add_dur(6);
  }
  return true;
}

// ran (diagnostics, NULL: off): thread 0 records role << 32 | unit of the unit it runs
template <int TR>
__device__ __forceinline__ void step_body(const StepArgs& g, unsigned long long* ran = nullptr) {
  constexpr int SUB = ST / TR;  // units per 128-row tile
  __shared__ double sPbuf[(64 + ST) * (LFM_STEP_KS + LDP)];
  double (*sP)[KB + LDP] = reinterpret_cast<double (*)[KB + LDP]>(sPbuf);
  double (*sPu)[LFM_STEP_KS + LDP] = reinterpret_cast<double (*)[LFM_STEP_KS + LDP]>(sPbuf);
  const int64_t b = blockIdx.x;
  // roles in blockIdx order: ahead (1), rest (2), tall (3), each padded to a multiple of 8
  const int cnt[3] = {g.na, g.nr, g.nt};
  const int64_t width[2] = {(int64_t)(g.na + 7) / 8 * 8, rest_wgs(g)};
  int seg = 0;
  int64_t base = 0;
  while (seg < 2 && b >= base + width[seg]) {
    base += width[seg];
    ++seg;
  }
  int64_t lo, hi;
  tall_or_xcd_range(seg, cnt[seg], b - base, &lo, &hi);
  const int64_t u = lo;
  if (u >= hi) return;
  const int role = seg + 1;
  if (ran && threadIdx.x == 0) *ran = ((unsigned long long)role << 32) | (unsigned long long)u;
  unsigned long long* const st = g.stamps;
  if (st) stamp_max(st, true);
  // diagnostics: summed unit durations per role (rest [5], tall [6], ahead [7]; 100 MHz)
  const unsigned long long t_unit = st ? __builtin_amdgcn_s_memrealtime() : 0;
  auto add_dur = [&](int slot) {
    if (threadIdx.x == 0)
      __hip_atomic_fetch_add(st + slot, __builtin_amdgcn_s_memrealtime() - t_unit,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  if (role == 1) {
    // device-coherent stores + a counter bump once they have completed: the tall units read
    // these rows with device-coherent loads (no L2 writeback / invalidate on either side)
    syrk_unit<true, TR, true, LFM_STEP_KS>(g.A, g.lda, g.s0, g.px, g.kd, g.T, 0, g.wn, u, g.wn, sPu,
                                           0, g.n, g.pad_end, g.zero_from,
                                           g.gen.tab ? &g.gen : nullptr);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    // 128-tile row of the unit (the band's enumeration order, syrk_unit)
    const int trow = LFM_BAND_ROWS ? g.wn + (int)(u / (SUB * g.wn))
                                   : g.wn + (int)(u % (SUB * (g.T - g.wn))) / SUB;
    if (threadIdx.x == 0 && g.a_done)
      __hip_atomic_fetch_add(&g.a_done[trow], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0 && g.xready && trow < g.wn + g.lead)
      __hip_atomic_fetch_add(g.xready, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (st) {
      stamp_max(st + 1);
      stamp_max(st + 3);
      add_dur(7);
    }
    return;
  }
  if (role == 2) {
    unsigned long long c0 = 0, r0 = 0;
    if (st) {
      c0 = __builtin_amdgcn_s_memtime();
      r0 = __builtin_amdgcn_s_memrealtime();
    }
    const bool lead = syrk_unit<true, TR, false, LFM_STEP_KS>(g.A, g.lda, g.s0, g.px, g.kd, g.T,
                                                              g.wn, g.T, u + g.rest_off, 0, sPu,
                                                              g.xready ? g.wn + g.lead : 0, g.n,
                                                              g.pad_end, g.zero_from,
                                                              g.gen.tab ? &g.gen : nullptr);
    if (lead) bump_after_stores(g.xready);
    if (st) {
      __syncthreads();
      stamp_max(st + 1);
      stamp_max(st + 3);
      if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(st + 4, __builtin_amdgcn_s_memtime() - c0, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(st + 5, __builtin_amdgcn_s_memrealtime() - r0, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    return;
  }
  tall_unit(g, u, sP, st, t_unit);
}

// Diagnostics (lfm_debug_trace): per workgroup {entry, exit} (s_memrealtime), the hardware
// id (HW_ID | XCC_ID << 32) and the launch tag | role << 32 | unit (role 0: padding)
template <int TR>
__device__ __forceinline__ void step_traced(const StepArgs& g) {
  __shared__ unsigned long long t0;  // in LDS: nothing held in registers across the body
  __shared__ unsigned long long ran;  // role << 32 | unit (0: padding, or nothing left to claim)
  if (threadIdx.x == 0) {
    t0 = __builtin_amdgcn_s_memrealtime();
    ran = 0;
  }
  __syncthreads();
  step_body<TR>(g, &ran);
  __syncthreads();
  if (threadIdx.x == 0) {
    const int64_t b = blockIdx.x;
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    unsigned long long* r = g.trace + 4 * b;
    r[0] = t0;
    r[1] = __builtin_amdgcn_s_memrealtime();
    r[2] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
    r[3] = (g.trace_tag << 40) | ran;
  }
}

// (256, 4): 128 VGPRs, 4 waves / SIMD (the zero-C tile body would otherwise take 134)
__global__ __launch_bounds__(256, 4) void step_kernel(StepArgs g) { step_body<64>(g); }
// The side-CU helper's launches (rest units only): the same body under its own name, so
// traces and counters keep the main-stream step launches apart
__global__ __launch_bounds__(256, 4) void helper_update_kernel(StepArgs g) { step_body<64>(g); }
// Both with the unit trace (lfm_debug_trace on): separate symbols, so the product kernels'
// code is the untraced body
__global__ __launch_bounds__(256, 4) void step_kernel_traced(StepArgs g) { step_traced<64>(g); }
__global__ __launch_bounds__(256, 4) void helper_update_kernel_traced(StepArgs g) {
  step_traced<64>(g);
}

// ---------------------------------------------------------- fused panel
// One block column of the look-ahead chain in one launch (w = 1 steps):
//   workgroups 0, 1   apply the pending rank-pkd update (panel columns pkb .. pkb + pkd) to the
//                     two 64-row slabs of the 128 x 128 diagonal block; workgroup 0 then waits
//                     for both and factors the block (potrf_block);
//   workgroups >= 2   each apply the pending update to 64 rows below the block, keep them in
//                     LDS, wait for the factor and solve them (trsm_rows).
// This replaces band-SYRK -> potrf -> trsm (three dependent launches) and their dispatch gaps.
// Order across workgroups: device-scope release / acquire on sync[1] (diagonal slabs written,
// +1 each) and sync[0] (factor written, = epoch). Workgroup 0 is dispatched first, so waiting
// workgroups never hold the slots it needs; a bounded wait still ends every workgroup (status
// PANEL_TIMEOUT) rather than hang.
constexpr size_t PANEL_LDS = (size_t)MB_DOUBLES * sizeof(double);
static_assert(MB_DOUBLES >= 64 * (NB + 1) && MB_DOUBLES >= (64 + ST) * (KB + LDP), "LDS union");

__device__ __forceinline__ bool wait_counter(unsigned* p, unsigned target, unsigned limit,
                                             const int* status) {
  __shared__ int ok;
  if (threadIdx.x == 0) ok = spin_until<true>(p, target, limit, status);
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return ok;
}

__global__ __launch_bounds__(256) void panel_kernel(double* __restrict__ A, int64_t lda,
                                                    int64_t kb, int64_t pkb, int pkd,
                                                    int64_t npiv, double* __restrict__ dinv,
                                                    double* __restrict__ parts, int k,
                                                    int* __restrict__ status,
                                                    unsigned* __restrict__ sync, unsigned epoch,
                                                    unsigned spin) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  __builtin_amdgcn_s_setprio(3);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = (w >> 1) * 32, wc = (w & 1) * 64;
  const int li = lane & 15, lk = lane >> 4;
  const int b = blockIdx.x;
  const int64_t i0 = b < 2 ? kb + 64 * b : kb + NB + 64 * (int64_t)(b - 2);
  double* Cb = A + (i0 + wr + lk) * lda + kb + wc + li;  // C[wr + lk][wc + li]
  const int ld4 = (int)(4 * lda);
  double acc[8][4];
#pragma unroll
  for (int ir = 0; ir < 8; ++ir)
#pragma unroll
    for (int jr = 0; jr < 4; ++jr) acc[ir][jr] = -Cb[ir * ld4 + jr * 16];
  if (pkd > 0)
    gemm_accumulate<64>(A + i0 * lda + pkb, lda, A + kb * lda + pkb, lda, pkd, acc,
                        reinterpret_cast<double (*)[KB + LDP]>(smem));
  if (b < 2) {
    // diagonal slab back to the matrix (the part above the diagonal is scratch)
#pragma unroll
    for (int ir = 0; ir < 8; ++ir)
#pragma unroll
      for (int jr = 0; jr < 4; ++jr) Cb[ir * ld4 + jr * 16] = -acc[ir][jr];
    __threadfence();
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add(&sync[1], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    if (b == 1) return;
    if (!wait_counter(&sync[1], 2u * epoch, spin, status)) {
      if (tid == 0) {
        timeout_at(status, 7);
        __hip_atomic_store(&sync[0], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
    potrf_block<15>(smem, A, lda, kb, npiv, dinv, parts, k, status);
    __threadfence();
    __syncthreads();
    if (tid == 0) __hip_atomic_store(&sync[0], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  // rows below the block: the solve's 64 x 129 LDS image (aliases the staging buffer)
  double (*sA)[NB + 1] = reinterpret_cast<double (*)[NB + 1]>(smem);
  __syncthreads();
#pragma unroll
  for (int ir = 0; ir < 8; ++ir)
#pragma unroll
    for (int jr = 0; jr < 4; ++jr) sA[wr + ir * 4 + lk][wc + jr * 16 + li] = -acc[ir][jr];
  if (!wait_counter(&sync[0], epoch, spin, status)) {
    if (tid == 0) timeout_at(status, 7);
    return;
  }
  trsm_rows(sA, A, lda, i0, kb, dinv);
}

// ---------------------------------------------------- schedule 3 chain (side stream)
// One launch per super-panel s on the side stream's own CUs (gridDim.x workgroups, one per
// CU, all co-resident): the whole factorisation of the diagonal block in the workspace,
// phases separated by grid barriers instead of kernel boundaries:
//   P0  Wk top = A[D] - X_{s-1}[D rows] X_{s-1}[D rows]^T (step s - 1's update of the block,
//       64 x 128 units), Wk bottom = identity
//   per block column c: potrf (workgroup 0) | panel solve of the rows below in Wk (64-row
//       units, D rows and identity rows) | update of the block's later columns (band units)
// and finally z (row n, when it falls in the block) and chain_done[s] = 1. Wk bottom ends as
// Bd = L11^{-T}, which the main stream's tall units multiply with.
struct ChainArgs {
  const double* A;
  int64_t lda;
  int64_t Kc;         // first row / column of the super-panel
  int w;              // width in 128-column blocks
  double* Wk;         // 2W x W, ld W
  int kd;             // W_{s-1}: depth of the pending update (0: none)
  int64_t n;
  double* dinv;
  double* linv;       // 128 x 128: transposed inverse of the current diagonal block (w > 1)
  double* parts;
  int* status;
  double* zvec;
  unsigned* bar;      // grid barrier counter (zeroed per call)
  unsigned* done;     // chain_done[s]
  unsigned long long* stamps;  // diagnostics (NULL: off): s_memrealtime per phase, [16]
  const unsigned* xready;  // NULL: inputs ready at launch; else wait for *xready >= xtarget and
  unsigned xtarget;        // read A[D] and the panel rows with device-coherent loads
  // PX (kd > 0): the block's rows of X_{s-1} = A[D rows, K0p .. K0p + kd) Bd_{s-1} are formed
  // here (into xd, ld kd) instead of waiting for the main stream's tall units
  int64_t K0p;             // first column of super-panel s - 1
  const double* Bdp;       // Bd_{s-1}: kd x kd, ld kd
  double* xd;              // W x kd scratch
  unsigned spin;           // time bound of the input wait, ticks (grid barriers: spin / 4)
};

// dynamic LDS of chain_kernel: the factor block and its inverse (packed 16x16 blocks)
constexpr size_t CHAIN_LDS = 2 * (size_t)MB_DOUBLES * sizeof(double);

// Grid barrier over the chain kernel's co-resident workgroups: release, count, acquire.
// Bounded: on timeout (or a timeout already recorded in *status) it returns false at once.
__device__ __forceinline__ bool grid_sync(unsigned* bar, unsigned target, int* status,
                                          unsigned limit) {
  __shared__ int ok;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    const bool good = spin_until<true, 1>(bar, target, limit, status);
    if (!good) timeout_at(status, 6);
    ok = good;
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return ok;
}

// Light grid barrier: no cache maintenance. Valid when every value another workgroup wrote
// before the barrier was stored write-through (agent-scope relaxed stores) and is read after it
// with device-coherent loads: the s_waitcnt orders this thread's stores before the arrival.
__device__ __forceinline__ bool grid_sync_light(unsigned* bar, unsigned target, int* status,
                                                unsigned limit) {
  __shared__ int ok;
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool good = spin_until<false, 1>(bar, target, limit, status);
    if (!good) timeout_at(status, 6);
    ok = good;
  }
  __syncthreads();
  return ok;
}


constexpr int CKS = 64;  // chain kernel GEMM stage depth
static_assert(2 * MB_DOUBLES >= (64 + ST) * (CKS + LDP), "chain LDS union");

// Small-tile GEMM for the chain's latency-bound phases: one 32 x 32 output tile per
// workgroup, so a 128-row block spreads over 16 workgroups instead of two 64 x 128 units
// (one CU's fp64 MFMA rate is 1/256 of the chip's: a 64 x 128 x 128 unit alone is ~7 us).
//   v[q] = sum_{k < kd} P[r][k] Q[k][c],  element (r, c) = ((tid + 256 q) >> 5, & 31)
// P: row-major, k contiguous (row r at pi + r ldi). Q: BT, K-major (element (k, c) at
// pj[k ldj + c]); !BT, j-major (element (k, c) at pj[c ldj + k]). kd: multiple of 128.
// Stages of 128 k are loaded with 16 coalesced 16-B loads per thread (the next stage is
// prefetched into registers while the current one is multiplied); the four waves each take
// 32 k of a stage and their partial tiles are summed through LDS at the end.
// LDS: smem[0, 2 * 32 * G32K) (operands) and then [0, 4 * 32 * 33) (partials, aliased).
constexpr int G32K = 129;  // LDS row stride of a 128-deep operand row (130: same time, A/B)
static_assert(2 * MB_DOUBLES >= 2 * 32 * G32K + 4 * 1024 && 2 * MB_DOUBLES >= 4 * 32 * 33,
              "gemm32 LDS (+ the in-chain solve's parked output tiles)");
template <bool BT, bool COH = false, bool PAIR = false>
__device__ __forceinline__ void gemm32(const double* __restrict__ pi, int64_t ldi,
                                       const double* __restrict__ pj, int64_t ldj, int kd,
                                       double (&v)[4], double* __restrict__ smem) {
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));  // opaque: index math is redone per call, not hoisted and held
  const int lane = tid & 63, w = tid >> 6;
  const int li = lane & 15, lk = lane >> 4;
  double* sA = smem;             // [32][G32K]: P rows
  double* sB = smem + 32 * G32K;  // [32][G32K]: Q columns (j-major)
#if LFM_G32_M16
  double4v acc4[2][2];  // 16 x 16 blocks: acc4[rb][jr][r] = element (16 rb + 4 r + lk, 16 jr + li)
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) acc4[rb][0] = acc4[rb][1] = (double4v){0.0, 0.0, 0.0, 0.0};
#define ACC(ir, jr) acc4[(ir) >> 2][jr][(ir) & 3]
#else
  double acc[8][2];
#pragma unroll
  for (int ir = 0; ir < 8; ++ir) acc[ir][0] = acc[ir][1] = 0.0;
#define ACC(ir, jr) acc[ir][jr]
#endif
  double2 pre[16];
  auto gload = [&](int k0) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int idx = tid + 256 * u;
      pre[u] = ld2<COH>(pi + (idx >> 6) * ldi + k0 + 2 * (idx & 63));
      pre[8 + u] = BT ? ld2<COH>(pj + (int64_t)(k0 + (idx >> 4)) * ldj + 2 * (idx & 15))
                      : ld2<COH>(pj + (idx >> 6) * ldj + k0 + 2 * (idx & 63));
    }
  };
  if (kd > 0) gload(0);
  for (int k0 = 0; k0 < kd; k0 += 128) {
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int idx = tid + 256 * u;
      double* d = sA + (idx >> 6) * G32K + 2 * (idx & 63);
      d[0] = pre[u].x;
      d[1] = pre[u].y;
      if (BT) {
        const int kr = idx >> 4, c = 2 * (idx & 15);
        sB[c * G32K + kr] = pre[8 + u].x;
        sB[(c + 1) * G32K + kr] = pre[8 + u].y;
      } else {
        double* e = sB + (idx >> 6) * G32K + 2 * (idx & 63);
        e[0] = pre[8 + u].x;
        e[1] = pre[8 + u].y;
      }
    }
    __syncthreads();
    if (k0 + 128 < kd) gload(k0 + 128);
#pragma unroll
    for (int kk = 32 * w; kk < 32 * w + 32; kk += 4) {
      const double b0 = sB[li * G32K + kk + lk], b1 = sB[(16 + li) * G32K + kk + lk];
#if LFM_G32_M16
      const double a0 = sA[li * G32K + kk + lk], a1 = sA[(16 + li) * G32K + kk + lk];
      acc4[0][0] = mfma16(a0, b0, acc4[0][0]);
      acc4[0][1] = mfma16(a0, b1, acc4[0][1]);
      acc4[1][0] = mfma16(a1, b0, acc4[1][0]);
      acc4[1][1] = mfma16(a1, b1, acc4[1][1]);
#else
      double a[8];
#pragma unroll
      for (int ir = 0; ir < 8; ++ir) a[ir] = sA[(ir * 4 + (lane & 3)) * G32K + kk + lk];
#pragma unroll
      for (int ir = 0; ir < 8; ++ir) {
        acc[ir][0] = mfma4(a[ir], b0, acc[ir][0]);
        acc[ir][1] = mfma4(a[ir], b1, acc[ir][1]);
      }
#endif
    }
  }
  __syncthreads();  // operand reads done: the partials alias them
  double* red = smem;  // [4][32][33]
#pragma unroll
  for (int ir = 0; ir < 8; ++ir)
#pragma unroll
    for (int jr = 0; jr < 2; ++jr) red[(w * 32 + ir * 4 + lk) * 33 + jr * 16 + li] = ACC(ir, jr);
#undef ACC
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    // PAIR: v[2h], v[2h + 1] = elements e, e + 1 with e = 2 tid + 512 h (one 16-B store each)
    const int e = PAIR ? 2 * tid + 512 * (q >> 1) + (q & 1) : tid + 256 * q, r = e >> 5, c = e & 31;
    v[q] = red[r * 33 + c] + red[(32 + r) * 33 + c] + red[(64 + r) * 33 + c] +
           red[(96 + r) * 33 + c];
  }
  __syncthreads();  // partials read: smem is free for the next call
}
// Every phase runs in 32 x 32 output tiles (gemm32) over all gridDim.x workgroups: one CU's
// fp64 rate is 1/256 of the chip's, so the latency-bound chain spreads each product thin.
// LIGHT (w = 1): every value one workgroup hands to another is stored write-through and
// loaded device-coherently, so the barriers, the input wait and the completion flag need no
// cache maintenance (an agent-scope fence costs ~1.7-3.5 us).
template <bool LIGHT>
__global__ __launch_bounds__(256) void chain_kernel(ChainArgs g) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int G = gridDim.x, wg = blockIdx.x, tid = threadIdx.x;
  const int W = g.w * NB;
  double* Aw = g.Wk - (g.Kc * W + g.Kc);  // the workspace with the matrix's row / column numbers
  unsigned nbar = 0;
  auto stamp = [&](int p) {
    if (g.stamps && wg == 0 && tid == 0 && p < 16) g.stamps[p] = __builtin_amdgcn_s_memrealtime();
  };
  auto sync = [&]() {
    return (LIGHT ? grid_sync_light : grid_sync)(g.bar, G * ++nbar, g.status, g.spin >> 2);
  };
  stamp(0);
  // the block's inputs come from the main stream's launch in flight: wait for its count
  if (g.xready) {
    __shared__ int okx;
    if (tid == 0) {
      okx = spin_until<false>(g.xready, g.xtarget, g.spin, g.status);
      if (!okx) timeout_at(g.status, 5);
    }
    __syncthreads();
    // one agent-scope acquire so the inputs below come through plain, cached loads (LIGHT:
    // device-coherent loads instead)
    if (!LIGHT) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (!okx) return;
  }
  stamp(14);
  if (g.kd > 0) {
    // PX in 32 x 32 tiles (K = 32 (cb + 1) rounded up to 128: Bd is upper triangular)
    const int nc = g.kd / 32, nu = (W / 32) * nc;
    for (int u = wg; u < nu; u += G) {
      const int cb = u % nc, rb = u / nc;
      const int kd = min(g.kd, (32 * (cb + 1) + 127) / 128 * 128);
      double v[4];
      gemm32<true, LIGHT, LIGHT>(g.A + (g.Kc + 32 * rb) * g.lda + g.K0p, g.lda, g.Bdp + 32 * cb,
                                 g.kd, kd, v, smem);
      if (LIGHT) {
        // element pairs, one 16-B write-through store each (xd: W x kd doubles, < 2^31 B)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int e = 2 * tid + 512 * h;
          st2_wt(g.xd, (unsigned)(((32 * rb + (e >> 5)) * g.kd + 32 * cb + (e & 31)) * 8), v[2 * h],
                 v[2 * h + 1]);
        }
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int e = tid + 256 * q;
          g.xd[(int64_t)(32 * rb + (e >> 5)) * g.kd + 32 * cb + (e & 31)] = v[q];
        }
      }
    }
    if (!sync()) return;
  }
  stamp(13);
  // P0: pending update of the block into the workspace, 32 x 32 lower tiles:
  // Wk[D] = A[D] - X X^T
  {
    const int nt = W / 32, ntile = nt * (nt + 1) / 2;
    for (int u = wg; u < ntile; u += G) {
      int ti = 0;
      while ((ti + 1) * (ti + 2) / 2 <= u) ++ti;
      const int tj = u - ti * (ti + 1) / 2;
      double v[4] = {0.0, 0.0, 0.0, 0.0};
      if (g.kd > 0)
        gemm32<false, LIGHT, LIGHT>(g.xd + (int64_t)32 * ti * g.kd, g.kd,
                                    g.xd + (int64_t)32 * tj * g.kd, g.kd, g.kd, v, smem);
      if (LIGHT) {
        // element pairs: one 16-B device-coherent load and one 16-B write-through store each
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int e = 2 * tid + 512 * h;
          const int il = 32 * ti + (e >> 5), jl = 32 * tj + (e & 31);
          const double2 a = ld2<true>(&g.A[(g.Kc + il) * g.lda + g.Kc + jl]);
          st2_wt(g.Wk, (unsigned)((il * W + jl) * 8), a.x - v[2 * h], a.y - v[2 * h + 1]);
        }
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int e = tid + 256 * q;
          const int64_t i = g.Kc + 32 * ti + (e >> 5), j = g.Kc + 32 * tj + (e & 31);
          Aw[i * W + j] = g.A[i * g.lda + j] - v[q];
        }
      }
    }
    // identity border (w = 1: Bd overwrites it whole, nothing reads it)
    for (int64_t idx = (int64_t)wg * 256 + tid; idx < (LIGHT ? 0 : (int64_t)W * W / 2);
         idx += (int64_t)G * 256) {
      const int r = (int)(idx / (W / 2)), c = 2 * (int)(idx % (W / 2));
      double2 v;
      v.x = (r == c) ? 1.0 : 0.0;
      v.y = (r == c + 1) ? 1.0 : 0.0;
      *reinterpret_cast<double2*>(&g.Wk[(int64_t)(W + r) * W + c]) = v;
    }
  }
  stamp(1);
  bool ok = sync();
  stamp(2);
  for (int c = 0; c < g.w && ok; ++c) {
    const int64_t kb = g.Kc + (int64_t)c * NB, r0 = kb + NB;
    // workgroup 0: factor block c and its full inverse; transposed into Bd directly when it is
    // the only block (w = 1: Bd = L11^{-T}), else into linv for the panel solve below
    if (wg == 0) {
      double* Li = smem + MB_DOUBLES;
      potrf_block<(LIGHT ? 127 : 47) | 128 | 512>(smem, Aw, W, kb, g.n, g.dinv, g.parts,
                                                  (int)(kb / NB), g.status, Li,
                                                  g.stamps && g.w == 1 ? g.stamps + 5 : nullptr);
      stamp(3 + 3 * c);
      store_inverse_t<LIGHT>(Li, g.w == 1 ? g.Wk + (int64_t)W * W : g.linv, g.w == 1 ? W : NB);
      stamp(4 + 3 * c);
    }
    if (g.w == 1) break;
    ok = sync();
    if (!ok) break;
    // panel solve of every workspace row below block c as a GEMM: X = A_c Linv_c^T
    const int64_t rows = g.Kc + 2 * W - r0;
    {
      // 32-row units, one workgroup each (the solve is in place: a unit owns its rows), the
      // four 32-column output tiles parked in LDS past gemm32's operands until all are formed
      double* park = smem + 2 * 32 * G32K;
      for (int64_t u = wg; u < rows / 32; u += G) {
        const int64_t ra = r0 + 32 * u;
#pragma unroll 1
        for (int jc = 0; jc < 4; ++jc) {
          double v[4];
          gemm32<true>(Aw + ra * W + kb, W, g.linv + 32 * jc, NB, NB, v, smem);
#pragma unroll
          for (int q = 0; q < 4; ++q) park[jc * 1024 + tid + 256 * q] = v[q];
        }
        __syncthreads();
#pragma unroll
        for (int jc = 0; jc < 4; ++jc)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int e = tid + 256 * q;
            Aw[(ra + (e >> 5)) * W + kb + 32 * jc + (e & 31)] = park[jc * 1024 + e];
          }
        __syncthreads();
      }
    }
    ok = sync();
    stamp(5 + 3 * c);
    if (!ok || c + 1 == g.w) break;
    const int hi = g.w - 1 - c;
    {
      // band update in 32 x 32 tiles: columns r0 .. r0 + 128 hi, every row below (diagonal
      // tiles whole: their upper part is never read)
      const int R32 = (int)(rows / 32), J32 = 4 * hi;
      int nt = 0;
      for (int jt = 0; jt < J32; ++jt) nt += R32 - jt;
      for (int u = wg; u < nt; u += G) {
        int jt = 0, rem = u;
        while (rem >= R32 - jt) {
          rem -= R32 - jt;
          ++jt;
        }
        const int it = jt + rem;
        const int64_t ra = r0 + 32 * it, ca = r0 + 32 * jt;
        double v[4];
        gemm32<false>(Aw + ra * W + kb, W, Aw + ca * W + kb, W, NB, v, smem);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int e = tid + 256 * q;
          Aw[(ra + (e >> 5)) * W + ca + (e & 31)] -= v[q];
        }
      }
    }
    ok = sync();
  }
  if (wg == 0) {
    if (g.n >= g.Kc && g.n < g.Kc + W) {
      const int r = (int)(g.n - g.Kc);
      // LIGHT (w = 1): row n of the factor from LDS (the block was not stored back)
      for (int c = tid; c < W; c += 256)
        g.zvec[g.Kc + c] = !LIGHT ? g.Wk[(int64_t)r * W + c]
                           : c <= r ? smem[(((r >> 4) * ((r >> 4) + 1) / 2) + (c >> 4)) *
                                               (IB * (IB + 1)) + (r & 15) * (IB + 1) + (c & 15)]
                                    : 0.0;
    }
    // LIGHT: Bd went out write-through and its readers load it device-coherently; zvec, parts
    // and status are read by later launches only
    if (LIGHT) __builtin_amdgcn_s_waitcnt(0);
    else __threadfence();
    __syncthreads();
    stamp(15);
    if (tid == 0)
      __hip_atomic_store(g.done, 1u, LIGHT ? __ATOMIC_RELAXED : __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Start-up check for schedule 3: can gridDim.x chain-sized workgroups (CHAIN_LDS each, so one
// per CU) be resident together on the side stream's CUs? Each arrives at a counter and waits
// (bounded, ~0.1 s) for all; ok[0] = 1 when every one saw the full count.
__global__ __launch_bounds__(256) void coresident_kernel(unsigned* bar, int* ok) {
  extern __shared__ double pad[];
  if (threadIdx.x == 0) {
    pad[0] = 0.0;
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned it = 0;
    while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gridDim.x &&
           ++it < (1u << 20))
      __builtin_amdgcn_s_sleep(2);
    if (it >= (1u << 20)) atomicExch(ok, 0);
  }
}

int chain_coresident(lfm_ctx* ctx, hipStream_t st, int G, bool* good) {
  hipFuncSetAttribute(reinterpret_cast<const void*>(&coresident_kernel),
                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)CHAIN_LDS);
  unsigned* d = nullptr;
  hipError_t e = hipMalloc((void**)&d, 16);
  if (e != hipSuccess) return hip_fail(ctx, e, "coresident probe");
  const unsigned init[2] = {0u, 1u};
  hipMemcpyAsync(d, init, 8, hipMemcpyHostToDevice, st);
  hipLaunchKernelGGL(coresident_kernel, dim3((unsigned)G), dim3(256), CHAIN_LDS, st, d,
                     reinterpret_cast<int*>(d + 1));
  unsigned h[2] = {0u, 0u};
  hipMemcpyAsync(h, d, 8, hipMemcpyDeviceToHost, st);
  e = hipStreamSynchronize(st);
  hipFree(d);
  *good = e == hipSuccess && h[0] == (unsigned)G && h[1] == 1u;
  return hip_fail(ctx, e, "coresident probe");
}

// ------------------------------------------------------------- finalize
// z = L^{-1} r: columns c < zsplit from zvec (schedule 3 keeps the panels out of A), the rest
// from row n of the factor.
__global__ __launch_bounds__(1024) void finalize_kernel(const double* __restrict__ A, int64_t lda,
                                                        int64_t n, const double* __restrict__ parts,
                                                        int nparts, const int* __restrict__ status,
                                                        int negative, double* __restrict__ out,
                                                        const double* __restrict__ zvec,
                                                        int64_t zsplit) {
  __shared__ double red[2][16];
  const int tid = threadIdx.x;
  double q = 0.0, ld = 0.0;
  for (int64_t c = tid; c < n; c += 1024) {
    const double z = c < zsplit ? zvec[c] : A[n * lda + c];
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
    out[4] = (double)status[1];
  }
}

__global__ void status_init_kernel(int* st) {
  st[0] = STATUS_NONE;
  st[1] = 0;  // which wait timed out first (timeout_at)
}


namespace {
struct Launcher {
  lfm_ctx* ctx;
  double* A;
  int64_t lda;
  int64_t Mp;   // rows of the (augmented) matrix being factored
  int64_t win;  // 0: trailing rows run to Mp; > 0: rows [s, s + win) only (bordered inverse)
  int64_t end(int64_t s) const { return win ? s + win : Mp; }
  void potrf(hipStream_t st, int64_t k, int64_t n) {
    hipEvent_t ev;
    prof_begin(ctx, K_POTRF, &ev, st);
    hipLaunchKernelGGL(potrf_diag_kernel<15>, dim3(1), dim3(256), MB_DOUBLES * sizeof(double), st,
                       A, lda, k * NB, n, ctx->linvT, ctx->parts, (int)k, ctx->status);
    prof_end(ctx, K_POTRF, ev, (double)NB * NB * NB / 3.0, 0, st);
  }
  // Panel solve of block column k over the rows below it, with the diagonal inverses.
  void trsm(hipStream_t st, int64_t k) {
    const int64_t s = (k + 1) * NB;
    const int64_t rows = end(s) - s;
    if (rows <= 0) return;
    hipEvent_t ev;
    prof_begin(ctx, K_TRSM, &ev, st);
    hipLaunchKernelGGL(trsm_kernel_v2, dim3((unsigned)(rows / 64)), dim3(256), 0, st, A, lda, s,
                       k * NB, ctx->linvT);
    prof_end(ctx, K_TRSM, ev, (double)rows * NB * NB, 2.0 * rows * NB * 8, st);
  }
  // Trailing update of tile columns [lo, hi) of the matrix starting at s0 (T = 128-tiles, in
  // 64-row slabs) with panel columns kb .. kb + kd. prio raises the look-ahead bands' waves.
  void syrk(hipStream_t st, int64_t s0, int64_t kb, int kd, int64_t T, int lo, int hi,
            int prio = 0) {
    if (T <= 0 || hi <= lo) return;
    hi = (int)std::min<int64_t>(hi, T);
    if (hi - lo > 8) hi = (int)T;  // wider than a band: the triangle of every column >= lo
    int64_t units = 0;
    double elems = 0;
    for (int tj = lo; tj < hi; ++tj) {
      units += 2 * (T - tj);
      elems += (double)(T - tj - 1) * ST * ST + (double)ST * (ST + 1) / 2;
    }
    if (units <= 0) return;
    hipEvent_t ev;
    prof_begin(ctx, K_SYRK, &ev, st);
    hipLaunchKernelGGL((syrk_kernel<true, 64>), dim3((unsigned)units), dim3(256), 0, st, A, lda,
                       s0, Panel{A + kb, lda, 0}, kd, (int)T, lo, hi, prio, 1, 0, (int64_t)0);
    prof_end(ctx, K_SYRK, ev, elems * 2.0 * kd, elems * 16.0, st);
  }
  int64_t tiles_from(int64_t s0) const { return (end(s0) - s0) / ST; }
  // Fused pending-update + factor + solve of block column k (panel_kernel).
  void panel(hipStream_t st, int64_t k, int64_t pkb, int pkd, int64_t n) {
    const int64_t kb = k * NB, s = kb + NB;
    const int64_t rows = std::max<int64_t>(end(s) - s, 0);
    const unsigned epoch = ++ctx->panel_epoch;
    hipEvent_t ev;
    prof_begin(ctx, K_PANEL, &ev, st);
    hipLaunchKernelGGL(panel_kernel, dim3((unsigned)(2 + rows / 64)), dim3(256), PANEL_LDS, st, A,
                       lda, kb, pkb, pkd, n, ctx->linvT, ctx->parts, (int)k, ctx->status,
                       ctx->psync, epoch, ctx->wait_ticks);
    prof_end(ctx, K_PANEL, ev,
             (double)NB * NB * NB / 3.0 + (double)rows * NB * NB + 2.0 * (rows + NB) * NB * pkd,
             0, st);
  }
  // Factor the super-panel of block columns [k, k + w): per column potrf + trsm, then the
  // update of the super-panel's remaining columns with it (K = 128). w = 1: one fused launch.
  void superpanel(hipStream_t st, int64_t k, int w, int64_t n) {
    if (w == 1) {
      panel(st, k, 0, 0, n);
      return;
    }
    for (int i = 0; i < w; ++i) {
      potrf(st, k + i, n);
      trsm(st, k + i);
      if (i + 1 < w) {
        const int64_t s0 = (k + i + 1) * NB;
        syrk(st, s0, (k + i) * NB, NB, tiles_from(s0), 0, w - 1 - i, 1);
      }
    }
  }
};
}  // namespace

// Diagnostics hook (liblfm_diag.so's lfm_probe_syrk, include/lfm_diag.h): ONE launch of the
// trailing-update kernel over a full lower triangle of T x T 128-tiles at depth kd on the
// n x n matrix ctx->A (operands prepared by the caller; X_s / X_{s+1} / counters after it).
// cio bit 0: C tile I/O (else the MFMAs alone), bit 4: on schedule 3's CU-masked bulk stream
// instead of every CU, bit 6: the step kernel's rest role (bit 5: without C loads). With bit
// 6, the rest of a w = 1 step launch's structure: bit 7 the ahead band (tile column 0 below
// the diagonal tile, the rest triangle then over columns >= 1, coherent stores, a_done
// bumps), bit 8 the tall units (X = A21 Bd at depth 128 for the rows below tile 0, no waits),
// bit 9 the panel read from a separate 128-wide buffer (the real steps' X_s) instead of A's
// own columns. Bit 11 (instead of bit 6): syrk_kernel's 128 x 128 units. Launches only: no
// kernel of its own, no allocation.
int probe_update_launch(lfm_ctx* ctx, hipStream_t st, int T, int kd, int cio, int64_t n,
                        size_t xb) {
  const unsigned units = (unsigned)((int64_t)T * (T + 1));
  const Panel pan{ctx->A, n, 0};
  if (cio & 64) {
    // the schedule-3 step kernel's rest role alone (the production unit: 16-deep stages,
    // 4 workgroups / CU, supertile order); bit 5: no C loads (C = 0, stores kept)
    StepArgs g{};
    g.A = ctx->A;
    g.lda = n;
    g.s0 = 512;
    g.px = pan;
    g.kd = kd;
    g.T = T;
    g.nr = (int)units;
    g.n = n;
    g.pad_end = INT64_MAX;
    g.spin = ctx->wait_ticks;
    g.zero_from = (cio & 32) ? 0 : INT64_MAX;
    g.copy_from = INT64_MAX;
    double* xs = ctx->A + (size_t)n * n;  // [X_s | X_{s+1} | counters]
    unsigned* ctr = reinterpret_cast<unsigned*>(xs + 2 * (xb / 8));
    if (cio & 512) g.px = Panel{xs, 128, 512};
    unsigned grid = (units + 7) / 8 * 8;
    if (cio & 128) {
      g.wn = 1;
      g.na = 2 * (T - 1);
      g.nr = (T - 1) * T;
      g.a_done = ctr;
      grid = (g.na + 7) / 8 * 8 + (g.nr + 7) / 8 * 8;
    }
    if (cio & 256) {
      g.tw = 1;
      g.tr0 = 512 + ST;
      g.tk0 = 0;
      g.nt = 2 * (T - 1) * LFM_TALL_SPLIT;
      g.Bd = ctx->A;
      g.X = xs + xb / 8;
      g.zvec = xs;
      g.a_done = nullptr;
      grid = (g.na + 7) / 8 * 8 + (g.nr + 7) / 8 * 8 + tall_grid(g.nt);
    }
    // unit-duration stamps in step slot 0 while lfm_debug_stamps is on (scripts/unit_time.py)
    g.stamps = ctx->dbg_stamps ? ctx->dbg_stamps + 256 * 16 : nullptr;
    hipLaunchKernelGGL(step_kernel, dim3(grid), dim3(256), 0, st, g);
  } else if (cio & 2048) {
    // 128 x 128 units (2 workgroups / CU, 64 x 64 per wave), the same triangle
    hipLaunchKernelGGL((syrk_kernel<true, 128>), dim3(units / 2), dim3(256), 0, st, ctx->A, n,
                       (int64_t)512, pan, kd, T, 0, T, 0, 1, 0, (int64_t)0);
  } else if (cio & 1) {
    hipLaunchKernelGGL((syrk_kernel<true, 64>), dim3(units), dim3(256), 0, st, ctx->A, n,
                       (int64_t)512, pan, kd, T, 0, T, 0, 1, 0, (int64_t)0);
  } else {
    hipLaunchKernelGGL((syrk_kernel<false, 64>), dim3(units), dim3(256), 0, st, ctx->A, n,
                       (int64_t)512, pan, kd, T, 0, T, 0, 1, 0, (int64_t)0);
  }
  return hip_fail(ctx, hipGetLastError(), "probe_update_launch");
}

bool chol_fuses_gram(const lfm_ctx* ctx, int mode, const GridLayout& lay, int64_t n) {
  return ctx->gram_fuse && lay.ok && lay.T % 256 == 0 && n % 256 == 0 && n >= 1024 &&
         s3_on(ctx) && mode != CHOL_SCHUR;
}

// Diagnostics: the next region of the unit trace (lfm_debug_trace) for a launch of `grid`
// workgroups, tagged with the launch count (bit 23: a side-CU helper launch); none while the
// trace is off or full
static void trace_launch(lfm_ctx* ctx, StepArgs& g, int64_t grid, bool helper) {
  g.trace = nullptr;
  if (!ctx->dbg_trace || ctx->dbg_trace_cur + grid > ctx->dbg_trace_cap) return;
  g.trace = ctx->dbg_trace + 4 * ctx->dbg_trace_cur;
  g.trace_tag = (unsigned long long)(ctx->dbg_trace_launch++ & 0x7fffff) | (helper ? 1ull << 23 : 0);
  ctx->dbg_trace_cur += grid;
}

int chol_factor_solve(lfm_ctx* ctx, double* A, int64_t lda, int64_t n, int64_t Mp, int negative,
                      double* d_out, int mode, const GramGen* gen) {
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&panel_kernel),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)PANEL_LDS);
    hipFuncSetAttribute(reinterpret_cast<const void*>(&potrf_diag_kernel<15>),
                        hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)(MB_DOUBLES * sizeof(double)));
    for (const void* f : {reinterpret_cast<const void*>(&chain_kernel<false>),
                          reinterpret_cast<const void*>(&chain_kernel<true>)})
      hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)CHAIN_LDS);
    attr = true;
  }
  // CHOL_MLL: factor the Mp x Mp augmented matrix (block columns holding pivots only).
  // CHOL_INVERSE: A is 2Mp x 2Mp, [[S_aug, .], [I, 0]]; all Mp/NB block columns of the top
  //   are eliminated with every trailing update restricted to the Mp-row window below the
  //   panel (the rows the identity border has reached), leaving -S_aug^{-1} in the bottom
  //   block: a Cholesky + triangular inverse + L^-T L^-1 product in N^3 flops on the same
  //   three kernels.
  // CHOL_SCHUR: eliminate the block columns holding the n pivots of an Mp x Mp matrix and
  //   apply every trailing update, so rows >= round_up(n, NB) end up holding the Schur
  //   complement (posterior covariance / mean correction, lfm_predict.hip).
  const bool bordered = mode == CHOL_INVERSE;
  const int64_t npb = (n + NB - 1) / NB;  // block columns that hold pivots
  const int64_t nblk = bordered ? Mp / NB : npb;
  int r = ensure(ctx, (void**)&ctx->parts, &ctx->parts_cap, (size_t)nblk * sizeof(double));
  if (r) return r;
  // schedule 3 for the MLL and for the bordered inverse (gradient); the Schur-complement
  // posterior keeps schedule 1
  const bool s3 = s3_on(ctx) && mode != CHOL_SCHUR;
  ctx->last_sched = s3 ? 3 : 1;
  // the bordered matrix's bottom rows [I, 0]: in memory for schedule 1; schedule 3 never reads
  // them before its window reaches them (StepArgs zero_from / copy_from)
  if (bordered && !s3) {
    r = launch_border_init(ctx, A, lda, Mp);
    if (r) return r;
  }
  // Step plan: super-panels of w = wbulk (5, schedule-3 MLL; else 4) block columns while the
  // trailing matrix has at least LFM_W4_MIN rows, w = 2 down to LFM_W2_MIN, then w = 1, so the
  // bulk trailing update runs with depth 128 w (C traffic per flop / w). Schedule 3: the bulk
  // width down to 6144 rows, then one or two w = 2 steps down to 5120 — the last deep update
  // would otherwise hold up the first w = 1 chains (measured 0.13-0.24 ms faster than going
  // straight to w = 1); its first super-panel is one block wide (its factor precedes any bulk
  // work).
  const int64_t w4min = ctx->w4min;
  // bulk width: 5 block columns (W = 640) for the MLL — its C traffic per flop is 4/5 of W = 512
  // and its chain still hides behind the update (A/B: -0.23..-0.26 ms per evaluation; W = 768
  // and 896 were slower, 1024 much slower); the bordered gradient keeps 4 (5 measured equal)
  const int wbulk = s3 ? (bordered ? LFM_WBORD : LFM_WBULK) : 4;
  const int64_t w2min = ctx->w2min >= 0 ? ctx->w2min : (s3 ? 5120 : 4096);
  const std::vector<std::pair<int64_t, int>> steps =
      plan_steps(nblk, Mp, NB, bordered, s3, wbulk, w4min, w2min, ctx->w0);
  const int S = (int)steps.size();
  r = ensure_events(ctx, 3 * (size_t)S + 3);  // [2 S + 3, 3 S + 3): LFM_S3_EVENTS=2
  if (r) return r;
  // fused gram (GramGen): in memory only the first block column (chain(0), X_0) and the next
  // super-panel's diagonal block (chain(1)); launch 0's update units generate the rest
  const bool fused = gen && s3 && S >= 2;
  if (gen) {
    const int64_t K10 = (int64_t)steps[0].second * NB;
    const int64_t K11 = fused ? (int64_t)(steps[1].first + steps[1].second) * NB : n;
    r = launch_gram_region(ctx, *gen, 0, n, 0, fused ? K10 : n, A, lda);
    if (!r && fused) r = launch_gram_region(ctx, *gen, K10, std::min(K11, n), K10, K11, A, lda);
    if (r) return r;
  }
  if (!s3 && !ctx->side) {
    // schedule 1's high-priority side stream, created on first use (schedule 3 never needs it)
    int least = 0, greatest = 0;
    hipDeviceGetStreamPriorityRange(&least, &greatest);
    if (hipStreamCreateWithPriority(&ctx->side, hipStreamNonBlocking, greatest) != hipSuccess)
      return hip_fail(ctx, hipErrorOutOfMemory, "side stream creation");
  }
  hipStream_t main = ctx->stream, side = ctx->side;
  hipEvent_t* ev = ctx->evs.data();  // [0]: inputs ready; E1_s = ev[1 + 2s]; E2_s = ev[2 + 2s]
  Launcher L{ctx, A, lda, bordered ? 2 * Mp : Mp, bordered ? Mp : 0};
  hipLaunchKernelGGL(status_init_kernel, dim3(1), dim3(1), 0, main, ctx->status);
  // the trailing update after the last super-panel matters only for the bordered rows
  auto trailing = [&](int s) { return s + 1 < S || mode != CHOL_MLL; };
  int64_t zsplit = 0;  // finalize: z columns below zsplit come from ctx->zvec
  if (s3) {
    // Schedule 3 on the CU-partitioned stream pair (LFM_SIDE_CUS CUs for the side stream),
    // ordered after / before ctx->stream's work. Side stream, per super-panel s (columns
    // [K0, K1), W = K1 - K0): chain_kernel factors only the W x W diagonal block, copied into a
    // workspace with an identity border, so it also yields Bd = L11^{-T}. Main stream: one
    // step_kernel per step applies step s's trailing update from X_s (the next super-panel's
    // columns first, then the rest) and finishes with X_{s+1} = A21 Bd_{s+1}, the tall panel
    // solve as a GEMM, once the side stream's factor of block s + 1 has landed. Cross-stream
    // order within a step is by device flags (ctx->flags), reset per call.
    // overlapped (a twin workspace of lfm_mll_multi_f64, ctx->ovl): chain(0), X_0, chain(1) and
    // launch 0 run on ctx->stream (the primary's overlap stream, behind this evaluation's gram),
    // the rest on the shared pair, after them and after the previous evaluation's launches
    const bool ovl = ctx->ovl && ctx->s3_events == 0 && S >= 2;
    hipEventRecord(ev[0], ctx->stream);
    main = ctx->m3;
    side = ctx->s3;
    if (!ovl) hipStreamWaitEvent(main, ev[0], 0);
    // the trailing matrix of a step whose super-panel ends at column K1: rows / columns
    // [K1, Mp) (MLL), or the Mp-row window [K1, K1 + Mp) the identity border has reached
    // (bordered: rows Mp + j are zero in panel columns < j; the window size is constant)
    auto rows_end = [&](int64_t K1) { return bordered ? K1 + Mp : Mp; };
    // MLL: rows past n are identity padding whose updates nothing reads; bordered: none is
    // skipped (the border rows have real entries in the padding columns, which are
    // eliminated too, so the padding rows' X must exist)
    const int64_t pad_end = bordered ? n + 1 : INT64_MAX;
    int wmax = 1;
    for (const auto& st : steps) wmax = std::max(wmax, st.second);
    const int64_t Wmax = (int64_t)wmax * NB, Tmax = Mp / ST + 1;
    // two workspaces: chain(s + 1) starts while the tall units of step s still read Bd_s
    r = ensure(ctx, (void**)&ctx->wk, &ctx->wk_bytes, (size_t)4 * Wmax * Wmax * sizeof(double));
    if (!r)
      r = ensure(ctx, (void**)&ctx->xbuf, &ctx->xbuf_bytes, (size_t)2 * Mp * Wmax * sizeof(double));
    if (!r) r = ensure(ctx, (void**)&ctx->zvec, &ctx->zvec_bytes, (size_t)Mp * sizeof(double));
    if (!r)
      r = ensure(ctx, (void**)&ctx->linv_full, &ctx->linv_full_bytes, (size_t)NB * NB * sizeof(double));
    if (!r) r = ensure(ctx, (void**)&ctx->xd, &ctx->xd_bytes, (size_t)Wmax * Wmax * sizeof(double));
    const size_t nflags = (size_t)S * (3 + Tmax);
    if (!r) r = ensure(ctx, (void**)&ctx->flags, &ctx->flags_bytes, nflags * sizeof(unsigned));
    if (r) return r;
    unsigned* chain_done = ctx->flags;     // [S]
    unsigned* a_done = ctx->flags + S;     // [S][Tmax]
    hipMemsetAsync(ctx->flags, 0, nflags * sizeof(unsigned), ovl ? ctx->stream : main);
    zsplit = n;
    auto xbuf = [&](int s) { return ctx->xbuf + (size_t)(s & 1) * Mp * Wmax; };
    unsigned* bars = a_done + (size_t)S * Tmax;  // [S] grid barrier counters of chain(s)
    unsigned* xready = bars + S;                  // [S] inputs of chain(s) landed (s >= 1)
    auto wkbuf = [&](int s) { return ctx->wk + (size_t)(s & 1) * 2 * Wmax * Wmax; };
    // launch j = s - 2 (step j's update) writes the inputs of chain(s), s >= 2: the block's
    // tiles (leading rest units, w_s (w_s + 1) 64-row slabs) and its rows of the columns of
    // super-panel s - 1 (leading ahead units, 2 w_s w_{s-1} slabs); chain(s) forms X_{s-1} of its
    // rows
    auto xtarget = [&](int s) {
      const int ws = steps[s].second;
      return (unsigned)(ws * (ws + 1) + 2 * ws * steps[s - 1].second);
    };
    // chain(s): factor block s on the side stream's CUs (one launch, see chain_kernel)
    auto chain = [&](int s, bool dev_wait = true) {
      ChainArgs c{};
      c.A = A;
      c.lda = lda;
      c.Kc = steps[s].first * NB;
      c.w = steps[s].second;
      c.Wk = wkbuf(s);
      if (s > 0) {
        if (dev_wait && s >= 2) {
          c.xready = xready + s;
          c.xtarget = xtarget(s);
        }
        c.kd = steps[s - 1].second * NB;
        c.K0p = steps[s - 1].first * NB;
        c.Bdp = wkbuf(s - 1) + (int64_t)c.kd * c.kd;
        c.xd = ctx->xd;
      }
      c.n = n;
      c.dinv = ctx->linvT;
      c.linv = ctx->linv_full;
      c.parts = ctx->parts;
      c.status = ctx->status;
      c.zvec = ctx->zvec;
      c.bar = bars + s;
      c.done = chain_done + s;
      c.spin = ctx->wait_ticks;
      c.stamps = ctx->dbg_stamps ? ctx->dbg_stamps + 16 * (size_t)std::min(s, 255) : nullptr;
      hipEvent_t pe;
      prof_begin(ctx, K_POTRF, &pe, side);
      hipLaunchKernelGGL(c.w == 1 ? chain_kernel<true> : chain_kernel<false>,
                         dim3((unsigned)ctx->side_cus), dim3(256), CHAIN_LDS, side, c);
      // algorithmic: the block's factor W^3 / 3, its pending update from X_{s-1} (the
      // block's lower elements x 2 kd) and its rows of X_{s-1} (W kd^2); issued adds the
      // block inverse (W^3) and the padded 32 x 32 tiles
      const double W = c.w * NB, kd = c.kd;
      prof_end(ctx, K_POTRF, pe, W * W * W / 3.0 + W * (W + 1) * kd + W * kd * kd, 0, side,
               W * W * W / 3.0 + W * W * W + W * W * kd + 2.0 * W * kd * kd);
    };
    // tall units of step s: rows [K1_s, Mp) x w_s column blocks
    auto tall_units = [&](int s) {
      const int64_t K1 = (steps[s].first + steps[s].second) * NB;
      return (int)((rows_end(K1) - K1) / 64 * steps[s].second * LFM_TALL_SPLIT);
    };
    // alg_adjust: algorithmic flops of the step's update done elsewhere (the side-CU helper's
    // tail, its own kernel class)
    auto launch_step = [&](StepArgs& g, double alg_adjust = 0.0) {
      g.n = n;  // padding rows past n are skipped
      g.pad_end = pad_end;
      if (!g.zero_from) g.zero_from = INT64_MAX;
      if (!g.copy_from) g.copy_from = INT64_MAX;
      g.spin = ctx->wait_ticks;
      const int64_t grid = (int64_t)(g.na + 7) / 8 * 8 + rest_wgs(g) + tall_grid(g.nt);
      if (grid == 0) return;
      // issued: every 64 x 128 unit in full (padding rows included), tall units as GEMMs with
      // the triangular inverse; algorithmic: the update of the unpadded augmented trailing
      // matrix (rows s0 .. n, residual row n included: it is the forward substitution) less
      // the next diagonal block (the chain's), and the triangular solve of the rows below
      // the next super-panel (rows .. n) against its W' x W' factor
      const double issued = ((double)g.na + g.nr) * 64 * ST * 2.0 * g.kd +
                            (double)g.nt * 64 * (ST / LFM_TALL_SPLIT) * NB * (g.tw + 1);
      double alg = 0.0;
      if (g.na + g.nr > 0) {
        // bordered: the whole Mp-row window is algorithmic (Cholesky + inverse = Mp^3)
        const double m = bordered ? (double)Mp : (double)(n - g.s0);
        const double d = std::min<double>(g.wn * NB, m);
        alg += 2.0 * g.kd * (m * (m + 1) / 2 + (bordered ? 0.0 : m) - d * (d + 1) / 2);
      }
      if (g.nt > 0) {
        const double W2 = (double)g.tw * NB;
        const int64_t rows = bordered ? rows_end(g.tk0) - g.tr0 : n + 1 - g.tr0;
        alg += (double)std::max<int64_t>(0, rows) * W2 * W2;
      }
      alg -= alg_adjust;
      trace_launch(ctx, g, grid, false);
      hipEvent_t pe;
      prof_begin(ctx, K_SYRK, &pe, main);
      hipLaunchKernelGGL(g.trace ? step_kernel_traced : step_kernel, dim3((unsigned)grid),
                         dim3(256), 0, main, g);
      prof_end(ctx, K_SYRK, pe, alg, 0, main, issued);
    };
    auto tall_args = [&](StepArgs& g, int s) {  // tall part of the step launch: step s's rows
      const int64_t K0 = steps[s].first * NB;
      const int w = steps[s].second;
      g.A = A;
      g.lda = lda;
      g.nt = tall_units(s);
      g.tr0 = K0 + (int64_t)w * NB;
      g.tk0 = K0;
      g.tw = w;
      g.Bd = wkbuf(s) + (int64_t)w * NB * w * NB;
      g.X = xbuf(s);
      if (bordered) g.copy_from = Mp + K0;
      g.n = n;
      g.zvec = ctx->zvec;
      g.chain_done = chain_done + s;
      g.status = ctx->status;
    };
    // update of step s (trailing matrix from K1_s), excluding the next diagonal block (none
    // after the last super-panel: the bordered mode's final update of its border block)
    auto update_args = [&](StepArgs& g, int s) {
      const int64_t K1 = (steps[s].first + steps[s].second) * NB;
      const int W = steps[s].second * NB, wn = s + 1 < S ? steps[s + 1].second : 0;
      const int T = (int)((rows_end(K1) - K1) / ST);
      g.A = A;
      g.lda = lda;
      g.s0 = K1;
      g.px = Panel{xbuf(s), W, K1};
      g.kd = W;
      g.T = T;
      g.wn = wn;
      if (bordered) g.zero_from = Mp + steps[s].first * NB;
      if (fused && s == 0) g.gen = *gen;
      g.na = 2 * wn * (T - wn);
      g.nr = (T - wn) * (T - wn + 1);  // two 64-row units per tile of the (T - wn)-tile triangle
      g.status = ctx->status;
    };
    // units of step s's rest triangle for the side-CU helper: the main launch of U unit-
    // equivalents takes D0 = U t / (S_m o) alone; giving x units to the helper's S_h slots,
    // which start after chain(s + 1) (Tc), balances at x t (1 / S_h + 1 / S_m) = o (D0 - Tc)
    const int helper_on = mode == CHOL_MLL || bordered ? ctx->helper : 0;
    const double helper_tc = ctx->helper_tc;    // chain(s + 1) + margin, us
    const double helper_min = ctx->helper_min;  // smallest D0 helped, us
    auto helper_share = [&](const StepArgs& g, int wnext) -> int64_t {
      if (!helper_on) return 0;
      return helper_units(g.kd, g.na, g.nr, g.nt / LFM_TALL_SPLIT, wnext, NB, ctx->cus,
                          ctx->side_cus, helper_tc, helper_min);
    };
    // side: chain(0) after the gram; every later chain(s) follows chain(s - 1) in stream order
    // and waits on the device for its inputs (xready[s]) from the main launch in flight
    if (ovl) {
      main = side = ctx->stream;
    } else {
      hipEventRecord(ev[0], main);
      hipStreamWaitEvent(side, ev[0], 0);
    }
    bool tail_marked = false;
    if (ctx->s3_events == 1) {
      // The same work ordered by stream events only (tall units in launches of their own after
      // the factor's event, chains after the tall launch's event) — for tools that serialise
      // dispatches (rocprofv3 --pmc), under which device-side waits between the two streams
      // could never be met.
      hipEvent_t* evc = ev + 1;      // [S] chain(s) done
      hipEvent_t* evt = ev + 1 + S;  // [S] X_s complete
      chain(0);
      hipEventRecord(evc[0], side);
      for (int s = 0; s < S; ++s) {
        if (s > 0) {
          StepArgs g{};  // step s - 1's trailing update only
          update_args(g, s - 1);
          launch_step(g);
        }
        hipStreamWaitEvent(main, evc[s], 0);
        StepArgs g{};  // X_s
        tall_args(g, s);
        g.chain_done = nullptr;
        launch_step(g);
        hipEventRecord(evt[s], main);
        if (s + 1 < S) {
          hipStreamWaitEvent(side, evt[s], 0);
          chain(s + 1, false);
          hipEventRecord(evc[s + 1], side);
        }
      }
      if (bordered) {
        StepArgs g{};  // the last super-panel's update of the border block
        update_args(g, S - 1);
        launch_step(g);
      }
    } else {
      // LFM_S3_EVENTS=2: these same launches, each also ordered by events after every launch
      // its device-side waits name (chain(s + 1) after launch s - 1, launch s after chain(s + 1)),
      // so a tool that serialises dispatches (rocprofv3 --pmc) counts the timed schedule's own
      // launches, one for one
      const bool serial = ctx->s3_events == 2;
      hipEvent_t* evC = ev + 2 * S + 3;  // [S] chain(s) done (serialised only)
      chain(0);
      if (serial) {
        hipEventRecord(evC[0], side);
        hipStreamWaitEvent(main, evC[0], 0);
      }
      {
        // X_0 once the first block is factored (its units wait for chain_done[0])
        StepArgs g{};
        tall_args(g, 0);
        launch_step(g);
      }
      hipEvent_t* evL = ev + 1;  // evL[2 s] = ev[1 + 2 s]: launch s done (main)
      hipEvent_t* evH = ev + 2;  // evH[2 s] = ev[2 + 2 s]: helper(s) done (side)
      bool helped = false;       // the previous step had a helper launch
      // algorithmic flops (profiling) of rest units [b0, b1) of a step's update: 2 kd per
      // updated lower element of their tiles, rows past n (identity padding) excluded
      auto units_alg = [&](int64_t s0u, int T, int wn, int kd, int64_t b0, int64_t b1) {
        double a = 0.0;
        for (int64_t b = b0; b < b1; ++b) {
          int ti, tj;
          rest_unit_tile(b, T, wn, LFM_SUPERTILE, &ti, &tj);
          const int64_t i0 = s0u + (int64_t)ti * 64, j0 = s0u + (int64_t)tj * ST;
          for (int64_t r = i0; r < i0 + 64 && (bordered || r <= n); ++r)
            a += (double)std::max<int64_t>(0, std::min<int64_t>(ST, r - j0 + 1));
        }
        return a * 2.0 * kd;
      };
      for (int s = 0; s + 1 < S; ++s) {
        if (serial && s >= 1) hipStreamWaitEvent(side, evL[2 * (s - 1)], 0);
        chain(s + 1);
        if (serial) {
          hipEventRecord(evC[s + 1], side);
          hipStreamWaitEvent(main, evC[s + 1], 0);
        }
        StepArgs g{};
        update_args(g, s);
        tall_args(g, s + 1);
        if (ctx->dbg_stamps) g.stamps = ctx->dbg_stamps + 256 * 16 + 8 * (size_t)std::min(s, 255);
        g.a_done = a_done + (size_t)s * Tmax;
        // the block after next: its tiles (rest) and rows (ahead) feed chain(s + 2)
        if (s + 2 < S) {
          g.xready = xready + s + 2;
          g.lead = steps[s + 2].second;
        }
        // Side-CU helper (LFM_HELPER): while the factor chain has slack (long launches), the
        // side stream runs the tail of this step's rest units after chain(s + 1), sized so it
        // ends with the main launch; launch s + 1 waits for it, chain(s + 2) follows it. Its
        // units store without write-through and bump no counter, so they never include a lead
        // tile of chain(s + 2).
        const int64_t total = g.nr;  // the step's rest enumeration
        const int64_t hu = s >= 1 && s + 2 < S
                               ? helper_clamp(helper_share(g, steps[s + 1].second), (int)total,
                                              g.T, g.wn, g.xready ? g.lead : 0, LFM_SUPERTILE)
                               : 0;
        g.nr = (int)(total - hu);
        const double alg_h =
            ctx->prof && hu > 0 ? units_alg(g.s0, g.T, g.wn, g.kd, total - hu, total) : 0.0;
        if (helped) hipStreamWaitEvent(main, evH[2 * (s - 1)], 0);
        // overlapped: the next evaluation may start once the launches before this evaluation's
        // tail have run (its first step below LFM_OVL_AT trailing rows)
        if (ctx->ovl && !tail_marked && s >= 1 && rows_end(g.s0) - g.s0 < ctx->ovl_at) {
          hipEventRecord(ctx->ovl_tail, main);
          tail_marked = true;
        }
        launch_step(g, alg_h);
        hipEventRecord(evL[2 * s], main);
        if (ovl && s == 0) {
          // the overlapped prologue ends with launch 0: the pair takes over after it (its tall
          // units waited for chain(1), so the prologue's chains are done too)
          main = ctx->m3;
          side = ctx->s3;
          hipStreamWaitEvent(main, evL[0], 0);
          hipStreamWaitEvent(side, evL[0], 0);
        }
        helped = hu > 0;
        if (hu > 0) {
          StepArgs h = g;
          h.na = 0;
          h.nt = 0;
          h.rest_off = total - hu;
          h.nr = (int)hu;
          h.stamps = nullptr;
          h.xready = nullptr;  // tail units: never the lead tiles
          trace_launch(ctx, h, (hu + 7) / 8 * 8, true);
          // X_s and step s's C input: launch s - 1 complete
          hipStreamWaitEvent(side, evL[2 * (s - 1)], 0);
          hipEvent_t pe;
          prof_begin(ctx, K_SIDE_SYRK, &pe, side);
          hipLaunchKernelGGL(h.trace ? helper_update_kernel_traced : helper_update_kernel,
                             dim3((unsigned)((hu + 7) / 8 * 8)), dim3(256), 0, side, h);
          prof_end(ctx, K_SIDE_SYRK, pe, alg_h, 0, side, (double)hu * 64 * ST * 2.0 * g.kd);
          hipEventRecord(evH[2 * s], side);
        }
      }
      if (bordered) {
        StepArgs g{};  // the last super-panel's update of the border block (-S_aug^{-1})
        update_args(g, S - 1);
        launch_step(g);
      }
    }
    if (ctx->ovl && !tail_marked) hipEventRecord(ctx->ovl_tail, main);
    hipEventRecord(ev[2 * S + 1], side);
    hipStreamWaitEvent(main, ev[2 * S + 1], 0);
  } else {
    // Schedule 1 (gradient / posterior modes, or no CU partition): super-panel s + 1 is
    // factored on the high-priority side stream while the main stream runs the bulk of step
    // s's trailing update.
    hipEventRecord(ev[0], main);
    hipStreamWaitEvent(side, ev[0], 0);
    L.superpanel(side, steps[0].first, steps[0].second, n);
    hipEventRecord(ev[1], side);
    for (int s = 0; s < S; ++s) {
      const int64_t k = steps[s].first;
      const int w = steps[s].second;
      const int64_t s0 = (k + w) * NB;
      const int64_t T = L.tiles_from(s0);
      hipStreamWaitEvent(main, ev[1 + 2 * s], 0);
      const bool nxt = s + 1 < S;
      const int wn = nxt ? steps[s + 1].second : 0;
      // main: the bulk of step s's trailing update (tile columns >= wn), depth 128 w
      if (trailing(s)) L.syrk(main, s0, k * NB, NB * w, T, wn, (int)T);
      hipEventRecord(ev[2 + 2 * s], main);
      if (nxt) {
        // side: the next super-panel's columns first (after main's previous bulk update,
        // which wrote the same tiles), then its factorisation
        if (s > 0) hipStreamWaitEvent(side, ev[2 + 2 * (s - 1)], 0);
        if (wn == 1) {
          L.panel(side, steps[s + 1].first, k * NB, NB * w, n);
        } else {
          L.syrk(side, s0, k * NB, NB * w, T, 0, wn, 1);
          L.superpanel(side, steps[s + 1].first, steps[s + 1].second, n);
        }
        hipEventRecord(ev[1 + 2 * (s + 1)], side);
      }
    }
  }
  r = hip_fail(ctx, hipGetLastError(), "cholesky launch");
  if (r) return r;
  hipEvent_t pe;
  prof_begin(ctx, K_FINALIZE, &pe, main);
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(1024), 0, main, A, lda, n, ctx->parts,
                     (int)npb, ctx->status, negative, d_out, ctx->zvec, zsplit);
  prof_end(ctx, K_FINALIZE, pe, 0, (double)n * 8, main);
  if (ctx->ovl) {
    // overlapped: the caller reads the result after ovl_done; ctx->stream (the overlap stream)
    // must not wait, the next evaluation's prologue is queued on it
    hipEventRecord(ctx->ovl_done, main);
  } else if (main != ctx->stream) {  // schedule 3 ran on the partitioned pair: back to ctx->stream
    hipEventRecord(ev[2 * S + 2], main);
    hipStreamWaitEvent(ctx->stream, ev[2 * S + 2], 0);
  }
  return hip_fail(ctx, hipGetLastError(), "finalize_kernel");
}

}  // namespace lfm
