// lfm_internal.h — shared declarations of the HIP implementation behind include/lfm.h.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/lfm.h"
#include "../../include/lfm_diag.h"
#include "lfm_host.h"

namespace lfm {

// Kernel classes tracked by the profiler (lfm_profile_*).
enum KClass {
  K_TABLES = 0,   // per-gene erf/exp tables of the structured gram
  K_GRAM_GRID,    // structured (shared uniform time grid) gram fill
  K_GRAM_DIRECT,  // general per-pair gram fill (any x, any flags)
  K_AUGMENT,      // residual row + padding rows of the augmented factor
  K_POTRF,        // diagonal-block factor + inverse (one workgroup)
  K_TRSM,         // panel solve  X = A * Linv^T  (fp64 MFMA)
  K_SYRK,         // trailing update C -= P P^T   (fp64 MFMA)
  K_FINALIZE,     // logdet + quadratic form -> scalar
  K_SMALL,        // one-workgroup-per-problem fused small-N MLL
  K_MEAN,         // mean_function
  K_GRAD,         // MLL gradient: W-weighted kernel-derivative reduction
  K_PANEL,        // fused pending update + diagonal factor + panel solve (one block column)
  K_SIDE_SYRK,    // schedule 3: the tail of a step's trailing update on the side CUs (helper)
  K_SMALL_GRAD,   // one-workgroup-per-problem value + gradient (and the in-kernel fit)
  K_NCLASS
};

extern const char* const kClassName[K_NCLASS];

struct ProfEvent {
  int cls;
  hipEvent_t a, b;
  double flops, bytes, issued;
};

}  // namespace lfm

struct lfm_ctx {
  int device = 0;
  hipStream_t stream = nullptr;  // main stream: gram fill, bulk trailing updates, finalize
  hipStream_t side = nullptr;    // high-priority look-ahead stream: panel factor + solve
  hipStream_t m3 = nullptr;      // schedule 3: bulk stream (CUs outside the chain's)
  hipStream_t s3 = nullptr;      // schedule 3: factor-chain stream (LFM_SIDE_CUS CUs)
  int side_req = 32;             // LFM_SIDE_CUS at creation: the reservation to (re)create
  int cus = 256;                 // compute units of the device
  std::vector<hipEvent_t> evs;   // cross-stream dependency events (timing disabled)
  std::string err;
  int nb = 128;  // Cholesky block size

  // device workspace, grown on demand
  double* A = nullptr;   size_t A_bytes = 0;     // augmented factor (Mp x Mp) / generic matrix
  double* tab = nullptr; size_t tab_bytes = 0;   // gene tables (fp64)
  float* tab32 = nullptr; size_t tab32_bytes = 0;// gene tables (fp32 copy)
  double* par = nullptr; size_t par_bytes = 0;   // packed hyperparameters + layout
  double* xin = nullptr; size_t xin_bytes = 0;   // staged x / y / loc inputs
  double* linvT = nullptr;                       // 8 x 16x16 inverses of the diagonal sub-blocks
  double* parts = nullptr; size_t parts_cap = 0; // per-block logdet partials
  int* status = nullptr;                         // [0] first failing pivot (INT_MAX = none)
  double* wk = nullptr; size_t wk_bytes = 0;     // schedule 3: diagonal block + identity border
  double* xbuf = nullptr; size_t xbuf_bytes = 0; // schedule 3: solved panel X = A21 L11^{-T}
  double* zvec = nullptr; size_t zvec_bytes = 0; // schedule 3: z = L^{-1} r
  double* linv_full = nullptr; size_t linv_full_bytes = 0; // schedule 3: 128x128 block inverse
  double* xd = nullptr; size_t xd_bytes = 0;     // schedule 3: the chain's rows of X_{s-1}
  unsigned* flags = nullptr; size_t flags_bytes = 0; // schedule 3: per-step device flags
  unsigned* psync = nullptr;                     // fused panel: [0] factor epoch, [1] slab count
  unsigned panel_epoch = 0;                      // fused panel launches so far
  int side_cus = 0;                              // CUs reserved for the side stream (LFM_SIDE_CUS)
  int sched = 3;                                 // look-ahead schedule 1 or 3 (LFM_SCHED)
  bool s3_yield = false;                         // this call runs schedule 1: nested in a
                                                 // shared hold of the device's tenancy lock
  int last_sched = 0;                            // schedule the last factorisation ran (diag)
  int s3_events = 0;  // LFM_S3_EVENTS: 1 schedule 3 ordered by events, 2 its timed launches serialised
  unsigned wait_ticks = 200000000u;              // device-side wait bound, 100 MHz ticks (2 s;
                                                 // LFM_DEVICE_WAIT_MS, LFM_DEBUG_SPIN_LIMIT)
  int64_t fallbacks = 0;                         // schedule-3 calls re-run on schedule 1 after a
                                                 // device-side wait timed out (lfm_ctx_fallbacks)
  bool grad_direct = false;                      // gradient: per-pair path only (LFM_GRAD_DIRECT)
  bool gram_fuse = true;                         // gram in the first update (LFM_GRAM_FUSE)
  // the other run-time knobs, also read once when the context is created
  int64_t w4min = 6144;   // LFM_W4_MIN: bulk super-panels while the trailing matrix has this many rows
  int64_t w2min = -1;     // LFM_W2_MIN: w = 2 down to this many rows (-1: 5120 schedule 3, else 4096)
  int w0 = 1;             // LFM_W0: width of schedule 3's first super-panel
  int helper = 1;         // LFM_HELPER: schedule 3's side-CU helper
  double helper_tc = 700, helper_min = 1200;  // LFM_HELPER_TC / LFM_HELPER_MIN, microseconds
  bool s3_fallback = true;   // LFM_S3_FALLBACK: re-run a stalled schedule-3 call on schedule 1
  double rccl_timeout_s = 300.0;  // LFM_RCCL_TIMEOUT_S: bound on every farm collective wait
  int farm_stall_ms = 0;  // LFM_DEBUG_FARM_STALL_MS: test stand-in for a late peer rank
  bool small_kernarg = true;  // LFM_SMALL_KERNARG: small batches' table in the kernel arguments
  double* gtab = nullptr; size_t gtab_bytes = 0; // gradient tables (grid layout)
  double* result = nullptr;                      // [0..] scalar results
  double* gacc = nullptr; size_t gacc_bytes = 0; // gradient accumulators + output

  unsigned long long* dbg_stamps = nullptr;     // lfm_debug_stamps: chain phases 256 x 16, then
                                                // step launches 256 x 8
  unsigned long long* dbg_trace = nullptr;      // lfm_debug_trace: 4 words per step-kernel unit
  int64_t dbg_trace_cap = 0, dbg_trace_cur = 0;  // records allocated / written
  unsigned dbg_trace_launch = 0;                 // launches traced so far

  // pinned host staging
  double* hpin = nullptr; size_t hpin_bytes = 0;

  // profiling
  bool prof = false;
  unsigned prof_mask = ~0u;  // kernel classes timed while prof is on
  std::vector<lfm::ProfEvent> pending;
  std::vector<hipEvent_t> pool;
  lfm_kstat stats[lfm::K_NCLASS];

  // farm (RCCL)
  void* comm = nullptr;
  bool comm_nb = false;  // communicator created non-blocking (calls polled, bounded)
  int nranks = 0, rank = -1;
  double* farm_buf = nullptr; size_t farm_bytes = 0;
  double* farm_h = nullptr; size_t farm_h_bytes = 0;  // pinned host staging of the all-gather
                                                      // (its own: a copy left queued by a timed-
                                                      // out call can only ever write here)
  double* farm_pub = nullptr; size_t farm_pub_bytes = 0;  // coherent pinned: the device-side
                                                          // round's gathered slots + seq word
  unsigned farm_seq = 0;    // device-side rounds published so far
  bool farm_stale = false;  // an aborted farm call may have left work queued (drained first)
  // the device-side round captured as one graph (LFM_FARM_GRAPH, default 1; read at creation),
  // replayed while its key (batch id, slots, sign, communicator generation) holds
  bool farm_graph_on = true;
  hipGraphExec_t farm_exec = nullptr;
  hipGraphExec_t farm_exec_old = nullptr;  // dropped by an aborted round: destroyed once drained
  uint64_t farm_exec_batch = 0, comm_gen = 0, farm_exec_gen = 0;
  int64_t farm_exec_slots = 0;
  int farm_exec_neg = -1;

  // C3's restart pipeline (lfm_mll_multi_f64): evaluation k runs on workspace
  // twin[k % 2], whose first launches (staging, gram, chain(0), X_0, chain(1), step 0) go to the
  // primary's overlap stream (CU-masked: the main CUs less LFM_OVL_RESERVE of them) once the
  // previous evaluation's tail has started, and whose later launches follow the previous
  // evaluation's in the primary's stream pair (m3 / s3, in stream order)
  lfm_ctx* twin[2] = {nullptr, nullptr};
  hipStream_t ovl_stream = nullptr;  // primary: the overlap stream
  bool borrowed = false;             // twin: stream (= the primary's ovl_stream), m3, s3 borrowed
  bool ovl = false;                  // twin: the factorisation in flight runs overlapped
  hipEvent_t ovl_tail = nullptr;     // twin: recorded on m3 ahead of its tail's first launch
  hipEvent_t ovl_done = nullptr;     // twin: recorded on m3 after its finalize
  hipEvent_t ovl_res = nullptr;      // twin: its result copied to the host (primary's stream)
  int ovl_on = 1;                    // LFM_OVERLAP: 0 evaluates lfm_mll_multi_f64's sets one by one
  int64_t ovl_at = 6144;             // LFM_OVL_AT: the tail starts at the first step whose
                                     // trailing matrix has fewer rows than this
  int ovl_reserve = 96;              // LFM_OVL_RESERVE: main CUs the overlap stream leaves to the
                                     // previous evaluation's tail
};

// ---------------------------------------------------------------- helpers
namespace lfm {

// Device status word (ctx->status[0], finalize copies it to result[3]): INT_MAX = every pivot
// positive; >= 0 = first non-positive / NaN pivot; STATUS_TIMEOUT = a bounded device-side
// wait ran out (it wins the atomicMin over any pivot index).
constexpr int STATUS_TIMEOUT = -2;
// LFM_OK, LFM_E_NOT_PD (pivot index in the message) or LFM_E_TIMEOUT for a status word.
int status_code(lfm_ctx* ctx, double st, double why = 0.0);

// The next factorisation on ctx runs schedule 3: the CU-partitioned pair exists and the call
// is not nested in a shared hold of the device's tenancy lock (lfm_api.hip DeviceTenancy).
inline bool s3_on(const lfm_ctx* ctx) {
  return ctx->sched == 3 && ctx->side_cus > 0 && !ctx->s3_yield;
}

int set_err(lfm_ctx* ctx, int code, const std::string& msg);
int hip_fail(lfm_ctx* ctx, hipError_t e, const char* what);
int ensure(lfm_ctx* ctx, void** p, size_t* cap, size_t bytes);
int ensure_pinned(lfm_ctx* ctx, size_t bytes);

// profiling hooks around a launch on ctx->stream
void prof_begin(lfm_ctx* ctx, int cls, hipEvent_t* a, hipStream_t st = nullptr);
// flops / bytes: algorithmic work of the launch; issued (< 0: = flops): what it issues
void prof_end(lfm_ctx* ctx, int cls, hipEvent_t a, double flops, double bytes,
              hipStream_t st = nullptr, double issued = -1.0);
int ensure_events(lfm_ctx* ctx, size_t count);
int prof_flush(lfm_ctx* ctx);

int chain_coresident(lfm_ctx* ctx, hipStream_t st, int G, bool* good);
int gene_clamp_host(double g, int64_t G);

// ------------------------------------------------------ launch wrappers
// Packed parameter block on the device (doubles):
//   [0,G) D   [G,2G) S   [2G,3G) B   then layout-specific arrays.
struct HypDev {
  const double* D;
  const double* S;
  const double* B;
  int G;
  double l;
};

// One problem of the fused small-N kernel: x / y in device memory; its hyperparameters as
// dsb = [true_d(G), true_s(G), true_b(G)] and sc = [l, obs_stddev, jitter], in device memory or
// in pinned host memory the kernel reads directly (lfm_batch: a resident batch uploads nothing
// per call). The kernel stages them in LDS first.
struct SmallProb {
  const double* x;
  const double* y;
  const double* dsb;
  const double* sc;
  int n, G;
  // grid layout (dataset_3d blocks on one uniform time grid; T = 0: none): the gram from the
  // per-gene tables of lfm_gram.hip (tables_doubles(G, T) doubles of LDS)
  int T = 0;
  double dt = 0.0;
  const double* times = nullptr;  // [T]
  const int* bg = nullptr;        // [n / T] gene of each block
};
// host: detect the grid layout of problem p and, when its tables fit the kernel's budget, put
// its times and block genes at hd (device address dd) and fill sp's grid fields; returns the
// doubles used (at most small_grid_doubles(n))
int64_t small_grid_pack(const double* x, int64_t n, int64_t G, SmallProb& sp, double* hd,
                        const double* dd);
inline int64_t small_grid_doubles(int64_t n) { return n + (n + 1) / 2; }
// largest per-problem grid table (doubles) in LDS: with n = 128 beside it the launch stays
// within a CU's 160 KB (launch_small_batch)
constexpr int SMALL_GRID_TAB_MAX = 2048;
constexpr int SMALL_MAX = 128;  // largest n handled by small_mll_kernel
constexpr int SMALL_GRAD_MAX = 127;  // largest n of the batched gradient / fit (two waves)

// gram kernels (lfm_gram.hip)
int launch_tables(lfm_ctx* ctx, const HypDev& h, const GridLayout& lay, const double* d_times,
                  double* tab);
// diagonal elements get (v + da1) + da2 — (K + jitter I) + sigma^2 I, objectives.py:71-72
template <typename OutT>
int launch_gram_grid(lfm_ctx* ctx, const HypDev& h, const GridLayout& lay, const double* tab,
                     const int* bg, int64_t n, double da1, double da2, int uplo, OutT* out,
                     int64_t ldo);
template <typename OutT>
int launch_gram_direct(lfm_ctx* ctx, const HypDev& h, const double* x, int64_t n,
                       const double* x2, int64_t m, double da1, double da2, int uplo, OutT* out,
                       int64_t ldo);
int launch_mean(lfm_ctx* ctx, const HypDev& h, const double* x, int64_t n, double* out);
int launch_h(lfm_ctx* ctx, const HypDev& h, const int64_t* j, const int64_t* k, const double* t1,
             const double* t2, int64_t n, double* out);
int launch_augment(lfm_ctx* ctx, const HypDev& h, const double* x, const double* y,
                   const double* loc, int64_t n, double* A, int64_t lda, int64_t Mp);

// The gram of an aligned grid layout (T % 256 == 0) fused into the factorisation's first
// trailing update (schedule 3): chol_factor_solve writes only the block columns the chains
// and the first panel solve read (launch_gram_region), and the first step's update units
// generate their Sigma tiles from the tables (gram_grid_aligned_kernel's arithmetic, bit-
// identical) instead of loading them. tab: tables_doubles layout; bg: block genes.
struct GramGen {
  const double* tab = nullptr;
  const int* bg = nullptr;
  int G = 0, Tn = 0;
  double da1 = 0.0, da2 = 0.0;
  int64_t n = 0;  // rows >= n (residual, padding) come from memory (augment_kernel)
};
int launch_gram_region(lfm_ctx* ctx, const GramGen& g, int64_t r0, int64_t r1, int64_t c0,
                       int64_t c1, double* out, int64_t ldo);

// cholesky kernels (lfm_chol.hip)
enum CholMode { CHOL_MLL = 0, CHOL_INVERSE = 1, CHOL_SCHUR = 2 };
// gen: the gram to fuse (lfm_api decides with chol_fuses_gram; the full gram is then NOT in A)
int chol_factor_solve(lfm_ctx* ctx, double* A, int64_t lda, int64_t n, int64_t Mp, int negative,
                      double* d_out, int mode = CHOL_MLL, const GramGen* gen = nullptr);
bool chol_fuses_gram(const lfm_ctx* ctx, int mode, const GridLayout& lay, int64_t n);
size_t tables_doubles(int G, int T);

// gradient kernels (lfm_grad.hip)
int launch_border_init(lfm_ctx* ctx, double* A, int64_t lda, int64_t Mp);
int posterior_blocked(lfm_ctx* ctx, const HypDev& h, const double* d_x, const double* d_y,
                      int64_t n, const double* d_dv, double diag_add, const double* d_t, int64_t m,
                      double* d_mean, double* d_cov);
int launch_grad(lfm_ctx* ctx, const HypDev& h, const double* d_x, int64_t n, const double* A,
                int64_t lda, int64_t Mp, double obs_stddev, int negative, double* acc,
                double* d_out, const GridLayout* lay = nullptr, const double* d_times = nullptr,
                const int* d_bg = nullptr);
// A resident batch small enough to travel in the kernel arguments (small_mll_kernel_args)
constexpr int SMALL_ARG_PROBS = 16, SMALL_ARG_HYP = 320;
struct SmallArgs {
  SmallProb probs[SMALL_ARG_PROBS];  // dsb / sc unused: the hyperparameters are below
  double hyp[SMALL_ARG_HYP];         // lfm_batch_mll_f64's packed layout
  int dsb_off[SMALL_ARG_PROBS], sc_off[SMALL_ARG_PROBS];
  double* out;
  int* status;
  int negative, tabs;
  double* grad;  // small_grad_kernel_args: the gradient, packed as hyp
};
static_assert(sizeof(SmallArgs) <= 4096, "kernel argument block");
// value and gradient of a batch of small problems (n <= SMALL_GRAD_MAX = 127; the launch's LDS
// map within 160 KB): a = the kernel-argument form
// (problem table and hyperparameters in the arguments) or NULL (d_probs, d_offs: the table and
// each problem's offsets of its vectors [0, nprob) and scalars [nprob, 2 nprob) in the packed
// layout, hyperparameters read through SmallProb::dsb / sc)
int launch_small_grad(lfm_ctx* ctx, SmallArgs* a, const SmallProb* d_probs, const int* d_offs,
                      int nprob, size_t lds, int negative, double* out, double* grad, int* status);
// LDS bytes of the gradient (fit = 0) or fit (fit = 1) launch over these problems (host table)
size_t small_grad_lds(const SmallProb* probs, int nprob, int fit);
// the fit kernel's launch: every problem's Adam steps on the device (lfm_small.hip FitArgs)
struct SmallFitLaunch {
  const SmallProb* probs;
  const int* offs;
  int nprob;
  double *raw, *mu, *nu, *history;
  const double* bias;
  int* status;
  double lr, b1, b2, eps, eps_root;
  int64_t step0, nsteps, spe;
  int fix, negative;
};
int launch_small_fit(lfm_ctx* ctx, const SmallFitLaunch& f, size_t lds);
int launch_small_args(lfm_ctx* ctx, SmallArgs& a, int nprob, int maxn, int maxg, int gridtab);
void small_batch_attrs();  // the MLL kernels' 160 KB LDS attribute (before launches / capture)
// gridtab: the largest small_grid_extra of the problems (doubles; 0: none on the grid path)
// LDS doubles a grid-layout problem adds to its map: the gram tables, the times, the block genes
size_t small_grid_extra(int n, int G, int T);
int launch_small_batch(lfm_ctx* ctx, const SmallProb* d_probs, int nprob, int maxn, int maxg,
                       int gridtab, int negative, double* d_out, int* d_status);

// Path of the advisory lock file behind schedule 3's cross-process tenancy (lfm_api.hip;
// empty if the device has no PCI bus id)
std::string tenancy_lock_path(int dev);

// Hook of the diagnostics library (liblfm_diag.so, lfm_diag.hip): one launch of the
// trailing-update kernel over a full triangle (lfm_chol.hip; launch only, no kernel of its own)
int probe_update_launch(lfm_ctx* ctx, hipStream_t st, int T, int kd, int cio, int64_t n,
                        size_t xb);

}  // namespace lfm
