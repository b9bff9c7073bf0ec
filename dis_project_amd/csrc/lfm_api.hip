// lfm_api.hip — the extern "C" boundary of include/lfm.h: context, workspace, input
// staging, x-layout detection, dispatch, profiling and the RCCL result farm.
//
// Every entry point binds the ctx's device, enqueues on the ctx's stream and is
// synchronous at return (one hipStreamSynchronize per call).
#include <dlfcn.h>
#include <fcntl.h>
#include <rccl/rccl.h>
#include <sys/file.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <ctime>
#include <memory>
#include <mutex>
#include <shared_mutex>

#include "lfm_internal.h"

using namespace lfm;

#ifndef LFM_GRAM_FUSE_DEFAULT
#define LFM_GRAM_FUSE_DEFAULT 1
#endif

namespace lfm {

const char* const kClassName[K_NCLASS] = {"tables",   "gram_grid", "gram_direct",
                                          "augment",  "potrf",     "trsm",
                                          "syrk",     "finalize",  "small_mll",
                                          "mean",     "grad",      "panel",
                                          "syrk_side", "small_grad"};

int set_err(lfm_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

int status_code(lfm_ctx* ctx, double st, double why) {
  const long long v = (long long)st;
  if (v == INT_MAX) return LFM_OK;
  if (v == STATUS_TIMEOUT) {
    static const char* const kind[] = {"unrecorded", "tall unit on the chain's factor",
                                       "tall unit on its ahead units", "early unit on its C tile",
                                       "early unit on its X rows", "chain input wait",
                                       "chain grid barrier", "fused panel wait"};
    const int k = why >= 0 && why < 8 ? (int)why : 0;
    return set_err(ctx, LFM_E_TIMEOUT,
                   std::string("device-side wait timed out (a cross-stream hand-off of the "
                               "factorisation stalled; first: ") + kind[k] +
                       "): the result is invalid, not a property of the input");
  }
  return set_err(ctx, LFM_E_NOT_PD,
                 "Cholesky failed: non-positive pivot at index " + std::to_string(v));
}

int hip_fail(lfm_ctx* ctx, hipError_t e, const char* what) {
  if (e == hipSuccess) return LFM_OK;
  const int code = (e == hipErrorOutOfMemory) ? LFM_E_OOM : LFM_E_HIP;
  return set_err(ctx, code, std::string(what) + ": " + hipGetErrorString(e));
}

int ensure(lfm_ctx* ctx, void** p, size_t* cap, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (*p && *cap >= bytes) return LFM_OK;
  if (*p) {
    hipError_t e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "sync before realloc");
    hipFree(*p);
    *p = nullptr;
    *cap = 0;
  }
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) {
    *p = nullptr;
    return set_err(ctx, LFM_E_OOM,
                   "hipMalloc(" + std::to_string(bytes) + " B): " + hipGetErrorString(e));
  }
  *cap = bytes;
  return LFM_OK;
}

int ensure_pinned(lfm_ctx* ctx, size_t bytes) {
  if (ctx->hpin && ctx->hpin_bytes >= bytes) return LFM_OK;
  if (ctx->hpin) {
    hipStreamSynchronize(ctx->stream);
    hipHostFree(ctx->hpin);
    ctx->hpin = nullptr;
  }
  hipError_t e = hipHostMalloc((void**)&ctx->hpin, bytes, hipHostMallocDefault);
  if (e != hipSuccess) return hip_fail(ctx, e, "hipHostMalloc");
  ctx->hpin_bytes = bytes;
  return LFM_OK;
}

// ----------------------------------------------------------- profiling
int ensure_events(lfm_ctx* ctx, size_t count) {
  while (ctx->evs.size() < count) {
    hipEvent_t e;
    hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming);
    if (r != hipSuccess) return hip_fail(ctx, r, "hipEventCreate");
    ctx->evs.push_back(e);
  }
  return LFM_OK;
}

void prof_begin(lfm_ctx* ctx, int cls, hipEvent_t* a, hipStream_t st) {
  *a = nullptr;
  if (!st) st = ctx->stream;
  if (!ctx->prof || !((ctx->prof_mask >> cls) & 1u)) return;
  if (ctx->pool.empty()) {
    hipEvent_t e;
    hipEventCreate(&e);
    ctx->pool.push_back(e);
  }
  *a = ctx->pool.back();
  ctx->pool.pop_back();
  hipEventRecord(*a, st);
}

void prof_end(lfm_ctx* ctx, int cls, hipEvent_t a, double flops, double bytes, hipStream_t st,
              double issued) {
  if (!ctx->prof || !a) return;
  if (!st) st = ctx->stream;
  if (ctx->pool.empty()) {
    hipEvent_t e;
    hipEventCreate(&e);
    ctx->pool.push_back(e);
  }
  hipEvent_t b = ctx->pool.back();
  ctx->pool.pop_back();
  hipEventRecord(b, st);
  ctx->pending.push_back(ProfEvent{cls, a, b, flops, bytes, issued < 0 ? flops : issued});
}

int prof_flush(lfm_ctx* ctx) {
  for (auto& p : ctx->pending) {
    float ms = 0;
    hipEventElapsedTime(&ms, p.a, p.b);
    lfm_kstat& s = ctx->stats[p.cls];
    s.launches += 1;
    s.total_ms += ms;
    s.flops += p.flops;
    s.bytes += p.bytes;
    s.issued_flops += p.issued;
    ctx->pool.push_back(p.a);
    ctx->pool.push_back(p.b);
  }
  ctx->pending.clear();
  return LFM_OK;
}

// -------------------------------------------------------- layout detect
int gene_clamp_host(double g, int64_t G) { return gene_index(g, (int)G); }

}  // namespace lfm

// ------------------------------------------------------------- staging
namespace {

struct Staged {
  HypDev h{};
  GridLayout lay;
  const double* d_times = nullptr;
  const int* d_bg = nullptr;
};

int check_hyp(lfm_ctx* ctx, const lfm_hyp* hyp) {
  if (!hyp) return set_err(ctx, LFM_E_ARG, "hyp is NULL");
  if (hyp->num_genes < 1 || hyp->num_genes > (1 << 20))
    return set_err(ctx, LFM_E_ARG, "num_genes must be in [1, 2^20]");
  if (!hyp->true_d || !hyp->true_s || !hyp->true_b)
    return set_err(ctx, LFM_E_ARG, "hyp true_d / true_s / true_b must not be NULL");
  return LFM_OK;
}

// Uploads D, S, B (and, for a grid layout, the time vector and block genes) into ctx->par.
int stage_hyp(lfm_ctx* ctx, const lfm_hyp* hyp, const double* x_host, int64_t n, bool want_grid,
              Staged* st, const GridLayout* known = nullptr) {
  int r = check_hyp(ctx, hyp);
  if (r) return r;
  const int64_t G = hyp->num_genes;
  if (known) st->lay = *known;
  else if (want_grid && x_host) st->lay = detect_grid(x_host, n, G);
  const int64_t T = st->lay.ok ? st->lay.T : 0;
  const int64_t nblk = st->lay.ok ? st->lay.nblk : 0;
  const size_t nd = (size_t)(3 * G + T);
  const size_t bytes = nd * 8 + (size_t)nblk * 4 + 16;
  r = ensure(ctx, (void**)&ctx->par, &ctx->par_bytes, bytes);
  if (r) return r;
  r = ensure_pinned(ctx, std::max<size_t>(bytes + 1024, 1 << 16));
  if (r) return r;
  // the previous call's copy out of hpin has completed (every call ends synchronised)
  double* hp = ctx->hpin;
  std::memcpy(hp, hyp->true_d, G * 8);
  std::memcpy(hp + G, hyp->true_s, G * 8);
  std::memcpy(hp + 2 * G, hyp->true_b, G * 8);
  if (T) std::memcpy(hp + 3 * G, st->lay.times.data(), T * 8);
  if (nblk) std::memcpy(reinterpret_cast<char*>(hp) + nd * 8, st->lay.block_gene.data(), nblk * 4);
  hipError_t e = hipMemcpyAsync(ctx->par, hp, bytes, hipMemcpyHostToDevice, ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "upload hyperparameters");
  st->h = HypDev{ctx->par, ctx->par + G, ctx->par + 2 * G, (int)G, hyp->l};
  st->d_times = ctx->par + 3 * G;
  st->d_bg = reinterpret_cast<const int*>(reinterpret_cast<const char*>(ctx->par) + nd * 8);
  return LFM_OK;
}

struct DeviceGuard {
  DeviceGuard(int dev) { hipSetDevice(dev); }
};

// ------------------------------------------------------ schedule-3 tenancy
// Schedule 3 is single tenant per GPU: its factor chain needs every one of its workgroups
// resident on the reserved CUs (one per CU, nearly all of the CU's LDS). Any other work on the
// GPU can starve it: two chains on the same CUs stall each other at their grid barriers, and a
// stream of smaller workgroups from another context (a schedule-1 factorisation, a gram fill)
// keeps refilling the LDS a waiting chain workgroup needs, while the resident ones spin until
// the bounded waits fire (LFM_E_TIMEOUT, minutes later: seen with two ranks of bench.py on one
// card at N = 16384). So the library holds a per-device readers-writer lock over its GPU work:
//   * exclusive: a schedule-3 factorisation (MLL, gradient, log_prob), from enqueue to the final
//     synchronise;
//   * shared: every other call that fills the GPU (schedule-1 factorisations, the posterior,
//     gram and cross-covariance fills). Shared holders run concurrently.
// In-process: a std::shared_mutex per device. Across processes: flock on
// $TMPDIR/lfm_gpu_<PCI bus id>.lock (LOCK_EX / LOCK_SH, the process's shared hold counted over
// its threads) behind a turnstile file (.turn, taken LOCK_EX for a moment by readers and held
// by a waiting writer), so a stream of readers cannot starve a schedule-3 call. Waits block:
// a call that finds the device busy runs when it is free, with its own schedule's arithmetic
// (the result is the same as running alone). The key is the PCI bus id, not the device ordinal,
// which depends on each process's HIP_VISIBLE_DEVICES. No lock is held while a call waits on
// anything but the GPU, so the order cannot deadlock; a nested request on a thread that already
// holds the device's lock is a no-op (a shared holder asking for exclusive runs schedule 1).
constexpr int kMaxDevices = 64;
TenancyLock g_dev[kMaxDevices];  // lfm_host.cpp: the readers-writer lock itself
std::mutex g_open_mu;
bool g_dev_opened[kMaxDevices] = {};
thread_local int t_depth[kMaxDevices] = {};
thread_local bool t_excl[kMaxDevices] = {};

// The device's lock files: $TMPDIR/lfm_gpu_<PCI bus id>.lock (and .turn), opened once
void device_lock_open(int dev) {
  std::lock_guard<std::mutex> lk(g_open_mu);
  if (g_dev_opened[dev]) return;
  g_dev_opened[dev] = true;
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), dev) != hipSuccess) {
    g_dev[dev].open("");  // in-process locking only
    return;
  }
  for (char* c = bus; *c; ++c)
    if (*c == ':' || *c == '.') *c = '_';
  const char* tmp = std::getenv("TMPDIR");
  g_dev[dev].open(std::string(tmp && *tmp ? tmp : "/tmp") + "/lfm_gpu_" + bus + ".lock");
}

}  // namespace

namespace lfm {
std::string tenancy_lock_path(int dev) {
  if (dev < 0 || dev >= kMaxDevices) return std::string();
  device_lock_open(dev);
  return g_dev[dev].path();
}
}  // namespace lfm

namespace {

class DeviceTenancy {
 public:
  // s3: the call would run schedule 3 (exclusive); else shared
  DeviceTenancy(lfm_ctx* ctx, bool s3) : ctx_(ctx) {
    ctx->s3_yield = false;
    const int dev = ctx->device;
    if (dev < 0 || dev >= kMaxDevices) return;
    if (t_depth[dev] > 0) {
      // nested on this thread: the held lock covers the call; a shared holder cannot upgrade
      if (s3 && !t_excl[dev]) ctx->s3_yield = true;
      ++t_depth[dev];
      dev_ = dev;
      nested_ = true;
      return;
    }
    device_lock_open(dev);
    dev_ = dev;
    excl_ = s3;
    if (excl_) g_dev[dev].lock_exclusive();
    else g_dev[dev].lock_shared();
    t_depth[dev] = 1;
    t_excl[dev] = excl_;
  }
  ~DeviceTenancy() {
    ctx_->s3_yield = false;
    if (dev_ < 0) return;
    if (nested_) {
      --t_depth[dev_];
      return;
    }
    t_depth[dev_] = 0;
    t_excl[dev_] = false;
    if (excl_) g_dev[dev_].unlock_exclusive();
    else g_dev[dev_].unlock_shared();
  }
  DeviceTenancy(const DeviceTenancy&) = delete;
  DeviceTenancy& operator=(const DeviceTenancy&) = delete;

 private:
  lfm_ctx* ctx_;
  int dev_ = -1;
  bool excl_ = false, nested_ = false;
};

int finish(lfm_ctx* ctx) {
  hipError_t e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "stream synchronize");
  // event pairs are read when the statistics are (lfm_profile_read / _reset), or in bulk past
  // 4096 pending: a profiled evaluation then spends no host time on ~130 event queries
  if (ctx->pending.size() > 4096) prof_flush(ctx);
  return LFM_OK;
}

int64_t round_up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }

// ------------------------------------------------------ schedule-3 stall fallback
// A schedule-3 factorisation whose device-side waits ran out (LFM_E_TIMEOUT after the time
// bound, lfm_chol.hip: another tenant of the GPU starved the chain's co-resident workgroups, or
// a tool serialised the two streams) is re-run once, inside the same call, on schedule 1 — the
// look-ahead on every CU, whose only device-side waits are between workgroups of one launch
// (dispatched in order, so each waits on work already running), under a 30 s bound. The caller
// gets the schedule-1 result (both schedules are held to the oracle at 1e-9 by the tests) and
// LFM_OK; the fallback is reported: lfm_ctx_fallbacks counts it and lfm_last_error names the
// stall. The reference never fails for scheduling reasons (trainer.py:126 just runs).
// LFM_S3_FALLBACK=0 turns it off (the tests of the timeout path itself).
constexpr unsigned kFallbackWaitTicks = 3000000000u;  // 30 s of the 100 MHz clock

template <class F>
int with_s3_fallback(lfm_ctx* ctx, F&& attempt) {
  const bool s3 = s3_on(ctx);
  int r = attempt();
  if (r != LFM_E_TIMEOUT || !s3 || !ctx->s3_fallback) return r;
  const std::string why = ctx->err;
  // the stalled call's waits have all ended (each within one bound, or at once after the first
  // timeout); drain both streams of the pair before the workspace is reused
  for (hipStream_t st : {ctx->m3, ctx->s3})
    if (st) hipStreamSynchronize(st);
  const unsigned ticks = ctx->wait_ticks;
  const bool had_side = ctx->side != nullptr;
  ctx->s3_yield = true;
  ctx->wait_ticks = std::max(ticks, kFallbackWaitTicks);
  r = attempt();
  ctx->wait_ticks = ticks;
  ctx->s3_yield = false;
  if (!had_side && ctx->side) {
    // schedule 1's high-priority stream was created for the re-run: give its hardware queue back
    // (an idle queue beside the partitioned pair slows the schedule-3 calls that follow, §5)
    hipStreamSynchronize(ctx->side);
    hipStreamDestroy(ctx->side);
    ctx->side = nullptr;
  }
  if (r == LFM_OK || r == LFM_E_NOT_PD) {
    ctx->fallbacks += 1;
    if (r == LFM_OK) ctx->err = "schedule 3 stalled (" + why + "); the call was re-run on schedule 1";
  }
  return r;
}

// Enqueue one MLL on ctx's streams: the lower triangle of ctx->A (lda = Mp) with Sigma = (K +
// jitter I) + sigma^2 I for x on the device (or generated inside the first update), the residual
// row n and identity padding; then the factorisation and the reduction into ctx->result.
int mll_enqueue(lfm_ctx* ctx, const Staged& st, const double* d_x, const double* d_y,
                const double* d_loc, int64_t n, const lfm_hyp* hyp, int negative) {
  const int64_t Mp = round_up(n + 1, 128);
  const double noise = hyp->obs_stddev * hyp->obs_stddev;  // objectives.py:66
  GramGen gen;
  const bool fuse = chol_fuses_gram(ctx, CHOL_MLL, st.lay, n);
  int r = LFM_OK;
  if (st.lay.ok) {
    r = ensure(ctx, (void**)&ctx->tab, &ctx->tab_bytes,
               tables_doubles(st.h.G, st.lay.T) * sizeof(double));
    if (r) return r;
    r = launch_tables(ctx, st.h, st.lay, st.d_times, ctx->tab);
    if (r) return r;
    // fused: the factorisation writes / generates Sigma itself (GramGen, lfm_chol.hip)
    if (fuse) gen = GramGen{ctx->tab, st.d_bg, st.h.G, st.lay.T, hyp->jitter, noise, n};
    else
      r = launch_gram_grid<double>(ctx, st.h, st.lay, ctx->tab, st.d_bg, n, hyp->jitter, noise,
                                   LFM_UPLO_LOWER, ctx->A, Mp);
  } else {
    r = launch_gram_direct<double>(ctx, st.h, d_x, n, d_x, n, hyp->jitter, noise,
                                   LFM_UPLO_LOWER, ctx->A, Mp);
  }
  if (r) return r;
  r = launch_augment(ctx, st.h, d_x, d_y, d_loc, n, ctx->A, Mp, Mp);
  if (r) return r;
  return chol_factor_solve(ctx, ctx->A, Mp, n, Mp, negative, ctx->result, CHOL_MLL,
                           fuse ? &gen : nullptr);
}

// mll_enqueue, then the result to the host (synchronous).
int mll_blocked(lfm_ctx* ctx, const Staged& st, const double* d_x, const double* d_y,
                const double* d_loc, int64_t n, const lfm_hyp* hyp, int negative, double* out) {
  const int64_t Mp = round_up(n + 1, 128);
  int r = ensure(ctx, (void**)&ctx->A, &ctx->A_bytes, (size_t)Mp * Mp * sizeof(double));
  if (r) return r;
  DeviceTenancy tenancy(ctx, s3_on(ctx));  // held to the final synchronise (finish)
  return with_s3_fallback(ctx, [&]() -> int {
    int r = mll_enqueue(ctx, st, d_x, d_y, d_loc, n, hyp, negative);
    if (r) return r;
    double* hres = ctx->hpin + (ctx->hpin_bytes / 8 - 8);
    hipMemcpyAsync(hres, ctx->result, 5 * sizeof(double), hipMemcpyDeviceToHost, ctx->stream);
    r = finish(ctx);
    if (r) return r;
    *out = hres[0];
    r = status_code(ctx, hres[3], hres[4]);
    if (r) *out = std::nan("");
    return r;
  });
}

int validate_x(lfm_ctx* ctx, const void* x, int64_t n) {
  if (!ctx) return LFM_E_ARG;
  if (!x) return set_err(ctx, LFM_E_ARG, "x is NULL");
  if (n < 1) return set_err(ctx, LFM_E_ARG, "n must be >= 1");
  if (n > (int64_t)1 << 30) return set_err(ctx, LFM_E_ARG, "n too large");
  return LFM_OK;
}

int check_mean_shape(lfm_ctx* ctx, int64_t n, const lfm_hyp* hyp) {
  // mean_function (model.py:145-149) repeats B/D in blocks of n // num_genes; the
  // reference's broadcast only succeeds when those blocks tile n exactly.
  if (n % hyp->num_genes != 0)
    return set_err(ctx, LFM_E_ARG,
                   "mean_function needs n divisible by num_genes (model.py:145-149)");
  return LFM_OK;
}

// small-N batch through one launch; probs already validated
}  // namespace

namespace lfm {
int64_t small_grid_pack(const double* x, int64_t n, int64_t G, SmallProb& sp, double* hd,
                        const double* dd) {
  sp.T = 0;
  const GridLayout lay = detect_grid(x, n, G);
  if (!lay.ok || tables_doubles((int)G, lay.T) > (size_t)SMALL_GRID_TAB_MAX) return 0;
  const int64_t T = lay.T, nblk = lay.nblk;
  std::memcpy(hd, lay.times.data(), T * 8);
  std::memcpy(hd + T, lay.block_gene.data(), nblk * sizeof(int));
  sp.T = (int)T;
  sp.dt = lay.dt;
  sp.times = dd;
  sp.bg = reinterpret_cast<const int*>(dd + T);
  return T + (nblk + 1) / 2;
}
}  // namespace lfm

namespace {

int small_batch(lfm_ctx* ctx, int64_t np, const lfm_problem* probs, const int64_t* idx,
                int negative, double* out, int* status) {
  // packed device buffer: per problem x(3n) y(n) D S B (3G) l obs_stddev jitter (3) doubles;
  // then the SmallProb array
  size_t nd = 0;
  int maxn = 1, maxg = 1;
  for (int64_t q = 0; q < np; ++q) {
    const lfm_problem& p = probs[idx[q]];
    nd += 4 * (size_t)p.n + 3 * (size_t)p.hyp.num_genes + 3 + small_grid_doubles(p.n);
    maxn = std::max<int>(maxn, (int)p.n);
    maxg = std::max<int>(maxg, (int)p.hyp.num_genes);
  }
  int gridtab = 0;
  const size_t bytes_d = nd * 8;
  const size_t bytes_p = (size_t)np * sizeof(SmallProb);
  const size_t bytes_o = (size_t)np * (8 + 4);
  const size_t total = round_up(bytes_d, 16) + round_up(bytes_p, 16) + bytes_o + 64;
  int r = ensure(ctx, (void**)&ctx->xin, &ctx->xin_bytes, total);
  if (r) return r;
  r = ensure_pinned(ctx, total + 4096);
  if (r) return r;
  char* hb = reinterpret_cast<char*>(ctx->hpin);
  char* db = reinterpret_cast<char*>(ctx->xin);
  double* hd = reinterpret_cast<double*>(hb);
  SmallProb* hp = reinterpret_cast<SmallProb*>(hb + round_up(bytes_d, 16));
  const double* dd = reinterpret_cast<const double*>(db);
  size_t off = 0;
  for (int64_t q = 0; q < np; ++q) {
    const lfm_problem& p = probs[idx[q]];
    const int64_t n = p.n, G = p.hyp.num_genes;
    SmallProb sp;
    std::memcpy(hd + off, p.x, 3 * n * 8);
    sp.x = dd + off;
    off += 3 * n;
    std::memcpy(hd + off, p.y, n * 8);
    sp.y = dd + off;
    off += n;
    sp.dsb = dd + off;
    std::memcpy(hd + off, p.hyp.true_d, G * 8);
    std::memcpy(hd + off + G, p.hyp.true_s, G * 8);
    std::memcpy(hd + off + 2 * G, p.hyp.true_b, G * 8);
    off += 3 * G;
    sp.sc = dd + off;
    hd[off] = p.hyp.l;
    hd[off + 1] = p.hyp.obs_stddev;
    hd[off + 2] = p.hyp.jitter;
    off += 3;
    sp.n = (int)n;
    sp.G = (int)G;
    off += small_grid_pack(p.x, n, G, sp, hd + off, dd + off);
    if (sp.T) gridtab = std::max<int>(gridtab, (int)small_grid_extra((int)n, (int)G, sp.T));
    hp[q] = sp;
  }
  const size_t up = round_up(bytes_d, 16) + bytes_p;
  hipError_t e = hipMemcpyAsync(db, hb, up, hipMemcpyHostToDevice, ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "upload small batch");
  double* d_out = reinterpret_cast<double*>(db + round_up(bytes_d, 16) + round_up(bytes_p, 16));
  int* d_st = reinterpret_cast<int*>(d_out + np);
  r = launch_small_batch(ctx, reinterpret_cast<const SmallProb*>(db + round_up(bytes_d, 16)),
                         (int)np, maxn, maxg, gridtab, negative, d_out, d_st);
  if (r) return r;
  double* h_out = reinterpret_cast<double*>(hb + round_up(bytes_d, 16) + round_up(bytes_p, 16));
  e = hipMemcpyAsync(h_out, d_out, np * 12, hipMemcpyDeviceToHost, ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "download small batch");
  r = finish(ctx);
  if (r) return r;
  const int* h_st = reinterpret_cast<const int*>(h_out + np);
  for (int64_t q = 0; q < np; ++q) {
    out[idx[q]] = h_out[q];
    if (status) status[idx[q]] = h_st[q] ? LFM_E_NOT_PD : LFM_OK;
  }
  return LFM_OK;
}

}  // namespace

template <typename OutT>
static int gram_impl(lfm_ctx* ctx, const double* x_host, const double* d_x, int64_t n,
                     const lfm_hyp* hyp, double diag_add, int uplo, OutT* d_out, int64_t ldo) {
  Staged st;
  int r = stage_hyp(ctx, hyp, x_host, n, true, &st);
  if (r) return r;
  if (st.lay.ok) {
    r = ensure(ctx, (void**)&ctx->tab, &ctx->tab_bytes,
               tables_doubles(st.h.G, st.lay.T) * sizeof(double));
    if (r) return r;
    r = launch_tables(ctx, st.h, st.lay, st.d_times, ctx->tab);
    if (r) return r;
    return launch_gram_grid<OutT>(ctx, st.h, st.lay, ctx->tab, st.d_bg, n, diag_add, 0.0, uplo,
                                  d_out, ldo);
  }
  return launch_gram_direct<OutT>(ctx, st.h, d_x, n, d_x, n, diag_add, 0.0, uplo, d_out, ldo);
}

template <typename OutT>
static int gram_host(lfm_ctx* ctx, const double* x, int64_t n, const lfm_hyp* hyp,
                     double diag_add, int uplo, OutT* out, int64_t ldo) {
  int r = validate_x(ctx, x, n);
  if (r) return r;
  if (!out || ldo < n) return set_err(ctx, LFM_E_ARG, "out is NULL or ldo < n");
  if (uplo != LFM_UPLO_FULL && uplo != LFM_UPLO_LOWER) return set_err(ctx, LFM_E_ARG, "bad uplo");
  DeviceGuard g(ctx->device);
  DeviceTenancy tenancy(ctx, false);
  r = ensure(ctx, (void**)&ctx->xin, &ctx->xin_bytes, (size_t)n * 3 * 8);
  if (r) return r;
  r = ensure(ctx, (void**)&ctx->A, &ctx->A_bytes, (size_t)n * n * sizeof(OutT));
  if (r) return r;
  OutT* dA = reinterpret_cast<OutT*>(ctx->A);
  hipMemcpyAsync(ctx->xin, x, n * 3 * 8, hipMemcpyHostToDevice, ctx->stream);
  if (uplo == LFM_UPLO_LOWER) hipMemsetAsync(dA, 0, (size_t)n * n * sizeof(OutT), ctx->stream);
  r = gram_impl<OutT>(ctx, x, ctx->xin, n, hyp, diag_add, uplo, dA, n);
  if (r) return r;
  hipError_t e = hipMemcpy2DAsync(out, ldo * sizeof(OutT), dA, n * sizeof(OutT),
                                  n * sizeof(OutT), n, hipMemcpyDeviceToHost, ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "download gram");
  return finish(ctx);
}

template <typename OutT>
static int gram_dev(lfm_ctx* ctx, const double* d_x, int64_t n, const lfm_hyp* hyp,
                    double diag_add, int uplo, OutT* d_out, int64_t ldo) {
  int r = validate_x(ctx, d_x, n);
  if (r) return r;
  if (!d_out || ldo < n) return set_err(ctx, LFM_E_ARG, "out is NULL or ldo < n");
  if (uplo != LFM_UPLO_FULL && uplo != LFM_UPLO_LOWER) return set_err(ctx, LFM_E_ARG, "bad uplo");
  DeviceGuard g(ctx->device);
  DeviceTenancy tenancy(ctx, false);
  std::vector<double> xh((size_t)n * 3);
  hipError_t e = hipMemcpyAsync(xh.data(), d_x, n * 3 * 8, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "read back x for layout detection");
  r = gram_impl<OutT>(ctx, xh.data(), d_x, n, hyp, diag_add, uplo, d_out, ldo);
  if (r) return r;
  return finish(ctx);
}

namespace {
int env_int_api(const char* name, int def) {
  const char* v = std::getenv(name);
  return v ? std::atoi(v) : def;
}
// Schedule 3's stream pair: CU mask bits [0, cus) for the factor chain (consecutive bits,
// which the hardware spreads over the XCDs: bit c lives on XCD c % 8), every other CU for the
// main (bulk) stream. The chain kernel needs all of its workgroups (one per CU) resident at
// once: checked here, halving the reservation until it holds. Each CU-masked stream holds a
// hardware queue of its own for the context's lifetime, idle or not.
hipError_t create_partition(lfm_ctx* ctx, int side_cus) {
  const int ncu = ctx->cus;
  if (ctx->m3 || side_cus <= 0 || side_cus >= ncu) return hipSuccess;
  for (int cus = side_cus; cus >= 4; cus /= 2) {
    // every XCD keeps the same number of main CUs, or the partition is refused (measured:
    // an XCD left without main CUs never ran the main launch's workgroups dealt to it)
    std::vector<int> per_xcd(8, 0);
    for (int c = cus; c < ncu; ++c) per_xcd[c % 8] += 1;
    if (*std::min_element(per_xcd.begin(), per_xcd.end()) !=
        *std::max_element(per_xcd.begin(), per_xcd.end()))
      continue;
    std::vector<uint32_t> mside((ncu + 31) / 32, 0u), mmain((ncu + 31) / 32, 0u);
    for (int c = 0; c < ncu; ++c) (c < cus ? mside : mmain)[c / 32] |= 1u << (c % 32);
    hipError_t e = hipExtStreamCreateWithCUMask(&ctx->m3, (uint32_t)mmain.size(), mmain.data());
    if (e == hipSuccess)
      e = hipExtStreamCreateWithCUMask(&ctx->s3, (uint32_t)mside.size(), mside.data());
    if (e != hipSuccess) return e;
    bool good = false;
    if (lfm::chain_coresident(ctx, ctx->s3, cus, &good) != LFM_OK) return hipErrorUnknown;
    if (good) {
      ctx->side_cus = cus;
      return hipSuccess;
    }
    hipStreamDestroy(ctx->m3);
    hipStreamDestroy(ctx->s3);
    ctx->m3 = ctx->s3 = nullptr;
  }
  ctx->side_cus = 0;  // no usable partition: schedule 1
  return hipSuccess;
}

// Give the pair's hardware queues back (schedule 1 never uses them). Measured on C3: idle
// CU-masked queues of other contexts in the process oversubscribe the hardware scheduler —
// one schedule-1 evaluation at a time ran 23.3 evals/s beside three idle partitioned contexts
// against 29.1 alone.
void twins_drop(lfm_ctx* ctx);
void release_partition(lfm_ctx* ctx) {
  twins_drop(ctx);  // they borrow the pair
  for (hipStream_t* st : {&ctx->s3, &ctx->m3})
    if (*st) {
      hipStreamSynchronize(*st);
      hipStreamDestroy(*st);
      *st = nullptr;
    }
  ctx->side_cus = 0;
}

// Main stream (every CU), and for schedule 3 the CU-partitioned pair:
// LFM_SIDE_CUS (default 32) CUs for the factor chain, the rest for the bulk
// (hipExtStreamCreateWithCUMask). The documented knobs read here:
//   LFM_SCHED            3 (default) or 1: the look-ahead schedule of the MLL factorisation
//                        (1: no CU partition is created; lfm_ctx_set_schedule changes it later)
//   LFM_SIDE_CUS         CUs reserved for the schedule-3 factor chain (0: schedule 1 only)
//   LFM_S3_EVENTS        1: schedule 3 ordered by stream events, tall units in launches of
//                        their own (for rocprofv3 --pmc); 2: the timed schedule's own launches,
//                        serialised by events so each one's device-side waits are met at dispatch
//   LFM_DEVICE_WAIT_MS   time bound of every device-side wait (default 2000 ms; lfm_chol.hip)
//   LFM_DEBUG_SPIN_LIMIT the same bound in raw 100 MHz ticks (tests force timeouts with 0)
//   LFM_GRAD_DIRECT      1: the gradient's per-pair path even on a grid layout (cross-check)
//   LFM_GRAM_FUSE        0: the full gram in its own kernel even where the first update could
//                        generate it (cross-check: the MLL is bit-identical either way)
//   LFM_W4_MIN / LFM_W2_MIN / LFM_W0   the step plan (lfm_chol.hip chol_factor_solve)
//   LFM_HELPER / LFM_HELPER_TC / LFM_HELPER_MIN   schedule 3's side-CU helper and its sizing
//   LFM_S3_FALLBACK      0: a stalled schedule-3 call returns LFM_E_TIMEOUT (no schedule-1 re-run)
//   LFM_RCCL_TIMEOUT_S   bound on every wait of the farm communicator (default 300 s)
//   LFM_DEBUG_FARM_STALL_MS  test stand-in for a late peer ahead of each all-gather
//   LFM_SMALL_KERNARG    0: resident batches read their problem table / hyperparameters from
//                        memory instead of the kernel arguments
//   LFM_FARM_GRAPH       0: a device-side farm round is enqueued call by call instead of
//                        replayed as one captured graph
//   LFM_OVERLAP / LFM_OVL_AT / LFM_OVL_RESERVE   lfm_mll_multi_f64's restart pipeline: on/off,
//                        the trailing rows below which an evaluation's tail starts (the next one's
//                        prologue may run), main CUs the overlap stream leaves to that tail
// Every knob is read here, once: a call never consults the environment.
hipError_t create_streams(lfm_ctx* ctx) {
  ctx->sched = env_int_api("LFM_SCHED", 3) == 1 ? 1 : 3;
  ctx->s3_events = (int)env_int_api("LFM_S3_EVENTS", 0);
  ctx->grad_direct = env_int_api("LFM_GRAD_DIRECT", 0) != 0;
  ctx->gram_fuse = env_int_api("LFM_GRAM_FUSE", LFM_GRAM_FUSE_DEFAULT) != 0;
  ctx->w4min = env_int_api("LFM_W4_MIN", 6144);
  ctx->w2min = env_int_api("LFM_W2_MIN", -1);
  ctx->w0 = std::max(1, env_int_api("LFM_W0", 1));
  ctx->helper = env_int_api("LFM_HELPER", 1);
  ctx->helper_tc = env_int_api("LFM_HELPER_TC", 700);
  ctx->helper_min = env_int_api("LFM_HELPER_MIN", 1200);
  ctx->s3_fallback = env_int_api("LFM_S3_FALLBACK", 1) != 0;
  if (const char* v = std::getenv("LFM_RCCL_TIMEOUT_S")) {
    const double t = std::atof(v);
    if (t > 0.0) ctx->rccl_timeout_s = t;
  }
  ctx->farm_stall_ms = std::max(0, env_int_api("LFM_DEBUG_FARM_STALL_MS", 0));
  ctx->small_kernarg = env_int_api("LFM_SMALL_KERNARG", 1) != 0;
  ctx->farm_graph_on = env_int_api("LFM_FARM_GRAPH", 1) != 0;
  if (const char* ms = std::getenv("LFM_DEVICE_WAIT_MS")) {
    // 100 MHz ticks; at most ~42 s (the bound is a 32-bit tick count)
    const double t = std::min(std::max(std::atof(ms), 0.0), 42000.0);
    ctx->wait_ticks = (unsigned)(t * 1e5);
  }
  if (const char* sl = std::getenv("LFM_DEBUG_SPIN_LIMIT"))
    ctx->wait_ticks = (unsigned)std::strtoul(sl, nullptr, 10);
  ctx->side_req = env_int_api("LFM_SIDE_CUS", 32);
  ctx->ovl_on = env_int_api("LFM_OVERLAP", 1);
  ctx->ovl_at = env_int_api("LFM_OVL_AT", 6144);
  ctx->ovl_reserve = std::max(0, env_int_api("LFM_OVL_RESERVE", 96));
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, ctx->device);
  if (prop.multiProcessorCount > 0) ctx->cus = prop.multiProcessorCount;
  // ctx->side (schedule 1's high-priority stream) is created on first use: schedule 3 never
  // launches on it, and an idle hardware queue beside the running ones costs
  hipError_t e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
  if (e != hipSuccess || ctx->sched != 3) return e;
  return create_partition(ctx, ctx->side_req);
}
}  // namespace

// =================================================================== C ABI
extern "C" {

int lfm_abi_version(void) { return LFM_ABI_VERSION; }

int lfm_device_count(int* out) {
  if (!out) return LFM_E_ARG;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) n = 0;
  *out = n;
  return e == hipSuccess ? LFM_OK : LFM_E_HIP;
}

int lfm_ctx_create(int device, lfm_ctx** out) {
  if (!out) return LFM_E_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return LFM_E_HIP;
  if (device < 0 || device >= ndev) return LFM_E_ARG;
  lfm_ctx* ctx = new lfm_ctx();
  ctx->device = device;
  std::memset(ctx->stats, 0, sizeof(ctx->stats));
  for (int i = 0; i < K_NCLASS; ++i)
    std::snprintf(ctx->stats[i].name, sizeof(ctx->stats[i].name), "%s", kClassName[i]);
  hipSetDevice(device);
  hipError_t e = create_streams(ctx);
  if (e == hipSuccess) e = hipMalloc((void**)&ctx->linvT, 128 * 128 * sizeof(double));
  if (e == hipSuccess) e = hipMalloc((void**)&ctx->status, 64);
  if (e == hipSuccess) e = hipMalloc((void**)&ctx->result, 64 * sizeof(double));
  if (e == hipSuccess) e = hipMalloc((void**)&ctx->psync, 64);
  // Deliberately on the null stream, after the context's streams: the hardware queues of a
  // process are opened in this order (stream, CU-masked pair, null stream), and the order
  // matters for one C2 evaluation (scripts/ab_lib.py, 5 interleaved rounds each): without the
  // null-stream queue 30.71 ms against 30.35; null queue first 30.29 and CU-masked pair
  // first 30.31 against 29.97 on another box. DESIGN.md §9.
  if (e == hipSuccess) e = hipMemset(ctx->psync, 0, 64);
  if (e != hipSuccess) {
    lfm_ctx_destroy(ctx);
    return LFM_E_HIP;
  }
  *out = ctx;
  return LFM_OK;
}

void lfm_ctx_destroy(lfm_ctx* ctx) {
  if (!ctx) return;
  hipSetDevice(ctx->device);
  twins_drop(ctx);
  if (ctx->borrowed) {
    // a restart-pipeline workspace: its streams are its primary's (drained by twins_drop)
    ctx->stream = ctx->m3 = ctx->s3 = nullptr;
    for (hipEvent_t e : {ctx->ovl_tail, ctx->ovl_done, ctx->ovl_res})
      if (e) hipEventDestroy(e);
  }
  if (ctx->stream) hipStreamSynchronize(ctx->stream);
  lfm_farm_destroy(ctx);
  for (void* p : {(void*)ctx->A, (void*)ctx->tab, (void*)ctx->tab32, (void*)ctx->par,
                  (void*)ctx->xin, (void*)ctx->linvT, (void*)ctx->parts, (void*)ctx->status,
                  (void*)ctx->result, (void*)ctx->farm_buf, (void*)ctx->gacc,
                  (void*)ctx->psync, (void*)ctx->wk, (void*)ctx->xbuf, (void*)ctx->zvec,
                  (void*)ctx->flags, (void*)ctx->linv_full, (void*)ctx->dbg_stamps, (void*)ctx->xd,
                  (void*)ctx->gtab})
    if (p) hipFree(p);
  if (ctx->hpin) hipHostFree(ctx->hpin);
  if (ctx->farm_h) hipHostFree(ctx->farm_h);
  if (ctx->farm_pub) hipHostFree(ctx->farm_pub);
  for (auto& p : ctx->pending) {
    hipEventDestroy(p.a);
    hipEventDestroy(p.b);
  }
  for (auto e : ctx->pool) hipEventDestroy(e);
  for (auto e : ctx->evs) hipEventDestroy(e);
  for (hipStream_t* st : {&ctx->side, &ctx->s3, &ctx->m3})
    if (*st) {
      hipStreamSynchronize(*st);
      hipStreamDestroy(*st);
    }
  if (ctx->stream) hipStreamDestroy(ctx->stream);
  delete ctx;
}

const char* lfm_last_error(const lfm_ctx* ctx) { return ctx ? ctx->err.c_str() : "null ctx"; }

int lfm_ctx_synchronize(lfm_ctx* ctx) {
  if (!ctx) return LFM_E_ARG;
  DeviceGuard g(ctx->device);
  return finish(ctx);
}

int lfm_ctx_set_block(lfm_ctx* ctx, int nb) {
  if (!ctx) return LFM_E_ARG;
  if (nb != 0 && nb != 128) return set_err(ctx, LFM_E_ARG, "block size must be 128 (or 0)");
  ctx->nb = 128;
  return LFM_OK;
}

int lfm_ctx_set_schedule(lfm_ctx* ctx, int schedule) {
  if (!ctx) return LFM_E_ARG;
  if (schedule == 0) schedule = env_int_api("LFM_SCHED", 3) == 1 ? 1 : 3;
  if (schedule != 1 && schedule != 3)
    return set_err(ctx, LFM_E_ARG, "schedule must be 1, 3 (or 0: the LFM_SCHED default)");
  DeviceGuard g(ctx->device);
  if (hipStreamSynchronize(ctx->stream) != hipSuccess)
    return set_err(ctx, LFM_E_HIP, "lfm_ctx_set_schedule: stream synchronize failed");
  if (schedule == 1) {
    release_partition(ctx);
  } else {
    if (create_partition(ctx, ctx->side_req) != hipSuccess)
      return set_err(ctx, LFM_E_HIP, "lfm_ctx_set_schedule: CU-masked stream creation failed");
    if (ctx->side_cus <= 0)
      return set_err(ctx, LFM_E_ARG, "schedule 3 needs the CU-partitioned stream pair, which "
                                     "this device / LFM_SIDE_CUS did not provide");
  }
  ctx->sched = schedule;
  return LFM_OK;
}

int lfm_ctx_fallbacks(const lfm_ctx* ctx, int64_t* out) {
  if (!ctx || !out) return LFM_E_ARG;
  *out = ctx->fallbacks;
  return LFM_OK;
}

int lfm_ctx_get_schedule(const lfm_ctx* ctx, int* out) {
  if (!ctx || !out) return LFM_E_ARG;
  *out = ctx->sched == 3 && ctx->side_cus > 0 ? 3 : 1;
  return LFM_OK;
}

int lfm_mean_function_f64(lfm_ctx* ctx, const double* x, int64_t n, const lfm_hyp* hyp,
                          double* out) {
  int r = validate_x(ctx, x, n);
  if (r) return r;
  if (!out) return set_err(ctx, LFM_E_ARG, "out is NULL");
  DeviceGuard g(ctx->device);
  Staged st;
  r = stage_hyp(ctx, hyp, x, n, false, &st);
  if (r) return r;
  r = check_mean_shape(ctx, n, hyp);
  if (r) return r;
  r = ensure(ctx, (void**)&ctx->xin, &ctx->xin_bytes, (size_t)n * 4 * 8);
  if (r) return r;
  hipMemcpyAsync(ctx->xin, x, n * 3 * 8, hipMemcpyHostToDevice, ctx->stream);
  r = launch_mean(ctx, st.h, ctx->xin, n, ctx->xin + 3 * n);
  if (r) return r;
  hipMemcpyAsync(out, ctx->xin + 3 * n, n * 8, hipMemcpyDeviceToHost, ctx->stream);
  return finish(ctx);
}

int lfm_h_f64(lfm_ctx* ctx, const lfm_hyp* hyp, const int64_t* j, const int64_t* k,
              const double* t1, const double* t2, int64_t n, double* out) {
  if (!ctx) return LFM_E_ARG;
  if (!j || !k || !t1 || !t2 || !out || n < 1) return set_err(ctx, LFM_E_ARG, "bad h arguments");
  DeviceGuard g(ctx->device);
  Staged st;
  int r = stage_hyp(ctx, hyp, nullptr, 0, false, &st);
  if (r) return r;
  r = ensure(ctx, (void**)&ctx->xin, &ctx->xin_bytes, (size_t)n * 5 * 8);
  if (r) return r;
  int64_t* dj = reinterpret_cast<int64_t*>(ctx->xin);
  int64_t* dk = dj + n;
  double* dt1 = ctx->xin + 2 * n;
  double* dt2 = ctx->xin + 3 * n;
  double* dout = ctx->xin + 4 * n;
  hipMemcpyAsync(dj, j, n * 8, hipMemcpyHostToDevice, ctx->stream);
  hipMemcpyAsync(dk, k, n * 8, hipMemcpyHostToDevice, ctx->stream);
  hipMemcpyAsync(dt1, t1, n * 8, hipMemcpyHostToDevice, ctx->stream);
  hipMemcpyAsync(dt2, t2, n * 8, hipMemcpyHostToDevice, ctx->stream);
  r = launch_h(ctx, st.h, dj, dk, dt1, dt2, n, dout);
  if (r) return r;
  hipMemcpyAsync(out, dout, n * 8, hipMemcpyDeviceToHost, ctx->stream);
  return finish(ctx);
}

int lfm_cross_covariance_f64(lfm_ctx* ctx, const double* x, int64_t n, const double* x2,
                             int64_t m, const lfm_hyp* hyp, double* out, int64_t ldo) {
  int r = validate_x(ctx, x, n);
  if (r) return r;
  r = validate_x(ctx, x2, m);
  if (r) return r;
  if (!out || ldo < m) return set_err(ctx, LFM_E_ARG, "out is NULL or ldo < m");
  DeviceGuard g(ctx->device);
  DeviceTenancy tenancy(ctx, false);
  Staged st;
  r = stage_hyp(ctx, hyp, nullptr, 0, false, &st);
  if (r) return r;
  r = ensure(ctx, (void**)&ctx->xin, &ctx->xin_bytes, (size_t)(n + m) * 3 * 8);
  if (r) return r;
  r = ensure(ctx, (void**)&ctx->A, &ctx->A_bytes, (size_t)n * m * 8);
  if (r) return r;
  hipMemcpyAsync(ctx->xin, x, n * 3 * 8, hipMemcpyHostToDevice, ctx->stream);
  hipMemcpyAsync(ctx->xin + 3 * n, x2, m * 3 * 8, hipMemcpyHostToDevice, ctx->stream);
  r = launch_gram_direct<double>(ctx, st.h, ctx->xin, n, ctx->xin + 3 * n, m, 0.0, 0.0,
                                 LFM_UPLO_FULL, ctx->A, m);
  if (r) return r;
  hipError_t e = hipMemcpy2DAsync(out, ldo * 8, ctx->A, m * 8, m * 8, n, hipMemcpyDeviceToHost,
                                  ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "download cross-covariance");
  return finish(ctx);
}



int lfm_gram_f64(lfm_ctx* ctx, const double* x, int64_t n, const lfm_hyp* hyp, double diag_add,
                 int uplo, double* out, int64_t ldo) {
  return gram_host<double>(ctx, x, n, hyp, diag_add, uplo, out, ldo);
}

int lfm_gram_f32(lfm_ctx* ctx, const double* x, int64_t n, const lfm_hyp* hyp, double diag_add,
                 int uplo, float* out, int64_t ldo) {
  return gram_host<float>(ctx, x, n, hyp, diag_add, uplo, out, ldo);
}


int lfm_gram_f64_dev(lfm_ctx* ctx, const double* d_x, int64_t n, const lfm_hyp* hyp,
                     double diag_add, int uplo, double* d_out, int64_t ldo) {
  return gram_dev<double>(ctx, d_x, n, hyp, diag_add, uplo, d_out, ldo);
}

int lfm_gram_f32_dev(lfm_ctx* ctx, const double* d_x, int64_t n, const lfm_hyp* hyp,
                     double diag_add, int uplo, float* d_out, int64_t ldo) {
  return gram_dev<float>(ctx, d_x, n, hyp, diag_add, uplo, d_out, ldo);
}

int lfm_mll_f64(lfm_ctx* ctx, const double* x, const double* y, int64_t n, const lfm_hyp* hyp,
                int negative, double* out) {
  int r = validate_x(ctx, x, n);
  if (r) return r;
  if (!y || !out) return set_err(ctx, LFM_E_ARG, "y / out is NULL");
  r = check_hyp(ctx, hyp);
  if (r) return r;
  r = check_mean_shape(ctx, n, hyp);
  if (r) return r;
  DeviceGuard g(ctx->device);
  if (n <= SMALL_MAX) {
    lfm_problem p{x, y, n, *hyp};
    int64_t idx = 0;
    int st = 0;
    r = small_batch(ctx, 1, &p, &idx, negative, out, &st);
    if (r) return r;
    if (st) return set_err(ctx, LFM_E_NOT_PD, "Cholesky failed: non-positive pivot");
    return LFM_OK;
  }
  Staged st;
  r = stage_hyp(ctx, hyp, x, n, true, &st);
  if (r) return r;
  r = ensure(ctx, (void**)&ctx->xin, &ctx->xin_bytes, (size_t)n * 4 * 8);
  if (r) return r;
  hipMemcpyAsync(ctx->xin, x, n * 3 * 8, hipMemcpyHostToDevice, ctx->stream);
  hipMemcpyAsync(ctx->xin + 3 * n, y, n * 8, hipMemcpyHostToDevice, ctx->stream);
  return mll_blocked(ctx, st, ctx->xin, ctx->xin + 3 * n, nullptr, n, hyp, negative, out);
}

int lfm_mll_grad_f64(lfm_ctx* ctx, const double* x, const double* y, int64_t n,
                     const lfm_hyp* hyp, int negative, double* value, double* grad) {
  int r = validate_x(ctx, x, n);
  if (r) return r;
  if (!y || !value || !grad) return set_err(ctx, LFM_E_ARG, "y / value / grad is NULL");
  r = check_hyp(ctx, hyp);
  if (r) return r;
  r = check_mean_shape(ctx, n, hyp);
  if (r) return r;
  DeviceGuard g(ctx->device);
  Staged st;
  r = stage_hyp(ctx, hyp, x, n, true, &st);
  if (r) return r;
  r = ensure(ctx, (void**)&ctx->xin, &ctx->xin_bytes, (size_t)n * 4 * 8);
  if (r) return r;
  const double* d_x = ctx->xin;
  const double* d_y = ctx->xin + 3 * n;
  hipMemcpyAsync(ctx->xin, x, n * 3 * 8, hipMemcpyHostToDevice, ctx->stream);
  hipMemcpyAsync(ctx->xin + 3 * n, y, n * 8, hipMemcpyHostToDevice, ctx->stream);
  // bordered 2Mp x 2Mp matrix [[S_aug, .], [I, 0]] (lfm_grad.hip)
  const int64_t Mp = round_up(n + 1, 128), M2 = 2 * Mp;
  r = ensure(ctx, (void**)&ctx->A, &ctx->A_bytes, (size_t)M2 * M2 * sizeof(double));
  if (r) return r;
  const int64_t G = hyp->num_genes;
  r = ensure(ctx, (void**)&ctx->gacc, &ctx->gacc_bytes, (size_t)(5 * G + 3) * sizeof(double));
  if (r) return r;
  const double noise = hyp->obs_stddev * hyp->obs_stddev;  // objectives.py:66
  DeviceTenancy tenancy(ctx, s3_on(ctx));  // held to the final synchronise (finish)
  return with_s3_fallback(ctx, [&]() -> int {
    int r = LFM_OK;
    GramGen gen;
    const bool fuse = chol_fuses_gram(ctx, CHOL_INVERSE, st.lay, n);
    if (st.lay.ok) {
      r = ensure(ctx, (void**)&ctx->tab, &ctx->tab_bytes,
                 tables_doubles(st.h.G, st.lay.T) * sizeof(double));
      if (r) return r;
      r = launch_tables(ctx, st.h, st.lay, st.d_times, ctx->tab);
      if (r) return r;
      if (fuse) gen = GramGen{ctx->tab, st.d_bg, st.h.G, st.lay.T, hyp->jitter, noise, n};
      else
        r = launch_gram_grid<double>(ctx, st.h, st.lay, ctx->tab, st.d_bg, n, hyp->jitter, noise,
                                     LFM_UPLO_LOWER, ctx->A, M2);
    } else {
      r = launch_gram_direct<double>(ctx, st.h, d_x, n, d_x, n, hyp->jitter, noise,
                                     LFM_UPLO_LOWER, ctx->A, M2);
    }
    if (r) return r;
    r = launch_augment(ctx, st.h, d_x, d_y, nullptr, n, ctx->A, M2, Mp);
    if (r) return r;
    r = chol_factor_solve(ctx, ctx->A, M2, n, Mp, negative, ctx->result, CHOL_INVERSE,
                          fuse ? &gen : nullptr);
    if (r) return r;
    double* d_out = ctx->gacc + 2 * G + 1;
    r = launch_grad(ctx, st.h, d_x, n, ctx->A, M2, Mp, hyp->obs_stddev, negative, ctx->gacc, d_out,
                    &st.lay, st.d_times, st.d_bg);
    if (r) return r;
    const size_t ng = (size_t)(3 * G + 2);
    r = ensure_pinned(ctx, (ng + 16) * sizeof(double));
    if (r) return r;
    double* hres = ctx->hpin;
    hipMemcpyAsync(hres, ctx->result, 5 * sizeof(double), hipMemcpyDeviceToHost, ctx->stream);
    hipMemcpyAsync(hres + 8, d_out, ng * sizeof(double), hipMemcpyDeviceToHost, ctx->stream);
    r = finish(ctx);
    if (r) return r;
    *value = hres[0];
    std::memcpy(grad, hres + 8, ng * sizeof(double));
    r = status_code(ctx, hres[3], hres[4]);
    if (r) {
      *value = std::nan("");
      for (size_t i = 0; i < ng; ++i) grad[i] = std::nan("");
    }
    return r;
  });
}

int lfm_posterior_f64(lfm_ctx* ctx, const double* x, const double* y, int64_t n,
                      const double* diag_vec, double diag_add, const double* t, int64_t m,
                      const lfm_hyp* hyp, double* mean, double* cov) {
  int r = validate_x(ctx, x, n);
  if (r) return r;
  r = validate_x(ctx, t, m);
  if (r) return r;
  if (!y || !mean || !cov) return set_err(ctx, LFM_E_ARG, "y / mean / cov is NULL");
  r = check_hyp(ctx, hyp);
  if (r) return r;
  r = check_mean_shape(ctx, n, hyp);
  if (r) return r;
  r = check_mean_shape(ctx, m, hyp);
  if (r) return r;
  if ((n + m) > (int64_t)1 << 17) return set_err(ctx, LFM_E_ARG, "n + m too large");
  DeviceGuard g(ctx->device);
  DeviceTenancy tenancy(ctx, false);  // schedule 1 (Schur complement), shared
  Staged st;
  r = stage_hyp(ctx, hyp, nullptr, 0, false, &st);
  if (r) return r;
  // xin: x (3n) y (n) v (n) t (3m) mean (m) cov (m*m)
  const size_t nd = 5 * (size_t)n + 4 * (size_t)m + (size_t)m * m;
  r = ensure(ctx, (void**)&ctx->xin, &ctx->xin_bytes, nd * 8);
  if (r) return r;
  double* d_x = ctx->xin;
  double* d_y = d_x + 3 * n;
  double* d_v = d_y + n;
  double* d_t = d_v + n;
  double* d_mean = d_t + 3 * m;
  double* d_cov = d_mean + m;
  hipMemcpyAsync(d_x, x, n * 3 * 8, hipMemcpyHostToDevice, ctx->stream);
  hipMemcpyAsync(d_y, y, n * 8, hipMemcpyHostToDevice, ctx->stream);
  if (diag_vec) hipMemcpyAsync(d_v, diag_vec, n * 8, hipMemcpyHostToDevice, ctx->stream);
  hipMemcpyAsync(d_t, t, m * 3 * 8, hipMemcpyHostToDevice, ctx->stream);
  r = posterior_blocked(ctx, st.h, d_x, d_y, n, diag_vec ? d_v : nullptr, diag_add, d_t, m,
                        d_mean, d_cov);
  if (r) return r;
  r = ensure_pinned(ctx, 64 * sizeof(double));
  if (r) return r;
  double* hres = ctx->hpin;
  hipMemcpyAsync(hres, ctx->result, 5 * sizeof(double), hipMemcpyDeviceToHost, ctx->stream);
  hipMemcpyAsync(mean, d_mean, m * 8, hipMemcpyDeviceToHost, ctx->stream);
  hipMemcpyAsync(cov, d_cov, (size_t)m * m * 8, hipMemcpyDeviceToHost, ctx->stream);
  r = finish(ctx);
  if (r) return r;
  r = status_code(ctx, hres[3], hres[4]);
  if (r) {
    const double nan = std::nan("");
    for (int64_t i = 0; i < m; ++i) mean[i] = nan;
    for (int64_t i = 0; i < m * m; ++i) cov[i] = nan;
  }
  return r;
}

int lfm_mll_f64_dev(lfm_ctx* ctx, const double* d_x, const double* d_y, int64_t n,
                    const lfm_hyp* hyp, int negative, double* out) {
  int r = validate_x(ctx, d_x, n);
  if (r) return r;
  if (!d_y || !out) return set_err(ctx, LFM_E_ARG, "y / out is NULL");
  r = check_hyp(ctx, hyp);
  if (r) return r;
  r = check_mean_shape(ctx, n, hyp);
  if (r) return r;
  DeviceGuard g(ctx->device);
  std::vector<double> xh((size_t)n * 3);
  hipError_t e = hipMemcpyAsync(xh.data(), d_x, n * 3 * 8, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "read back x for layout detection");
  if (n <= SMALL_MAX) {
    std::vector<double> yh((size_t)n);
    e = hipMemcpyAsync(yh.data(), d_y, n * 8, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "read back y");
    return lfm_mll_f64(ctx, xh.data(), yh.data(), n, hyp, negative, out);
  }
  Staged st;
  r = stage_hyp(ctx, hyp, xh.data(), n, true, &st);
  if (r) return r;
  return mll_blocked(ctx, st, d_x, d_y, nullptr, n, hyp, negative, out);
}

// A device-resident dataset evaluated many times: x (and, for small n, y) read back once,
// the grid layout analysed once per gene count.
struct lfm_data {
  const double* d_x;
  const double* d_y;
  int64_t n;
  int device;
  std::vector<double> xh, yh;
  int64_t lay_G = -1;
  GridLayout lay;
};

int lfm_data_create(lfm_ctx* ctx, const double* d_x, const double* d_y, int64_t n,
                    lfm_data** out) {
  int r = validate_x(ctx, d_x, n);
  if (r) return r;
  if (!d_y || !out) return set_err(ctx, LFM_E_ARG, "y / out is NULL");
  DeviceGuard g(ctx->device);
  std::unique_ptr<lfm_data> d(new lfm_data);
  d->d_x = d_x;
  d->d_y = d_y;
  d->n = n;
  d->device = ctx->device;
  d->xh.resize((size_t)n * 3);
  hipError_t e = hipMemcpyAsync(d->xh.data(), d_x, n * 3 * 8, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess && n <= SMALL_MAX) {
    d->yh.resize((size_t)n);
    e = hipMemcpyAsync(d->yh.data(), d_y, n * 8, hipMemcpyDeviceToHost, ctx->stream);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "read back the dataset");
  *out = d.release();
  return LFM_OK;
}

int lfm_data_destroy(lfm_data* data) {
  delete data;
  return LFM_OK;
}

int lfm_mll_f64_data(lfm_ctx* ctx, lfm_data* data, const lfm_hyp* hyp, int negative,
                     double* out) {
  if (!ctx) return LFM_E_ARG;
  if (!data || !out) return set_err(ctx, LFM_E_ARG, "data / out is NULL");
  if (data->device != ctx->device) return set_err(ctx, LFM_E_ARG, "dataset of another device");
  int r = check_hyp(ctx, hyp);
  if (r) return r;
  const int64_t n = data->n;
  r = check_mean_shape(ctx, n, hyp);
  if (r) return r;
  DeviceGuard g(ctx->device);
  if (n <= SMALL_MAX) return lfm_mll_f64(ctx, data->xh.data(), data->yh.data(), n, hyp, negative, out);
  if (data->lay_G != hyp->num_genes) {
    data->lay = detect_grid(data->xh.data(), n, hyp->num_genes);
    data->lay_G = hyp->num_genes;
  }
  Staged st;
  r = stage_hyp(ctx, hyp, data->xh.data(), n, true, &st, &data->lay);
  if (r) return r;
  return mll_blocked(ctx, st, data->d_x, data->d_y, nullptr, n, hyp, negative, out);
}

}  // extern "C"

namespace {
// ------------------------------------------------------ C3 restart pipeline
// Workspace i of ctx's restart pipeline (lfm_mll_multi_f64): an lfm_ctx with its own buffers,
// events and flags, whose streams are ctx's — m3 / s3 (in stream order after the previous
// evaluation's launches) and the overlap stream (CU-masked: every CU outside the chain's and the
// first LFM_OVL_RESERVE main CUs, which the previous evaluation's tail keeps).
int twin_get(lfm_ctx* ctx, int i, lfm_ctx** out) {
  if (ctx->twin[i]) {
    *out = ctx->twin[i];
    return LFM_OK;
  }
  if (!ctx->ovl_stream) {
    const int lo = std::min(ctx->cus - 64, ctx->side_cus + ctx->ovl_reserve);
    std::vector<uint32_t> mk((ctx->cus + 31) / 32, 0u);
    for (int c = lo; c < ctx->cus; ++c) mk[c / 32] |= 1u << (c % 32);
    hipError_t e = hipExtStreamCreateWithCUMask(&ctx->ovl_stream, (uint32_t)mk.size(), mk.data());
    if (e != hipSuccess) {
      ctx->ovl_stream = nullptr;
      return hip_fail(ctx, e, "overlap stream");
    }
  }
  std::unique_ptr<lfm_ctx> t(new lfm_ctx());
  t->borrowed = true;
  t->device = ctx->device;
  t->stream = ctx->ovl_stream;
  t->m3 = ctx->m3;
  t->s3 = ctx->s3;
  t->side_req = ctx->side_req;
  t->side_cus = ctx->side_cus;
  t->cus = ctx->cus;
  t->sched = 3;
  t->wait_ticks = ctx->wait_ticks;
  t->grad_direct = ctx->grad_direct;
  t->gram_fuse = ctx->gram_fuse;
  t->w4min = ctx->w4min;
  t->w2min = ctx->w2min;
  t->w0 = ctx->w0;
  t->helper = ctx->helper;
  t->helper_tc = ctx->helper_tc;
  t->helper_min = ctx->helper_min;
  t->s3_fallback = false;  // lfm_mll_multi_f64 re-runs a stalled set itself
  t->ovl_at = ctx->ovl_at;
  std::memset(t->stats, 0, sizeof(t->stats));
  hipError_t e = hipMalloc((void**)&t->linvT, 128 * 128 * sizeof(double));
  if (e == hipSuccess) e = hipMalloc((void**)&t->status, 64);
  if (e == hipSuccess) e = hipMalloc((void**)&t->result, 64 * sizeof(double));
  if (e == hipSuccess) e = hipMalloc((void**)&t->psync, 64);
  if (e == hipSuccess) e = hipMemsetAsync(t->psync, 0, 64, t->stream);
  for (hipEvent_t* ev : {&t->ovl_tail, &t->ovl_done, &t->ovl_res})
    if (e == hipSuccess) e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
  if (e == hipSuccess) e = hipStreamSynchronize(t->stream);
  if (e != hipSuccess) {
    lfm_ctx_destroy(t.release());
    return hip_fail(ctx, e, "restart pipeline workspace");
  }
  *out = ctx->twin[i] = t.release();
  return LFM_OK;
}

// Drain and free the pipeline's workspaces and its overlap stream (the pair they borrow is
// about to go, or the context is).
void twins_drop(lfm_ctx* ctx) {
  if (ctx->borrowed || (!ctx->twin[0] && !ctx->twin[1] && !ctx->ovl_stream)) return;
  for (hipStream_t st : {ctx->ovl_stream, ctx->m3, ctx->s3, ctx->stream})
    if (st) hipStreamSynchronize(st);
  for (lfm_ctx*& t : ctx->twin) {
    lfm_ctx_destroy(t);
    t = nullptr;
  }
  if (ctx->ovl_stream) hipStreamDestroy(ctx->ovl_stream);
  ctx->ovl_stream = nullptr;
}
}  // namespace

extern "C" {

// C3 (BASELINE.json configs[2]): nsets hyperparameter sets on one resident dataset. On schedule
// 3 the evaluations are pipelined over two workspaces: evaluation k + 1's prologue (staging, its
// gram tables / region, chain(0), X_0, chain(1) and step 0) runs on the overlap stream while
// evaluation k is in its chain-bound tail, and the rest of it follows evaluation k's launches
// on the partitioned pair. Every evaluation runs the same kernels on the same inputs as
// lfm_mll_f64_data: the values are bit-identical. Otherwise (small n, schedule 1, profiling,
// LFM_OVERLAP=0, differing gene counts) the sets are evaluated one by one.
int lfm_mll_multi_f64(lfm_ctx* ctx, lfm_data* data, int64_t nsets, const lfm_hyp* hyps,
                      int negative, double* out, int* status) {
  if (!ctx) return LFM_E_ARG;
  if (!data || !out || nsets < 0 || (nsets > 0 && !hyps))
    return set_err(ctx, LFM_E_ARG, "data / hyps / out is NULL or nsets < 0");
  if (data->device != ctx->device) return set_err(ctx, LFM_E_ARG, "dataset of another device");
  const int64_t n = data->n;
  bool same_genes = true;
  for (int64_t k = 0; k < nsets; ++k) {
    int r = check_hyp(ctx, &hyps[k]);
    if (!r) r = check_mean_shape(ctx, n, &hyps[k]);
    if (r) return r;
    same_genes = same_genes && hyps[k].num_genes == hyps[0].num_genes;
  }
  DeviceGuard g(ctx->device);
  int worst = LFM_OK;
  // one set through lfm_mll_f64_data (its own schedule-3 fallback): NOT_PD -> NaN and status
  auto one = [&](int64_t k) -> int {
    int r = lfm_mll_f64_data(ctx, data, &hyps[k], negative, &out[k]);
    if (status) status[k] = r;
    if (r == LFM_E_NOT_PD) {
      out[k] = std::nan("");
      worst = LFM_E_NOT_PD;
      return LFM_OK;
    }
    return r;
  };
  const bool pipelined = nsets >= 2 && n > SMALL_MAX && ctx->ovl_on && s3_on(ctx) &&
                         !ctx->prof && ctx->s3_events == 0 && !ctx->dbg_stamps &&
                         !ctx->dbg_trace && same_genes;
  if (!pipelined) {
    for (int64_t k = 0; k < nsets; ++k)
      if (int r = one(k)) return r;
    if (worst) set_err(ctx, LFM_E_NOT_PD, "Cholesky failed for at least one hyperparameter set");
    return worst;
  }
  if (data->lay_G != hyps[0].num_genes) {
    data->lay = detect_grid(data->xh.data(), n, hyps[0].num_genes);
    data->lay_G = hyps[0].num_genes;
  }
  DeviceTenancy tenancy(ctx, true);  // exclusive, to the last result
  const int64_t Mp = round_up(n + 1, 128);
  lfm_ctx* tw[2];
  for (int i = 0; i < 2; ++i) {
    int r = twin_get(ctx, i, &tw[i]);
    if (!r) r = ensure(tw[i], (void**)&tw[i]->A, &tw[i]->A_bytes, (size_t)Mp * Mp * sizeof(double));
    if (!r) r = ensure_pinned(tw[i], 1 << 16);
    if (r) {
      if (r != LFM_E_ARG) ctx->err = tw[i]->err.empty() ? ctx->err : tw[i]->err;
      return r;
    }
  }
  auto hres = [&](lfm_ctx* t) { return t->hpin + (t->hpin_bytes / 8 - 8); };
  // enqueue set k on workspace k % 2, its prologue gated on set k - 1's tail
  auto enqueue = [&](int64_t k) -> int {
    lfm_ctx* t = tw[k & 1];
    t->ovl = true;
    t->err.clear();
    if (k > 0) hipStreamWaitEvent(t->stream, tw[(k - 1) & 1]->ovl_tail, 0);
    Staged st;
    int r = stage_hyp(t, &hyps[k], data->xh.data(), n, true, &st, &data->lay);
    if (!r) r = mll_enqueue(t, st, data->d_x, data->d_y, nullptr, n, &hyps[k], negative);
    if (!r) {
      hipStreamWaitEvent(ctx->stream, t->ovl_done, 0);
      hipMemcpyAsync(hres(t), t->result, 5 * sizeof(double), hipMemcpyDeviceToHost, ctx->stream);
      hipEventRecord(t->ovl_res, ctx->stream);
      r = hip_fail(ctx, hipGetLastError(), "restart pipeline enqueue");
    } else {
      ctx->err = t->err;
    }
    return r;
  };
  // the host side of set k: LFM_OK / LFM_E_NOT_PD (NaN), LFM_E_TIMEOUT (the caller re-runs)
  auto collect = [&](int64_t k) -> int {
    lfm_ctx* t = tw[k & 1];
    hipError_t e = hipEventSynchronize(t->ovl_res);
    if (e != hipSuccess) return hip_fail(ctx, e, "restart pipeline result");
    const double* h = hres(t);
    out[k] = h[0];
    int r = status_code(t, h[3], h[4]);
    if (status) status[k] = r;
    if (r == LFM_E_NOT_PD) {
      out[k] = std::nan("");
      worst = LFM_E_NOT_PD;
      r = LFM_OK;
    }
    if (r) ctx->err = t->err;
    return r;
  };
  auto drain = [&] {
    for (hipStream_t st : {ctx->ovl_stream, ctx->m3, ctx->s3, ctx->stream})
      if (st) hipStreamSynchronize(st);
    tw[0]->ovl = tw[1]->ovl = false;
  };
  int64_t done = 0;  // sets collected
  int r = enqueue(0);
  for (int64_t k = 1; !r && k <= nsets; ++k) {
    if (k < nsets) r = enqueue(k);
    if (!r) {
      r = collect(k - 1);
      if (!r) done = k;
    }
  }
  drain();
  if (r == LFM_E_TIMEOUT) {
    // a device-side wait ran out (another tenant starved the chain): the rest one by one,
    // each with lfm_mll_f64_data's own schedule-1 re-run
    ctx->fallbacks += 1;
    r = LFM_OK;
    for (int64_t k = done; !r && k < nsets; ++k) r = one(k);
  }
  if (r) return r;
  if (worst) set_err(ctx, LFM_E_NOT_PD, "Cholesky failed for at least one hyperparameter set");
  return worst;
}

int lfm_mll_batch_f64(lfm_ctx* ctx, int64_t nprob, const lfm_problem* probs, int negative,
                      double* out, int* status) {
  if (!ctx) return LFM_E_ARG;
  if (nprob < 0 || (nprob > 0 && (!probs || !out)))
    return set_err(ctx, LFM_E_ARG, "bad batch arguments");
  DeviceGuard g(ctx->device);
  std::vector<int64_t> small, big;
  for (int64_t q = 0; q < nprob; ++q) {
    const lfm_problem& p = probs[q];
    int r = validate_x(ctx, p.x, p.n);
    if (r) return r;
    if (!p.y) return set_err(ctx, LFM_E_ARG, "problem y is NULL");
    r = check_hyp(ctx, &p.hyp);
    if (r) return r;
    r = check_mean_shape(ctx, p.n, &p.hyp);
    if (r) return r;
    (p.n <= SMALL_MAX ? small : big).push_back(q);
  }
  int worst = LFM_OK;
  if (!small.empty()) {
    int r = small_batch(ctx, (int64_t)small.size(), probs, small.data(), negative, out, status);
    if (r) return r;
  }
  for (int64_t q : big) {
    int r = lfm_mll_f64(ctx, probs[q].x, probs[q].y, probs[q].n, &probs[q].hyp, negative, &out[q]);
    if (status) status[q] = r;
    if (r && r != LFM_E_NOT_PD) return r;  // LFM_E_TIMEOUT included: never a NaN slot
  }
  if (status)
    for (int64_t q = 0; q < nprob; ++q)
      if (status[q] == LFM_E_NOT_PD) worst = LFM_E_NOT_PD;
  return worst;
}

// A batch of small problems registered once (the C5 ablation farm, notebook.py:33-75): x / y
// and the problem table live in HBM; the packed hyperparameters, the results and the status
// words live in one pinned host buffer the kernel reads and writes directly, so an evaluation is
// one memcpy into that buffer, ONE kernel launch and one stream synchronise — no copy commands.
struct lfm_batch {
  uint64_t id = 0;  // unique per process (never reused): keys the farm's captured graph
  int device = 0;
  int64_t nprob = 0, nhyp = 0;
  int maxn = 1, maxg = 1, gridtab = 0;
  char* dmem = nullptr;     // device: x / y (+ grid times / block genes) of every problem, then
                            // the SmallProb table
  SmallProb* dprobs = nullptr;
  double* hbuf = nullptr;   // pinned host, coherent: hyp [nhyp] | out [nprob] | status [nprob]
                            // (int); the kernel reads / writes it directly and the host spins on
                            // the status words, so it must not be cached on the device side
  hipEvent_t done = nullptr;  // recorded after every launch on the batch: destroy waits on it
  // small enough for the kernel arguments (LFM_SMALL_KERNARG, default on; read at creation)
  bool use_args = false;
  std::vector<SmallProb> table;      // host copy of the problem table
  std::vector<int> dsb_off, sc_off;  // each problem's offsets in the packed hyperparameters
  int* doffs = nullptr;              // device: dsb_off then sc_off (the gradient / fit kernels)
  double* hgrad = nullptr;           // pinned (in hbuf): the gradient, packed as hyp [nhyp]
  size_t lds_grad = 0, lds_fit = 0;  // the gradient / fit launches' LDS (0: not possible)
  // the fit's device buffers (grown on demand): raw mu nu [3 nhyp] | bias [2 nsteps] |
  // history [nsteps nprob] | status [nprob]
  char* fitbuf = nullptr;
  size_t fit_bytes = 0;
};

int lfm_batch_create(lfm_ctx* ctx, int64_t nprob, const lfm_problem* probs, lfm_batch** out) {
  if (!ctx) return LFM_E_ARG;
  if (!out || nprob < 1 || !probs) return set_err(ctx, LFM_E_ARG, "bad batch arguments");
  *out = nullptr;
  int64_t nd = 0, nhyp = 0;
  int maxn = 1, maxg = 1;
  for (int64_t q = 0; q < nprob; ++q) {
    const lfm_problem& p = probs[q];
    int r = validate_x(ctx, p.x, p.n);
    if (r) return r;
    if (!p.y) return set_err(ctx, LFM_E_ARG, "problem y is NULL");
    if (p.n > SMALL_MAX)
      return set_err(ctx, LFM_E_ARG, "lfm_batch: every problem needs n <= 128 (one workgroup each)");
    if (p.hyp.num_genes < 1 || p.hyp.num_genes > p.n)
      return set_err(ctx, LFM_E_ARG, "lfm_batch: num_genes must be in [1, n]");
    r = check_mean_shape(ctx, p.n, &p.hyp);
    if (r) return r;
    nd += 4 * p.n + small_grid_doubles(p.n);
    nhyp += 3 * p.hyp.num_genes + 3;
    maxn = std::max<int>(maxn, (int)p.n);
    maxg = std::max<int>(maxg, (int)p.hyp.num_genes);
  }
  DeviceGuard g(ctx->device);
  std::unique_ptr<lfm_batch> b(new lfm_batch);
  static std::atomic<uint64_t> next_id{0};
  b->id = ++next_id;
  b->device = ctx->device;
  b->nprob = nprob;
  b->nhyp = nhyp;
  b->maxn = maxn;
  b->maxg = maxg;
  const size_t bytes_d = round_up(nd * 8, 16), bytes_p = round_up((size_t)nprob * sizeof(SmallProb), 16);
  const size_t bytes_o = 2 * (size_t)nprob * sizeof(int);
  hipError_t e = hipMalloc((void**)&b->dmem, bytes_d + bytes_p + bytes_o);
  if (e != hipSuccess) return hip_fail(ctx, e, "lfm_batch_create: device buffer");
  // coherent (fine-grained): the kernel reads the hyperparameters a call has just written and
  // its result / status stores must reach the host's spin without a stream synchronise,
  // whatever HIP_HOST_COHERENT says
  e = hipHostMalloc((void**)&b->hbuf, (size_t)(2 * nhyp + 2 * nprob) * 8, hipHostMallocCoherent);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&b->done, hipEventDisableTiming);
  if (e != hipSuccess) {
    hipFree(b->dmem);
    if (b->hbuf) hipHostFree(b->hbuf);
    return hip_fail(ctx, e, "lfm_batch_create: pinned buffer");
  }
  b->dprobs = reinterpret_cast<SmallProb*>(b->dmem + bytes_d);
  b->doffs = reinterpret_cast<int*>(b->dmem + bytes_d + bytes_p);
  b->hgrad = b->hbuf + nhyp + 2 * nprob;
  std::vector<double> hd((size_t)nd);
  std::vector<SmallProb> table((size_t)nprob);
  const double* dd = reinterpret_cast<const double*>(b->dmem);
  int64_t off = 0, hv = 0, hs = 0;
  const int64_t nvec = nhyp - 3 * nprob;  // the vectors first, then the scalars
  for (int64_t q = 0; q < nprob; ++q) {
    const lfm_problem& p = probs[q];
    const int64_t n = p.n, G = p.hyp.num_genes;
    SmallProb& sp = table[q];
    std::memcpy(&hd[off], p.x, 3 * n * 8);
    sp.x = dd + off;
    off += 3 * n;
    std::memcpy(&hd[off], p.y, n * 8);
    sp.y = dd + off;
    off += n;
    sp.dsb = b->hbuf + hv;
    hv += 3 * G;
    sp.sc = b->hbuf + nvec + hs;
    hs += 3;
    sp.n = (int)n;
    sp.G = (int)G;
    off += small_grid_pack(p.x, n, G, sp, &hd[off], dd + off);
    if (sp.T) b->gridtab = std::max<int>(b->gridtab, (int)small_grid_extra((int)n, (int)G, sp.T));
    b->dsb_off.push_back((int)(hv - 3 * G));
    b->sc_off.push_back((int)(nvec + hs - 3));
  }
  b->use_args = ctx->small_kernarg && nprob <= SMALL_ARG_PROBS &&
                nhyp <= SMALL_ARG_HYP;
  b->table = table;
  // the gradient / fit kernels: every problem's augmented matrix on one or two waves
  // (n + 1 <= 128) and its LDS map within a CU's 160 KB
  if (maxn <= SMALL_GRAD_MAX) {
    b->lds_grad = small_grad_lds(table.data(), (int)nprob, 0);
    b->lds_fit = small_grad_lds(table.data(), (int)nprob, 1);
    if (b->lds_grad > 160 * 1024) b->lds_grad = 0;
    if (b->lds_fit > 160 * 1024) b->lds_fit = 0;
  }
  std::vector<int> offs(b->dsb_off);
  offs.insert(offs.end(), b->sc_off.begin(), b->sc_off.end());
  e = hipMemcpyAsync(b->dmem, hd.data(), (size_t)nd * 8, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(b->dprobs, table.data(), (size_t)nprob * sizeof(SmallProb),
                       hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(b->doffs, offs.data(), bytes_o, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) {
    hipFree(b->dmem);
    hipHostFree(b->hbuf);
    return hip_fail(ctx, e, "lfm_batch_create: upload");
  }
  *out = b.release();
  return LFM_OK;
}

int lfm_batch_hyp_size(const lfm_batch* batch, int64_t* out) {
  if (!batch || !out) return LFM_E_ARG;
  *out = batch->nhyp;
  return LFM_OK;
}

int lfm_batch_destroy(lfm_batch* batch) {
  if (!batch) return LFM_OK;
  hipSetDevice(batch->device);
  // an evaluation returns once its status words land, possibly before its kernel has retired:
  // wait for the batch's last launch (not the whole device: other contexts' streams may be busy
  // or stuck) before the buffers go
  if (batch->done) {
    hipEventSynchronize(batch->done);
    hipEventDestroy(batch->done);
  }
  hipFree(batch->dmem);
  if (batch->fitbuf) hipFree(batch->fitbuf);
  hipHostFree(batch->hbuf);
  delete batch;
  return LFM_OK;
}

}  // extern "C"

namespace {
// One launch of the batch's MLL kernel: results to `out` (the pinned buffer, or a device buffer
// such as the farm's send slots), the status words (reset to -1 here, each written last by its
// workgroup after a system-scope fence) to the pinned buffer.
// The previous call on a batch returned on its status words, possibly before its kernel had
// retired: a fault past that point surfaces at the batch's next call (this query of that launch's
// completion event, long signalled in the normal case), not at some later synchronise.
int batch_prev_ok(lfm_ctx* ctx, const lfm_batch* batch) {
  if (!batch->done) return LFM_OK;
  const hipError_t e = hipEventQuery(batch->done);
  if (e != hipSuccess && e != hipErrorNotReady)
    return hip_fail(ctx, e, "the batch's previous launch");
  return LFM_OK;
}

int batch_launch(lfm_ctx* ctx, lfm_batch* batch, const double* hyp, int negative, double* out) {
  if (int r = batch_prev_ok(ctx, batch)) return r;
  const int64_t np = batch->nprob;
  int* hst = reinterpret_cast<int*>(batch->hbuf + batch->nhyp + np);
  for (int64_t q = 0; q < np; ++q) hst[q] = -1;  // a problem's status word is written last
  int r;
  if (batch->use_args) {
    // the problem table and the hyperparameters travel in the kernel arguments
    SmallArgs a;
    std::memcpy(a.probs, batch->table.data(), (size_t)np * sizeof(SmallProb));
    std::memcpy(a.hyp, hyp, (size_t)batch->nhyp * 8);
    std::memcpy(a.dsb_off, batch->dsb_off.data(), (size_t)np * sizeof(int));
    std::memcpy(a.sc_off, batch->sc_off.data(), (size_t)np * sizeof(int));
    a.out = out;
    a.status = hst;
    a.negative = negative;
    r = launch_small_args(ctx, a, (int)np, batch->maxn, batch->maxg, batch->gridtab);
  } else {
    std::memcpy(batch->hbuf, hyp, (size_t)batch->nhyp * 8);
    r = launch_small_batch(ctx, batch->dprobs, (int)np, batch->maxn, batch->maxg,
                           batch->gridtab, negative, out, hst);
  }
  if (r) return r;
  hipEventRecord(batch->done, ctx->stream);
  return LFM_OK;
}

// Result words the host is still waiting for: a signalling-NaN payload that no kernel writes
// (its arithmetic yields values or the canonical quiet NaN; the padding slots are all-ones).
constexpr uint64_t RESULT_PENDING = 0x7FF41F0DCAFE0001ull;
void mark_pending(double* p, int64_t count) {
  uint64_t* w = reinterpret_cast<uint64_t*>(p);
  for (int64_t q = 0; q < count; ++q) w[q] = RESULT_PENDING;
}
bool all_landed(const double* p, int64_t count) {
  const uint64_t* w = reinterpret_cast<const uint64_t*>(p);
  for (int64_t q = 0; q < count; ++q)
    if (__atomic_load_n(&w[q], __ATOMIC_ACQUIRE) == RESULT_PENDING) return false;
  return true;
}

// The host side of a call whose kernel writes results and status words into the batch's
// pinned buffer: spin until EVERY word the call reads has landed — the status words (-1 before
// the launch), the results and the gradient (RESULT_PENDING before the launch) — rather than on
// the status words alone: each word is its own completion flag, so the host never depends on the
// order in which two posted writes to host memory become visible (the kernel's system-scope fence
// orders their issue). ~µs sooner than the kernel's end-of-dispatch signal
// behind hipStreamSynchronize; past 20 ms, or while profiling (the events want the stream),
// synchronise the stream instead, which also surfaces a kernel fault.
int batch_wait(lfm_ctx* ctx, int64_t np, const int* hst, const double* vals, int64_t nv,
               const double* grads = nullptr, int64_t ng = 0) {
  bool landed = false;
  if (!ctx->prof) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      landed = true;
      for (int64_t q = 0; q < np && landed; ++q)
        landed = __atomic_load_n(&hst[q], __ATOMIC_ACQUIRE) != -1;
      landed = landed && all_landed(vals, nv) && all_landed(grads, ng);
      if (landed || std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) break;
      __builtin_ia32_pause();
    }
  }
  return landed ? LFM_OK : finish(ctx);
}

// statuses of the batch's last call -> status[] (optional); LFM_E_NOT_PD if any problem failed
int batch_status(lfm_ctx* ctx, const lfm_batch* batch, int* status) {
  const int* hst = reinterpret_cast<const int*>(batch->hbuf + batch->nhyp + batch->nprob);
  int worst = LFM_OK;
  for (int64_t q = 0; q < batch->nprob; ++q) {
    const int s = hst[q] ? LFM_E_NOT_PD : LFM_OK;
    if (status) status[q] = s;
    if (s) worst = s;
  }
  if (worst) set_err(ctx, LFM_E_NOT_PD, "Cholesky failed: non-positive pivot in a batch problem");
  return worst;
}
}  // namespace

extern "C" {

int lfm_batch_mll_f64(lfm_ctx* ctx, lfm_batch* batch, const double* hyp, int negative,
                      double* out, int* status) {
  if (!ctx) return LFM_E_ARG;
  if (!batch || !hyp || !out) return set_err(ctx, LFM_E_ARG, "batch / hyp / out is NULL");
  if (batch->device != ctx->device) return set_err(ctx, LFM_E_ARG, "batch of another device");
  DeviceGuard g(ctx->device);
  const int64_t np = batch->nprob;
  double* hres = batch->hbuf + batch->nhyp;
  mark_pending(hres, np);
  int r = batch_launch(ctx, batch, hyp, negative, hres);
  if (r) return r;
  r = batch_wait(ctx, np, reinterpret_cast<const int*>(hres + np), hres, np);
  if (r) return r;
  std::memcpy(out, hres, (size_t)np * 8);
  return batch_status(ctx, batch, status);
}

int lfm_batch_mll_grad_f64(lfm_ctx* ctx, lfm_batch* batch, const double* hyp, int negative,
                           double* value, double* grad, int* status) {
  if (!ctx) return LFM_E_ARG;
  if (!batch || !hyp || !value || !grad)
    return set_err(ctx, LFM_E_ARG, "batch / hyp / value / grad is NULL");
  if (batch->device != ctx->device) return set_err(ctx, LFM_E_ARG, "batch of another device");
  if (!batch->lds_grad)
    return set_err(ctx, LFM_E_ARG, "lfm_batch_mll_grad_f64: every problem needs n <= 127 and its "
                                   "map within 160 KB of LDS; use lfm_mll_grad_f64");
  DeviceGuard g(ctx->device);
  const int64_t np = batch->nprob;
  double* hres = batch->hbuf + batch->nhyp;
  int* hst = reinterpret_cast<int*>(hres + np);
  if (int e = batch_prev_ok(ctx, batch)) return e;
  for (int64_t q = 0; q < np; ++q) hst[q] = -1;
  mark_pending(hres, np);
  mark_pending(batch->hgrad, batch->nhyp);
  int r;
  if (batch->use_args) {
    SmallArgs a;
    std::memcpy(a.probs, batch->table.data(), (size_t)np * sizeof(SmallProb));
    std::memcpy(a.hyp, hyp, (size_t)batch->nhyp * 8);
    std::memcpy(a.dsb_off, batch->dsb_off.data(), (size_t)np * sizeof(int));
    std::memcpy(a.sc_off, batch->sc_off.data(), (size_t)np * sizeof(int));
    a.tabs = 1;
    r = launch_small_grad(ctx, &a, nullptr, nullptr, (int)np, batch->lds_grad, negative, hres,
                          batch->hgrad, hst);
  } else {
    std::memcpy(batch->hbuf, hyp, (size_t)batch->nhyp * 8);
    r = launch_small_grad(ctx, nullptr, batch->dprobs, batch->doffs, (int)np, batch->lds_grad,
                          negative, hres, batch->hgrad, hst);
  }
  if (r) return r;
  hipEventRecord(batch->done, ctx->stream);
  r = batch_wait(ctx, np, hst, hres, np, batch->hgrad, batch->nhyp);
  if (r) return r;
  int worst = LFM_OK;
  std::memcpy(grad, batch->hgrad, (size_t)batch->nhyp * 8);
  for (int64_t q = 0; q < np; ++q) {
    value[q] = hres[q];
    const int s = hst[q] ? LFM_E_NOT_PD : LFM_OK;
    if (status) status[q] = s;
    if (s) worst = s;
  }
  if (worst) set_err(ctx, LFM_E_NOT_PD, "Cholesky failed: non-positive pivot in a batch problem");
  return worst;
}

int lfm_batch_fit_f64(lfm_ctx* ctx, lfm_batch* batch, const lfm_adam* opt, int negative,
                      int64_t step0, int64_t nsteps, double* raw, double* mu, double* nu,
                      double* history, int* status) {
  if (!ctx) return LFM_E_ARG;
  if (!batch || !opt || !raw || !mu || !nu || (nsteps > 0 && !history) || step0 < 0 ||
      nsteps < 0 || opt->num_steps_per_epoch < 1)
    return set_err(ctx, LFM_E_ARG, "bad fit arguments");
  if (batch->device != ctx->device) return set_err(ctx, LFM_E_ARG, "batch of another device");
  if (!batch->lds_fit)
    return set_err(ctx, LFM_E_ARG, "lfm_batch_fit_f64: every problem needs n <= 127 and its map "
                                   "within 160 KB of LDS");
  if (nsteps == 0) return LFM_OK;
  DeviceGuard g(ctx->device);
  if (int e = batch_prev_ok(ctx, batch)) return e;
  const int64_t np = batch->nprob, nh = batch->nhyp;
  const size_t b_par = 3 * (size_t)nh * 8, b_bias = 2 * (size_t)nsteps * 8;
  const size_t b_hist = (size_t)nsteps * np * 8, b_st = (size_t)np * sizeof(int);
  const size_t need = b_par + b_bias + b_hist + b_st;
  if (batch->fit_bytes < need) {
    hipStreamSynchronize(ctx->stream);
    if (batch->fitbuf) hipFree(batch->fitbuf);
    batch->fitbuf = nullptr;
    batch->fit_bytes = 0;
    hipError_t e = hipMalloc((void**)&batch->fitbuf, need);
    if (e != hipSuccess) return hip_fail(ctx, e, "lfm_batch_fit_f64: device buffer");
    batch->fit_bytes = need;
  }
  double* d_par = reinterpret_cast<double*>(batch->fitbuf);
  double* d_bias = d_par + 3 * nh;
  double* d_hist = d_bias + 2 * nsteps;
  int* d_st = reinterpret_cast<int*>(d_hist + nsteps * np);
  // optax's bias corrections 1 - b^count, count = step0 + s + 1, with the host's pow (the
  // restatement's numbers: dis_project_amd/trainer.py adam)
  std::vector<double> bias((size_t)2 * nsteps), par((size_t)3 * nh);
  for (int64_t s = 0; s < nsteps; ++s) {
    const double count = (double)(step0 + s + 1);
    bias[2 * s] = 1.0 - std::pow(opt->b1, count);
    bias[2 * s + 1] = 1.0 - std::pow(opt->b2, count);
  }
  std::memcpy(par.data(), raw, nh * 8);
  std::memcpy(par.data() + nh, mu, nh * 8);
  std::memcpy(par.data() + 2 * nh, nu, nh * 8);
  hipError_t e = hipMemcpyAsync(d_par, par.data(), b_par, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(d_bias, bias.data(), b_bias, hipMemcpyHostToDevice, ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "lfm_batch_fit_f64: upload");
  SmallFitLaunch f{};
  f.probs = batch->dprobs;
  f.offs = batch->doffs;
  f.nprob = (int)np;
  f.raw = d_par;
  f.mu = d_par + nh;
  f.nu = d_par + 2 * nh;
  f.history = d_hist;
  f.bias = d_bias;
  f.status = d_st;
  f.lr = opt->learning_rate;
  f.b1 = opt->b1;
  f.b2 = opt->b2;
  f.eps = opt->eps;
  f.eps_root = opt->eps_root;
  f.step0 = step0;
  f.nsteps = nsteps;
  f.spe = opt->num_steps_per_epoch;
  f.fix = opt->fix_params != 0;
  f.negative = negative;
  int r = launch_small_fit(ctx, f, batch->lds_fit);
  if (r) return r;
  hipEventRecord(batch->done, ctx->stream);
  std::vector<int> st((size_t)np);
  e = hipMemcpyAsync(par.data(), d_par, b_par, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(history, d_hist, b_hist, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(st.data(), d_st, b_st, hipMemcpyDeviceToHost, ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "lfm_batch_fit_f64: download");
  r = finish(ctx);
  if (r) return r;
  // the packed layout's jitter slots pass through unchanged (a static field, model.py:64)
  std::memcpy(raw, par.data(), nh * 8);
  std::memcpy(mu, par.data() + nh, nh * 8);
  std::memcpy(nu, par.data() + 2 * nh, nh * 8);
  int worst = LFM_OK;
  for (int64_t q = 0; q < np; ++q) {
    if (status) status[q] = st[q];
    if (st[q]) worst = LFM_E_NOT_PD;
  }
  if (worst)
    set_err(ctx, LFM_E_NOT_PD, "Cholesky failed during the fit of a batch problem (its loss "
                               "and parameters are NaN from that step on, as JAX's)");
  return worst;
}

int lfm_log_prob_f64(lfm_ctx* ctx, const double* loc, const double* scale, int64_t n,
                     int64_t lds, const double* y, double* out) {
  if (!ctx) return LFM_E_ARG;
  if (!loc || !scale || !y || !out || n < 1 || lds < n)
    return set_err(ctx, LFM_E_ARG, "bad log_prob arguments");
  DeviceGuard g(ctx->device);
  const int64_t Mp = round_up(n + 1, 128);
  int r = ensure(ctx, (void**)&ctx->A, &ctx->A_bytes, (size_t)Mp * Mp * sizeof(double));
  if (r) return r;
  r = ensure(ctx, (void**)&ctx->xin, &ctx->xin_bytes, (size_t)n * 2 * 8);
  if (r) return r;
  hipMemcpyAsync(ctx->xin, loc, n * 8, hipMemcpyHostToDevice, ctx->stream);
  hipMemcpyAsync(ctx->xin + n, y, n * 8, hipMemcpyHostToDevice, ctx->stream);
  r = ensure_pinned(ctx, 1 << 16);
  if (r) return r;
  DeviceTenancy tenancy(ctx, s3_on(ctx));  // held to the final synchronise (finish)
  return with_s3_fallback(ctx, [&]() -> int {
    // the factorisation overwrites A: a fallback re-run uploads scale again
    hipError_t e = hipMemcpy2DAsync(ctx->A, Mp * 8, scale, lds * 8, n * 8, n,
                                    hipMemcpyHostToDevice, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "upload scale");
    HypDev h{nullptr, nullptr, nullptr, 1, 1.0};
    int r = launch_augment(ctx, h, nullptr, ctx->xin + n, ctx->xin, n, ctx->A, Mp, Mp);
    if (r) return r;
    r = chol_factor_solve(ctx, ctx->A, Mp, n, Mp, 0, ctx->result);
    if (r) return r;
    double* hres = ctx->hpin + (ctx->hpin_bytes / 8 - 8);
    hipMemcpyAsync(hres, ctx->result, 5 * sizeof(double), hipMemcpyDeviceToHost, ctx->stream);
    r = finish(ctx);
    if (r) return r;
    *out = hres[0];
    r = status_code(ctx, hres[3], hres[4]);
    if (r) *out = std::nan("");
    return r;
  });
}

int lfm_dev_alloc(lfm_ctx* ctx, size_t bytes, void** out) {
  if (!ctx || !out) return LFM_E_ARG;
  DeviceGuard g(ctx->device);
  hipError_t e = hipMalloc(out, bytes ? bytes : 16);
  return hip_fail(ctx, e, "lfm_dev_alloc");
}

int lfm_dev_free(lfm_ctx* ctx, void* p) {
  if (!ctx) return LFM_E_ARG;
  DeviceGuard g(ctx->device);
  hipStreamSynchronize(ctx->stream);
  return hip_fail(ctx, hipFree(p), "lfm_dev_free");
}

int lfm_memcpy_h2d(lfm_ctx* ctx, void* dst, const void* src, size_t bytes) {
  if (!ctx) return LFM_E_ARG;
  DeviceGuard g(ctx->device);
  hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "h2d");
  return finish(ctx);
}

int lfm_memcpy_d2h(lfm_ctx* ctx, void* dst, const void* src, size_t bytes) {
  if (!ctx) return LFM_E_ARG;
  DeviceGuard g(ctx->device);
  hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "d2h");
  return finish(ctx);
}

int lfm_memset_dev(lfm_ctx* ctx, void* dst, int value, size_t bytes) {
  if (!ctx || (!dst && bytes)) return LFM_E_ARG;
  DeviceGuard g(ctx->device);
  hipError_t e = hipMemsetAsync(dst, value, bytes, ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "memset");
  return finish(ctx);
}

int lfm_profile_enable(lfm_ctx* ctx, int on) {
  if (!ctx) return LFM_E_ARG;
  ctx->prof = on != 0;
  return LFM_OK;
}

int lfm_profile_classes(lfm_ctx* ctx, unsigned mask) {
  if (!ctx) return LFM_E_ARG;
  ctx->prof_mask = mask;
  return LFM_OK;
}

int lfm_profile_reset(lfm_ctx* ctx) {
  if (!ctx) return LFM_E_ARG;
  DeviceGuard g(ctx->device);
  finish(ctx);
  prof_flush(ctx);
  for (int i = 0; i < K_NCLASS; ++i) {
    ctx->stats[i].launches = 0;
    ctx->stats[i].total_ms = 0;
    ctx->stats[i].flops = 0;
    ctx->stats[i].bytes = 0;
    ctx->stats[i].issued_flops = 0;
  }
  return LFM_OK;
}

int lfm_profile_read(lfm_ctx* ctx, lfm_kstat* stats, int max, int* count) {
  if (!ctx || !count) return LFM_E_ARG;
  DeviceGuard g(ctx->device);
  finish(ctx);
  prof_flush(ctx);
  *count = K_NCLASS;
  for (int i = 0; i < std::min(max, (int)K_NCLASS); ++i) stats[i] = ctx->stats[i];
  return LFM_OK;
}

// ------------------------------------------------------------- RCCL farm
// librccl is opened lazily so the library loads (and the CPU tests run) without it.
namespace {
// Holds its stream for `ticks` of the 100 MHz constant clock, then exits (one wave).
__global__ void stall_kernel(unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

// The end of a device-side farm round: the gathered slots to pinned host memory, then the round's
// sequence number — the host's completion signal (it spins on that word instead of synchronising
// the stream: microseconds sooner). ONE wave (launched with 64 threads): the sequence word's
// system-scope release store waits for every store the wave issued before it (s_waitcnt
// vmcnt(0) is per wave) after the L2 write-back, so the slots land first; a per-thread
// __threadfence_system before it would only repeat that write-back.
__global__ __launch_bounds__(64) void farm_publish_kernel(const double* __restrict__ src,
                                                         int64_t count, double* __restrict__ dst,
                                                         unsigned* seq_word, unsigned seq) {
  for (int64_t i = threadIdx.x; i < count; i += 64) dst[i] = src[i];
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_store(seq_word, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct Rccl {
  void* h = nullptr;
  ncclResult_t (*getUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*commInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*allGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t,
                            hipStream_t) = nullptr;
  ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
  const char* (*errStr)(ncclResult_t) = nullptr;
  // optional (non-blocking communicator, bounded waits): absent -> blocking init
  ncclResult_t (*commInitRankConfig)(ncclComm_t*, int, ncclUniqueId, int, ncclConfig_t*) = nullptr;
  ncclResult_t (*commGetAsyncError)(ncclComm_t, ncclResult_t*) = nullptr;
  ncclResult_t (*commAbort)(ncclComm_t) = nullptr;
};
Rccl g_rccl;

int rccl_load(lfm_ctx* ctx) {
  if (g_rccl.h) return LFM_OK;
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
  if (!h) return set_err(ctx, LFM_E_RCCL, std::string("dlopen librccl: ") + dlerror());
  g_rccl.getUniqueId = (decltype(g_rccl.getUniqueId))dlsym(h, "ncclGetUniqueId");
  g_rccl.commInitRank = (decltype(g_rccl.commInitRank))dlsym(h, "ncclCommInitRank");
  g_rccl.allGather = (decltype(g_rccl.allGather))dlsym(h, "ncclAllGather");
  g_rccl.commDestroy = (decltype(g_rccl.commDestroy))dlsym(h, "ncclCommDestroy");
  g_rccl.errStr = (decltype(g_rccl.errStr))dlsym(h, "ncclGetErrorString");
  g_rccl.commInitRankConfig =
      (decltype(g_rccl.commInitRankConfig))dlsym(h, "ncclCommInitRankConfig");
  g_rccl.commGetAsyncError = (decltype(g_rccl.commGetAsyncError))dlsym(h, "ncclCommGetAsyncError");
  g_rccl.commAbort = (decltype(g_rccl.commAbort))dlsym(h, "ncclCommAbort");
  if (!g_rccl.getUniqueId || !g_rccl.commInitRank || !g_rccl.allGather || !g_rccl.commDestroy)
    return set_err(ctx, LFM_E_RCCL, "librccl lacks a required symbol");
  g_rccl.h = h;
  return LFM_OK;
}

int rccl_fail(lfm_ctx* ctx, ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return LFM_OK;
  return set_err(ctx, LFM_E_RCCL,
                 std::string(what) + ": " + (g_rccl.errStr ? g_rccl.errStr(r) : "rccl error"));
}

// Bound on every wait of a non-blocking communicator (seconds, LFM_RCCL_TIMEOUT_S at context
// creation, default 300): a peer rank that died or never joined ends the call with LFM_E_RCCL
// instead of a hang.
double rccl_timeout_s(const lfm_ctx* ctx) { return ctx->rccl_timeout_s; }

double mono_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

// Waiting on a latency-bound exchange (a 16-256 B all-gather takes tens of microseconds over
// xGMI): poll tightly for the first 2 ms, then back off to 20 us sleeps, and to 200 us past
// 100 ms (a peer still initialising, or one that never arrives before the deadline).
struct Backoff {
  double t0 = mono_s();
  void pause() const {
    const double el = mono_s() - t0;
    if (el < 2e-3) return;  // spin: the next poll follows at once
    usleep(el < 0.1 ? 20 : 200);
  }
};

// End a communicator after a failed or timed-out operation: ncclCommAbort (a non-blocking
// communicator's pending kernels are released), and the context forgets it.
// Work the aborted call left queued on the stream (its copies into the farm's pinned staging,
// its publish kernel) may still run: farm_stale makes the next call drain it first (bounded), and
// abandon the staging buffers if it does not drain (a bounded leak instead of a late write into
// memory the next call is using).
// Forget the captured farm round (its buffers, batch or communicator are changing; nothing of it
// is in flight).
void farm_graph_reset(lfm_ctx* ctx) {
  if (ctx->farm_exec) hipGraphExecDestroy(ctx->farm_exec);
  ctx->farm_exec = nullptr;
  ctx->farm_exec_batch = 0;
}

void rccl_drop(lfm_ctx* ctx) {
  // a replay of the captured round may still be queued: the graph is set aside and destroyed
  // only once the stream has drained (farm_drain_stale; a second abort before that leaks one)
  if (ctx->farm_exec) {
    ctx->farm_exec_old = ctx->farm_exec;
    ctx->farm_exec = nullptr;
    ctx->farm_exec_batch = 0;
  }
  if (!ctx->comm) return;
  if (g_rccl.commAbort) g_rccl.commAbort((ncclComm_t)ctx->comm);
  else if (g_rccl.commDestroy) g_rccl.commDestroy((ncclComm_t)ctx->comm);
  ctx->comm = nullptr;
  ctx->nranks = 0;
  ctx->rank = -1;
  ctx->farm_stale = true;
}

// Poll a non-blocking communicator until its pending operation leaves ncclInProgress.
int rccl_poll(lfm_ctx* ctx, ncclComm_t comm, const char* what) {
  const double end = mono_s() + rccl_timeout_s(ctx);
  const Backoff bo;
  for (;;) {
    ncclResult_t st = ncclInProgress;
    const ncclResult_t q = g_rccl.commGetAsyncError(comm, &st);
    if (q != ncclSuccess) return rccl_fail(ctx, q, what);
    if (st != ncclInProgress) return rccl_fail(ctx, st, what);
    if (mono_s() > end)
      return set_err(ctx, LFM_E_RCCL, std::string(what) + ": timed out (a peer rank did not join)");
    bo.pause();
  }
}

// Bounded wait for everything enqueued on the context's stream (the collective included): a
// collective whose peers never arrive would otherwise block the stream, and the caller, forever.
int rccl_stream_wait(lfm_ctx* ctx, const char* what) {
  const double end = mono_s() + rccl_timeout_s(ctx);
  const Backoff bo;
  hipError_t e;
  while ((e = hipStreamQuery(ctx->stream)) == hipErrorNotReady) {
    const double now = mono_s();
    if (now > end) {
      char waited[64];
      std::snprintf(waited, sizeof(waited), " after %.2f s", now - bo.t0);
      return set_err(ctx, LFM_E_RCCL,
                     std::string(what) + ": timed out" + waited + " (a peer rank did not arrive)");
    }
    bo.pause();
  }
  return hip_fail(ctx, e, what);
}
}  // namespace

int lfm_farm_unique_id(lfm_ctx* ctx, unsigned char id[128]) {
  if (!ctx || !id) return LFM_E_ARG;
  int r = rccl_load(ctx);
  if (r) return r;
  DeviceGuard g(ctx->device);
  ncclUniqueId u;
  r = rccl_fail(ctx, g_rccl.getUniqueId(&u), "ncclGetUniqueId");
  if (r) return r;
  std::memcpy(id, u.internal, 128);
  return LFM_OK;
}

int lfm_farm_init(lfm_ctx* ctx, const unsigned char id[128], int nranks, int rank) {
  if (!ctx || !id || nranks < 1 || rank < 0 || rank >= nranks) return LFM_E_ARG;
  int r = rccl_load(ctx);
  if (r) return r;
  DeviceGuard g(ctx->device);
  if (ctx->comm) lfm_farm_destroy(ctx);
  ncclUniqueId u;
  std::memcpy(u.internal, id, 128);
  ncclComm_t comm = nullptr;
  bool nb = false;
  if (g_rccl.commInitRankConfig && g_rccl.commGetAsyncError && g_rccl.commAbort) {
    // non-blocking communicator: the init (and every later call) is polled against a deadline
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    const ncclResult_t q = g_rccl.commInitRankConfig(&comm, nranks, u, rank, &cfg);
    if (q == ncclSuccess || q == ncclInProgress) {
      r = rccl_poll(ctx, comm, "ncclCommInitRankConfig");
      if (r) {
        g_rccl.commAbort(comm);
        return r;
      }
      nb = true;
    } else if (q != ncclInvalidArgument) {
      return rccl_fail(ctx, q, "ncclCommInitRankConfig");
    } else {
      comm = nullptr;  // a library that rejects this config layout: blocking init below
    }
  }
  if (!nb) {
    r = rccl_fail(ctx, g_rccl.commInitRank(&comm, nranks, u, rank), "ncclCommInitRank");
    if (r) return r;
  }
  ctx->comm = comm;
  ctx->comm_nb = nb;
  ctx->nranks = nranks;
  ctx->rank = rank;
  ++ctx->comm_gen;
  return LFM_OK;
}

}  // extern "C"

namespace {
// Before a farm call writes its host staging: work a dropped (timed-out) call left queued is
// drained, within the communicator's time bound; if it does not drain, the staging buffers it
// could still write are abandoned (never freed, never reused) and fresh ones are made.
int farm_drain_stale(lfm_ctx* ctx) {
  if (!ctx->farm_stale) return LFM_OK;
  const double end = mono_s() + std::min(rccl_timeout_s(ctx), 5.0);
  const Backoff bo;
  hipError_t e;
  while ((e = hipStreamQuery(ctx->stream)) == hipErrorNotReady && mono_s() < end) bo.pause();
  if (e == hipErrorNotReady) {
    farm_graph_reset(ctx);
    ctx->farm_h = nullptr;  // abandoned: a queued copy may still land in it
    ctx->farm_h_bytes = 0;
    ctx->farm_pub = nullptr;
    ctx->farm_pub_bytes = 0;
    ctx->farm_buf = nullptr;  // (device) the same for the queued collective's buffers
    ctx->farm_bytes = 0;
  } else if (e != hipSuccess) {
    return hip_fail(ctx, e, "draining the aborted farm call");
  } else if (ctx->farm_exec_old) {
    hipGraphExecDestroy(ctx->farm_exec_old);
    ctx->farm_exec_old = nullptr;
  }
  ctx->farm_stale = false;
  return LFM_OK;
}

// The device-side round's buffers: send [slots] | recv [nranks slots] on the device, the
// publish target (recv's copy + a sequence word) in coherent pinned host memory.
int farm_buffers(lfm_ctx* ctx, size_t slots) {
  const size_t in = slots * 8, out = in * ctx->nranks;
  const double* before = ctx->farm_buf;
  int r = ensure(ctx, (void**)&ctx->farm_buf, &ctx->farm_bytes, in + out);
  if (r) return r;
  if (ctx->farm_buf != before) farm_graph_reset(ctx);
  const size_t pub = out + 64;
  if (!ctx->farm_pub || ctx->farm_pub_bytes < pub) {
    farm_graph_reset(ctx);
    if (ctx->farm_pub) {
      hipStreamSynchronize(ctx->stream);
      hipHostFree(ctx->farm_pub);
      ctx->farm_pub = nullptr;
    }
    hipError_t e = hipHostMalloc((void**)&ctx->farm_pub, pub, hipHostMallocCoherent);
    if (e != hipSuccess) return hip_fail(ctx, e, "farm publish buffer");
    ctx->farm_pub_bytes = pub;
  }
  return LFM_OK;
}

int farm_wait(lfm_ctx* ctx, const unsigned* seq_word, unsigned seq, int64_t count, double* recv);

// Enqueue the all-gather of `slots` doubles per rank (send -> recv, device) and the publish of
// recv to the pinned host buffer, then wait (bounded) for the round's sequence word; on any error
// or timeout the communicator is aborted (LFM_E_RCCL / LFM_E_HIP) and nothing is copied out.
int farm_gather_publish(lfm_ctx* ctx, int64_t slots, double* recv) {
  double* dsend = ctx->farm_buf;
  double* drecv = ctx->farm_buf + slots;
  const int64_t count = slots * ctx->nranks;
  unsigned* seq_word = reinterpret_cast<unsigned*>(ctx->farm_pub + count);
  // test instrument: a collective whose peers are late (LFM_DEBUG_FARM_STALL_MS)
  if (const int stall = ctx->farm_stall_ms)
    hipLaunchKernelGGL(stall_kernel, dim3(1), dim3(64), 0, ctx->stream,
                       (unsigned long long)stall * 100000ull);
  const ncclResult_t q = g_rccl.allGather(dsend, drecv, (size_t)slots, ncclFloat64,
                                         (ncclComm_t)ctx->comm, ctx->stream);
  int r = ctx->comm_nb && q == ncclInProgress ? rccl_poll(ctx, (ncclComm_t)ctx->comm, "ncclAllGather")
                                               : rccl_fail(ctx, q, "ncclAllGather");
  if (r) {
    rccl_drop(ctx);
    return r;
  }
  const unsigned seq = ++ctx->farm_seq;
  mark_pending(ctx->farm_pub, count);
  hipLaunchKernelGGL(farm_publish_kernel, dim3(1), dim3(64), 0, ctx->stream, drecv, count,
                     ctx->farm_pub, seq_word, seq);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    rccl_drop(ctx);
    return hip_fail(ctx, e, "farm publish");
  }
  return farm_wait(ctx, seq_word, seq, count, recv);
}

// The host's side of a device-side round: wait (bounded) for the publish kernel's sequence word,
// then copy the gathered slots out; on a fault or timeout the communicator is aborted.
int farm_wait(lfm_ctx* ctx, const unsigned* seq_word, unsigned seq, int64_t count, double* recv) {
  hipError_t e;
  // one bounded wait for the whole chain (kernel, collective, publish): the sequence word — a
  // tight spin for the first 2 ms (a round takes tens of microseconds), then the stream is
  // polled between backed-off checks, so a fault surfaces instead of running out the bound
  const double end = mono_s() + rccl_timeout_s(ctx);
  const Backoff bo;
  const auto t_spin = std::chrono::steady_clock::now() + std::chrono::milliseconds(2);
  // published: the sequence word AND every slot (each marked RESULT_PENDING before the round;
  // no reliance on the order in which the slots' and the word's writes reach host memory)
  auto published = [&] {
    return __atomic_load_n(seq_word, __ATOMIC_ACQUIRE) == seq && all_landed(ctx->farm_pub, count);
  };
  while (!published() && std::chrono::steady_clock::now() < t_spin) __builtin_ia32_pause();
  while (!published()) {
    e = hipStreamQuery(ctx->stream);
    if (e != hipSuccess && e != hipErrorNotReady) {
      rccl_drop(ctx);
      return hip_fail(ctx, e, "farm round");
    }
    if (e == hipSuccess && !published()) {
      rccl_drop(ctx);
      return set_err(ctx, LFM_E_HIP, "farm round: the stream drained without publishing");
    }
    const double now = mono_s();
    if (now > end) {
      char waited[64];
      std::snprintf(waited, sizeof(waited), " after %.2f s", now - bo.t0);
      rccl_drop(ctx);
      return set_err(ctx, LFM_E_RCCL, std::string("farm round: timed out") + waited +
                                          " (a peer rank did not arrive)");
    }
    bo.pause();
  }
  std::memcpy(recv, ctx->farm_pub, (size_t)count * 8);
  return LFM_OK;
}

// The round's publish value when it is replayed from the captured graph (a graph's kernel
// arguments are fixed): the host clears the word before each replay. The enqueued path counts
// from 1 and never reaches it.
constexpr unsigned FARM_GRAPH_SEQ = 0xFFFFFFFFu;

// Capture one device-side round — the padding memset (slots > nprob), the batch's MLL kernel
// reading its hyperparameters from the batch's pinned buffer, ncclAllGather, the publish kernel —
// as a graph, so a round costs one graph launch instead of three enqueues and RCCL's host-side
// enqueue of the collective (which left the GPU idle between the kernel and the collective).
// Returns LFM_OK with ctx->farm_exec set, or non-zero when capture is not possible (the caller
// then enqueues; the graph stays off for this context).
int farm_graph_build(lfm_ctx* ctx, lfm_batch* batch, int negative, int64_t slots) {
  farm_graph_reset(ctx);
  small_batch_attrs();
  const int64_t np = batch->nprob;
  double* dsend = ctx->farm_buf;
  double* drecv = ctx->farm_buf + slots;
  const int64_t count = slots * ctx->nranks;
  unsigned* seq_word = reinterpret_cast<unsigned*>(ctx->farm_pub + count);
  int* hst = reinterpret_cast<int*>(batch->hbuf + batch->nhyp + np);
  hipError_t e = hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeRelaxed);
  if (e != hipSuccess) return hip_fail(ctx, e, "farm graph: begin capture");
  int r = LFM_OK;
  if (slots > np)
    e = hipMemsetAsync(dsend + np, 0xFF, (size_t)(slots - np) * 8, ctx->stream);
  if (e == hipSuccess)
    r = launch_small_batch(ctx, batch->dprobs, (int)np, batch->maxn, batch->maxg, batch->gridtab,
                           negative, dsend, hst);
  else
    r = hip_fail(ctx, e, "farm graph: padding");
  // test instrument: a collective whose peers are late (LFM_DEBUG_FARM_STALL_MS), captured too
  if (!r && ctx->farm_stall_ms)
    hipLaunchKernelGGL(stall_kernel, dim3(1), dim3(64), 0, ctx->stream,
                       (unsigned long long)ctx->farm_stall_ms * 100000ull);
  if (!r) {
    const ncclResult_t q = g_rccl.allGather(dsend, drecv, (size_t)slots, ncclFloat64,
                                           (ncclComm_t)ctx->comm, ctx->stream);
    r = ctx->comm_nb && q == ncclInProgress ? rccl_poll(ctx, (ncclComm_t)ctx->comm, "ncclAllGather")
                                            : rccl_fail(ctx, q, "ncclAllGather");
  }
  if (!r) {
    hipLaunchKernelGGL(farm_publish_kernel, dim3(1), dim3(64), 0, ctx->stream, drecv, count,
                       ctx->farm_pub, seq_word, FARM_GRAPH_SEQ);
    r = hip_fail(ctx, hipGetLastError(), "farm graph: publish");
  }
  hipGraph_t graph = nullptr;
  e = hipStreamEndCapture(ctx->stream, &graph);
  if (!r && e != hipSuccess) r = hip_fail(ctx, e, "farm graph: end capture");
  if (!r) {
    e = hipGraphInstantiate(&ctx->farm_exec, graph, nullptr, nullptr, 0);
    if (e != hipSuccess) {
      ctx->farm_exec = nullptr;
      r = hip_fail(ctx, e, "farm graph: instantiate");
    }
  }
  if (graph) hipGraphDestroy(graph);
  (void)hipGetLastError();
  if (r) {
    farm_graph_reset(ctx);
    return r;
  }
  ctx->farm_exec_batch = batch->id;
  ctx->farm_exec_slots = slots;
  ctx->farm_exec_neg = negative;
  ctx->farm_exec_gen = ctx->comm_gen;
  return LFM_OK;
}
}  // namespace

extern "C" {

int lfm_farm_batch_mll_f64(lfm_ctx* ctx, lfm_batch* batch, const double* hyp, int negative,
                           int64_t slots, double* recv, int* status) {
  if (!ctx) return LFM_E_ARG;
  if (!batch || !hyp || !recv || slots < batch->nprob || slots < 1)
    return set_err(ctx, LFM_E_ARG, "bad farm round arguments (slots >= nprob >= 1)");
  if (batch->device != ctx->device) return set_err(ctx, LFM_E_ARG, "batch of another device");
  if (!ctx->comm) return set_err(ctx, LFM_E_STATE, "farm not initialised");
  DeviceGuard g(ctx->device);
  int r = farm_drain_stale(ctx);
  if (!r) r = farm_buffers(ctx, (size_t)slots);
  if (r) return r;
  // replayed from the captured graph (not while profiling: its events want the enqueued launches)
  if (ctx->farm_graph_on && !ctx->prof) {
    if (!ctx->farm_exec || ctx->farm_exec_batch != batch->id || ctx->farm_exec_slots != slots ||
        ctx->farm_exec_neg != negative || ctx->farm_exec_gen != ctx->comm_gen) {
      // capture not possible here: enqueue from now on (an error of the collective itself
      // surfaces again on the enqueued path below)
      if (farm_graph_build(ctx, batch, negative, slots)) ctx->farm_graph_on = false;
    }
    if (ctx->farm_exec) {
      const int64_t np = batch->nprob, count = slots * ctx->nranks;
      std::memcpy(batch->hbuf, hyp, (size_t)batch->nhyp * 8);
      int* hst = reinterpret_cast<int*>(batch->hbuf + batch->nhyp + np);
      for (int64_t q = 0; q < np; ++q) hst[q] = -1;
      unsigned* seq_word = reinterpret_cast<unsigned*>(ctx->farm_pub + count);
      mark_pending(ctx->farm_pub, count);
      __atomic_store_n(seq_word, 0u, __ATOMIC_RELEASE);
      hipError_t e = hipGraphLaunch(ctx->farm_exec, ctx->stream);
      if (e != hipSuccess) {
        rccl_drop(ctx);
        return hip_fail(ctx, e, "farm graph launch");
      }
      hipEventRecord(batch->done, ctx->stream);
      r = farm_wait(ctx, seq_word, FARM_GRAPH_SEQ, count, recv);
      if (r) return r;
      return batch_status(ctx, batch, status);
    }
  }
  // this rank's padding slots: NaN (all-ones bytes), then the kernel writes its nprob slots
  if (slots > batch->nprob) {
    const hipError_t e = hipMemsetAsync(ctx->farm_buf + batch->nprob, 0xFF,
                                        (size_t)(slots - batch->nprob) * 8, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "farm round: padding slots");
  }
  r = batch_launch(ctx, batch, hyp, negative, ctx->farm_buf);
  if (r) return r;
  r = farm_gather_publish(ctx, slots, recv);
  if (r) return r;
  // the statuses landed before the kernel retired, and the kernel before the collective
  return batch_status(ctx, batch, status);
}

int lfm_farm_allgather_f64(lfm_ctx* ctx, const double* send, int64_t count, double* recv) {
  if (!ctx || !send || !recv || count < 1) return LFM_E_ARG;
  if (!ctx->comm) return set_err(ctx, LFM_E_STATE, "farm not initialised");
  DeviceGuard g(ctx->device);
  int rs = farm_drain_stale(ctx);
  if (rs) return rs;
  const size_t in = (size_t)count * 8, out = in * ctx->nranks;
  const double* before = ctx->farm_buf;
  int r = ensure(ctx, (void**)&ctx->farm_buf, &ctx->farm_bytes, in + out);
  if (r) return r;
  // the captured farm round holds the old device buffer's addresses: forget it
  if (ctx->farm_buf != before) farm_graph_reset(ctx);
  // host side through a pinned buffer of the farm's own: every copy is truly asynchronous (a
  // copy into pageable memory would block past the deadline below), and a copy a timed-out call
  // leaves queued can only ever write into this buffer — never the caller's, never the staging
  // other calls use
  if (!ctx->farm_h || ctx->farm_h_bytes < in + out) {
    if (ctx->farm_h) {
      hipStreamSynchronize(ctx->stream);
      hipHostFree(ctx->farm_h);
      ctx->farm_h = nullptr;
    }
    hipError_t e = hipHostMalloc((void**)&ctx->farm_h, in + out, hipHostMallocDefault);
    if (e != hipSuccess) return hip_fail(ctx, e, "farm staging buffer");
    ctx->farm_h_bytes = in + out;
  }
  double* hsend = ctx->farm_h;
  double* hrecv = ctx->farm_h + count;
  double* dsend = ctx->farm_buf;
  double* drecv = ctx->farm_buf + count;
  std::memcpy(hsend, send, in);
  hipError_t e = hipMemcpyAsync(dsend, hsend, in, hipMemcpyHostToDevice, ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "farm upload");
  // test instrument: a collective whose peers are late, stood in for by a kernel that holds
  // the stream for LFM_DEBUG_FARM_STALL_MS (the one-GPU box cannot host a second rank)
  if (const int stall = ctx->farm_stall_ms) {
    hipLaunchKernelGGL(stall_kernel, dim3(1), dim3(64), 0, ctx->stream,
                       (unsigned long long)stall * 100000ull);
  }
  const ncclResult_t q = g_rccl.allGather(dsend, drecv, (size_t)count, ncclFloat64,
                                         (ncclComm_t)ctx->comm, ctx->stream);
  if (ctx->comm_nb && q == ncclInProgress) r = rccl_poll(ctx, (ncclComm_t)ctx->comm, "ncclAllGather");
  else r = rccl_fail(ctx, q, "ncclAllGather");
  if (!r) {
    e = hipMemcpyAsync(hrecv, drecv, out, hipMemcpyDeviceToHost, ctx->stream);
    if (e != hipSuccess) r = hip_fail(ctx, e, "farm download");
  }
  // one bounded wait for the collective and the copy behind it (the latency-bound exchange has
  // a single synchronisation point); a blocking communicator waits unbounded, as RCCL would
  if (!r) r = ctx->comm_nb ? rccl_stream_wait(ctx, "ncclAllGather") : finish(ctx);
  if (r) {
    rccl_drop(ctx);
    return r;
  }
  std::memcpy(recv, hrecv, out);
  return LFM_OK;
}

int lfm_farm_destroy(lfm_ctx* ctx) {
  if (!ctx) return LFM_E_ARG;
  farm_graph_reset(ctx);
  if (ctx->farm_exec_old && hipStreamQuery(ctx->stream) == hipSuccess) {
    hipGraphExecDestroy(ctx->farm_exec_old);
    ctx->farm_exec_old = nullptr;
  }
  if (ctx->comm && g_rccl.commDestroy) g_rccl.commDestroy((ncclComm_t)ctx->comm);
  ctx->comm = nullptr;
  ctx->nranks = 0;
  ctx->rank = -1;
  return LFM_OK;
}

}  // extern "C"
