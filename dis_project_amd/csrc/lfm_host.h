// lfm_host.h — host-only logic of liblfm: x-layout detection, the factorisation's step plan,
// the host mirror of the trailing update's unit enumeration and the side-CU helper's sizing.
// Plain C++ (no HIP types), so lfm_host.cpp also builds into the host sanitizer check
// (tests/native, `make -C tests/native asan`) with g++ -fsanitize=address,undefined.
#pragma once

#include <atomic>
#include <cmath>
#include <cstdint>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <utility>
#include <vector>

#if defined(__HIPCC__)
#define LFM_HD __host__ __device__
#else
#define LFM_HD
#endif

namespace lfm {

// JAX gather semantics for a gene index stored as a float: trunc toward zero, negative wraps
// by +G, clamp to [0, G - 1] (NaN -> 0).
LFM_HD inline int gene_index(double g, int G) {
  double tg = trunc(g);
  if (tg < 0) tg += (double)G;
  if (!(tg >= 0)) tg = 0;  // also catches NaN
  if (tg > (double)(G - 1)) tg = (double)(G - 1);
  return (int)tg;
}
// int(flag) as the reference's switches read it (trunc; NaN -> 0; saturated)
LFM_HD inline long long flag_int(double f) {
  double tf = trunc(f);
  if (!(tf == tf)) return 0;
  if (tf > 4e18) tf = 4e18;
  if (tf < -4e18) tf = -4e18;
  return (long long)tf;
}

// Structure of x detected on the host: rows come in blocks of T consecutive rows that share
// one uniform time vector t[tau] = t0 + tau*dt, one gene index per block and flag 1 — the
// layout dataset_3d (src/dataset.py:358-399) produces.
struct GridLayout {
  bool ok = false;
  int T = 0;          // timepoints per block
  int nblk = 0;       // number of blocks (= n / T)
  double t0 = 0, dt = 0;
  std::vector<double> times;   // [T]  the actual time values of block 0
  std::vector<int> block_gene; // [nblk] clamped gene index per block
};

GridLayout detect_grid(const double* x, int64_t n, int64_t G);

// Super-panel plan of a blocked factorisation over nblk block columns of width nb: (first
// block column, width in block columns) per step. Width wbulk (the first bulk step 4) while
// the trailing matrix has >= w4min rows, 4 if wbulk does not fit, 2 down to w2min rows, else
// 1; schedule 3 starts with a super-panel of w0 (1 or 2) columns. Bordered (the gradient's
// inverse): the trailing window is a constant Mp + nb rows.
std::vector<std::pair<int64_t, int>> plan_steps(int64_t nblk, int64_t Mp, int nb, bool bordered,
                                                bool s3, int wbulk, int64_t w4min,
                                                int64_t w2min, int w0 = 1);

// Rest regions of at most this many tile columns are enumerated as bands (column by column),
// wider ones as the supertiled triangle below (lfm_chol.hip unit_tile).
constexpr int kBandMaxCols = 8;

// Host mirror of the step kernel's rest-triangle enumeration (64-row slabs x 128-column tiles,
// Q x Q supertiles; lfm_chol.hip syrk_unit): unit b -> (64-row slab ti, 128-column tile tj)
// relative to the trailing matrix, tile columns [tj_lo, T).
void rest_unit_tile(int64_t b, int T, int tj_lo, int Q, int* ti_out, int* tj_out);

// The side-CU helper's share of a step's rest units: the main launch of U unit-equivalents
// takes D0 = U t / (S_m o) alone (t: one depth-kd unit, o: slot occupancy, S_m / S_h: the
// main / side stream's workgroup slots); giving x units to the helper, which starts after
// the next chain (tc, us), balances at x t (1 / S_h + 1 / S_m) = o (D0 - tc). No helper for
// D0 < dmin; at most half the rest units.
int64_t helper_units(int kd, int na, int nr, int nt, int wnext, int nb, int cus, int side_cus,
                     double tc, double dmin);

// Caps a helper share hu (the tail [nr - hu, nr) of the enumeration) so that it holds no lead
// tile (tile rows and columns < wn + lead: the inputs of the chain two steps ahead, which only
// the main launch writes through and counts). In the supertile order every unit of triangle
// rows < lead precedes the first unit of supertile row ceil(lead / Q). Returns 0 if the
// enumeration mirror still finds a lead tile in the tail, and for band-enumerated regions
// (T - wn <= kBandMaxCols).
int64_t helper_clamp(int64_t hu, int nr, int T, int wn, int lead, int Q);

// Readers-writer lock over one GPU's library work (lfm_api.hip DeviceTenancy: a schedule-3
// factorisation exclusive, all other GPU work shared). In-process a std::shared_mutex; across
// processes flock on `path` (LOCK_EX / LOCK_SH; the process's shared hold is counted over its
// threads, taken by the first reader and dropped by the last) behind a turnstile file (`path`
// with ".turn" for ".lock"): a writer holds the turnstile while it waits for the readers to
// drain, and every reader passes through it first, so a stream of readers, of this process or
// another, cannot starve a writer. flock is per open file description, so two TenancyLock
// objects on one path behave like two processes. Waits block; nothing is held while waiting on
// anything but these locks.
class TenancyLock {
 public:
  // Opens (creating) the lock and turnstile files once; false: unavailable (the lock is then
  // in-process only). Thread-safe; later calls return the first result.
  bool open(const std::string& path);
  void lock_exclusive();
  void unlock_exclusive();
  void lock_shared();
  void unlock_shared();
  std::string path();
  // 0, or the errno of the first flock failure (the lock is then in-process only)
  int error() const { return err_.load(std::memory_order_acquire); }
  ~TenancyLock();

 private:
  bool files() const;                     // the cross-process part is in use
  void fail(int e, const char* what);     // records (and logs) the first flock failure
  std::atomic<int> err_{0};
  bool fd_held_ = false;  // LOCK_EX on fd_ held by this process's exclusive holder
  bool sh_held_ = false;  // LOCK_SH on fd_ held for this process's shared holders (fd_mu_)
  std::shared_mutex rw_;  // in-process readers-writer lock
  std::mutex turn_mu_;    // this process's threads at the turnstile, one at a time
  std::mutex fd_mu_;      // readers_ and the flock state of fd_
  std::mutex open_mu_;
  int readers_ = 0;       // this process's shared holders (LOCK_SH held while > 0)
  int fd_ = -1, turn_ = -1;
  bool opened_ = false, ok_ = false;
  std::string path_;
};

}  // namespace lfm
