// lfm_host.cpp — host-only logic of liblfm (lfm_host.h): plain C++, compiled into liblfm.so and
// into the host sanitizer check (tests/native/host_check.cpp).
#include "lfm_host.h"

#include <fcntl.h>
#include <sys/file.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <climits>
#include <cstdio>
#include <cstring>

namespace lfm {

GridLayout detect_grid(const double* x, int64_t n, int64_t G) {
  GridLayout L;
  if (!x || n < 1 || G < 1 || n > INT_MAX || G > INT_MAX) return L;
  const int g0 = gene_index(x[1], (int)G);
  int64_t T = 1;
  while (T < n && gene_index(x[3 * T + 1], (int)G) == g0) ++T;
  if (n % T != 0) return L;
  const int64_t nblk = n / T;
  L.times.resize(T);
  for (int64_t t = 0; t < T; ++t) L.times[t] = x[3 * t];
  L.block_gene.resize(nblk);
  for (int64_t b = 0; b < nblk; ++b) {
    const int gb = gene_index(x[3 * b * T + 1], (int)G);
    L.block_gene[b] = gb;
    for (int64_t t = 0; t < T; ++t) {
      const double* r = x + 3 * (b * T + t);
      if (r[2] != 1.0) return GridLayout();                    // all rows gene rows (flag 1)
      if (gene_index(r[1], (int)G) != gb) return GridLayout(); // one gene per block
      if (std::memcmp(&r[0], &L.times[t], sizeof(double)) != 0) return GridLayout();  // shared
    }
  }
  const double t0 = L.times[0];
  const double dt = T > 1 ? (L.times[T - 1] - t0) / (double)(T - 1) : 0.0;
  double scale = 1.0;
  for (double t : L.times) scale = std::max(scale, std::fabs(t));
  for (int64_t t = 0; t < T; ++t)
    if (!(std::fabs(L.times[t] - (t0 + (double)t * dt)) <= 1e-12 * scale)) return GridLayout();
  L.T = (int)T;
  L.nblk = (int)nblk;
  L.t0 = t0;
  L.dt = dt;
  L.ok = true;
  return L;
}

std::vector<std::pair<int64_t, int>> plan_steps(int64_t nblk, int64_t Mp, int nb, bool bordered,
                                                bool s3, int wbulk, int64_t w4min,
                                                int64_t w2min, int w0) {
  std::vector<std::pair<int64_t, int>> steps;
  for (int64_t k = 0; k < nblk;) {
    const int64_t m = bordered ? Mp + nb : Mp - k * nb;
    int w = 1;
    // the first bulk super-panel stays 4 wide: its chain runs beside the shallow first update
    const int wk = steps.size() == 1 ? 4 : wbulk;
    if (m >= w4min && k + wk <= nblk) w = wk;
    else if (m >= w4min && k + 4 <= nblk) w = 4;
    else if (m >= w2min && k + 2 <= nblk) w = 2;
    if (k == 0 && s3) w = (w0 == 2 && nblk >= 2) ? 2 : 1;
    steps.emplace_back(k, w);
    k += w;
  }
  return steps;
}

void rest_unit_tile(int64_t b, int T, int tj_lo, int Q, int* ti_out, int* tj_out) {
  constexpr int SUB = 2;  // 64-row slabs per 128-row tile
  const int sub = (int)(b % SUB);
  b /= SUB;
  int a = (int)((std::sqrt(8.0 * (double)b + 1.0) - 1.0) * 0.5);
  while ((int64_t)(a + 1) * (a + 2) / 2 <= b) ++a;
  while ((int64_t)a * (a + 1) / 2 > b) --a;
  int tj, ti;
  if (Q > 1) {
    const int R = a / Q, r0 = R * Q, qr = std::min(Q, T - tj_lo - r0);
    const int64_t off = b - (int64_t)r0 * (r0 + 1) / 2;
    const int64_t full = (int64_t)R * qr * Q;
    int lr, lc;
    if (off < full) {
      const int C = (int)(off / (qr * Q)), t = (int)(off % (qr * Q));
      lr = t / Q;
      lc = C * Q + t % Q;
    } else {
      const int d = (int)(off - full);
      lr = (int)((std::sqrt(8.0 * (double)d + 1.0) - 1.0) * 0.5);
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
  *ti_out = ti;
  *tj_out = tj;
}

int64_t helper_units(int kd, int na, int nr, int nt, int wnext, int nb, int cus, int side_cus,
                     double tc, double dmin) {
  if (kd <= 0 || side_cus <= 0 || cus <= side_cus) return 0;
  const double t = 154.0 * kd / 640.0 + 4.0;  // one depth-kd unit, us (step timeline)
  const double o = 0.9;
  const double sm = 4.0 * (cus - side_cus), sh = 4.0 * side_cus;
  const double tall_eq = (double)nt * (wnext + 1) / 2.0 * nb / kd;
  const double units = (double)na + nr + tall_eq;
  const double d0 = units * t / (sm * o);
  if (d0 < dmin) return 0;
  const double x = o * (d0 - tc) / (t * (1.0 / sh + 1.0 / sm));
  return std::max<int64_t>(0, std::min<int64_t>((int64_t)x, nr / 2));
}

int64_t helper_clamp(int64_t hu, int nr, int T, int wn, int lead, int Q) {
  // a rest region of at most 8 tile columns is enumerated on the device as a band, column by
  // column (lfm_chol.hip unit_tile), not as this triangle: no helper there (its tail would be
  // the last columns, lead tiles included)
  if (hu <= 0 || T - wn <= kBandMaxCols) return 0;
  Q = std::max(Q, 1);
  const int64_t r0e = std::min<int64_t>((int64_t)(lead + Q - 1) / Q * Q, (int64_t)T - wn);
  hu = std::min<int64_t>(hu, (int64_t)nr - r0e * (r0e + 1));  // 2 slabs per triangle tile
  if (hu <= 0) return 0;
  for (int64_t b = nr - hu; b < nr; ++b) {
    int ti, tj;
    rest_unit_tile(b, T, wn, Q, &ti, &tj);
    if (ti / 2 < wn + lead && tj < wn + lead) return 0;
  }
  return hu;
}

namespace {
// flock, restarted when a signal interrupts the wait; 0 or the errno of the failure
int flock_retry(int fd, int op) {
  for (;;) {
    if (::flock(fd, op) == 0) return 0;
    if (errno != EINTR) return errno;
  }
}

// flock needs no write access: a file another user created (mode 0666 less their umask) is
// opened read-only rather than dropping to in-process locking
int open_lock_file(const std::string& p) {
  int fd = ::open(p.c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0666);
  if (fd < 0 && errno == EACCES) fd = ::open(p.c_str(), O_RDONLY | O_CLOEXEC);
  return fd;
}
}  // namespace

bool TenancyLock::open(const std::string& path) {
  std::lock_guard<std::mutex> lk(open_mu_);
  if (opened_) return ok_;
  opened_ = true;
  path_ = path;
  if (path.size() < 5 || path.compare(path.size() - 5, 5, ".lock") != 0) return ok_ = false;
  fd_ = open_lock_file(path);
  turn_ = open_lock_file(path.substr(0, path.size() - 5) + ".turn");
  if (fd_ < 0 || turn_ < 0) {
    if (fd_ >= 0) ::close(fd_);
    if (turn_ >= 0) ::close(turn_);
    fd_ = turn_ = -1;
    return ok_ = false;
  }
  return ok_ = true;
}

std::string TenancyLock::path() {
  std::lock_guard<std::mutex> lk(open_mu_);
  return path_;
}

// The first flock failure (ENOLCK on a filesystem without locks, EBADF, ...) turns the
// cross-process part off for good: logged once with the cause, so a later schedule-3 stall
// beside another process can be traced to the missing lock; the in-process lock still holds.
bool TenancyLock::files() const { return fd_ >= 0 && err_.load(std::memory_order_acquire) == 0; }

void TenancyLock::fail(int e, const char* what) {
  int expected = 0;
  if (err_.compare_exchange_strong(expected, e))
    std::fprintf(stderr,
                 "liblfm: flock(%s) on %s failed: %s; the schedule-3 tenancy lock is in-process "
                 "only from now on (another process on this GPU can stall schedule 3)\n",
                 what, path_.c_str(), std::strerror(e));
}

void TenancyLock::lock_exclusive() {
  rw_.lock();
  if (files()) {
    std::lock_guard<std::mutex> tl(turn_mu_);
    // readers arriving from now on wait at the turnstile, then the readers already in drain
    if (int e = flock_retry(turn_, LOCK_EX)) return fail(e, "turnstile, exclusive");
    if (int e = flock_retry(fd_, LOCK_EX)) fail(e, "lock, exclusive");
    else fd_held_ = true;
    if (int e = flock_retry(turn_, LOCK_UN)) fail(e, "turnstile, release");
  }
}

void TenancyLock::unlock_exclusive() {
  if (fd_held_) {
    fd_held_ = false;
    if (int e = flock_retry(fd_, LOCK_UN)) fail(e, "lock, release");
  }
  rw_.unlock();
}

void TenancyLock::lock_shared() {
  rw_.lock_shared();
  if (fd_ < 0) return;
  if (files()) {
    std::lock_guard<std::mutex> tl(turn_mu_);
    // behind any writer waiting in another process
    if (int e = flock_retry(turn_, LOCK_EX)) fail(e, "turnstile, shared");
    else if (int e2 = flock_retry(turn_, LOCK_UN)) fail(e2, "turnstile, release");
  }
  // every shared holder is counted, whatever the file lock's state: the LOCK_SH taken by the
  // first is released by the last (sh_held_), also if a failure turned the files off between
  std::lock_guard<std::mutex> fl(fd_mu_);
  if (readers_++ == 0 && files()) {
    if (int e = flock_retry(fd_, LOCK_SH)) fail(e, "lock, shared");
    else sh_held_ = true;
  }
}

void TenancyLock::unlock_shared() {
  if (fd_ >= 0) {
    std::lock_guard<std::mutex> fl(fd_mu_);
    if (--readers_ == 0 && sh_held_) {
      sh_held_ = false;
      if (int e = flock_retry(fd_, LOCK_UN)) fail(e, "lock, release");
    }
  }
  rw_.unlock_shared();
}

TenancyLock::~TenancyLock() {
  if (fd_ >= 0) ::close(fd_);
  if (turn_ >= 0) ::close(turn_);
}

}  // namespace lfm
