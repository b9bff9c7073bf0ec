// host_check.cpp — the host-side code of liblfm (dis_project_amd/csrc/lfm_host.cpp) and the
// C++ oracle (oracle/lfm_cpu.cpp) under AddressSanitizer + UBSan: built and run
// by `make -C tests/native asan` (tests/test_host_asan.py). Exits non-zero on the first failed
// check; the sanitizers abort on any memory / UB error.
#include <fcntl.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "../../dis_project_amd/csrc/lfm_host.h"

extern "C" {
int lfm_cpu_gram(const double* x, int64_t n, int64_t G, const double* D, const double* S,
                 double l, double diag_add, double* K, int64_t ldk, int threads);
int lfm_cpu_gram_rows_f32(const double* x, int64_t n, int64_t G, const double* D,
                          const double* S, double l, double diag_add, const int64_t* rows,
                          int64_t nrows, float* out, int threads);
int64_t lfm_cpu_potrf(double* A, int64_t n, int64_t lda, int threads);
double lfm_cpu_mll(const double* x, const double* y, int64_t n, int64_t G, const double* D,
                   const double* S, const double* B, double l, double obs_stddev, double jitter,
                   int negative, int threads, double* work, double* info);
}

static int failures = 0;
#define CHECK(c, ...)                                     \
  do {                                                    \
    if (!(c)) {                                           \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                  \
      std::fprintf(stderr, "\n");                         \
      if (++failures > 20) std::exit(1);                  \
    }                                                     \
  } while (0)

using namespace lfm;

// every (64-row slab, 128-column tile) of the rest triangle exactly once
static void check_enumeration() {
  int cases = 0;
  for (int Q : {1, 2, 6}) {
    for (int T = 1; T <= 40; ++T) {
      for (int lo = 0; lo < T && lo <= 6; ++lo) {
        const int m = T - lo;
        const int64_t units = (int64_t)m * (m + 1);  // 2 slabs per tile of the m-tile triangle
        std::set<std::pair<int, int>> seen;
        for (int64_t b = 0; b < units; ++b) {
          int ti, tj;
          rest_unit_tile(b, T, lo, Q, &ti, &tj);
          const int tr = ti / 2;
          CHECK(tj >= lo && tj <= tr && tr < T, "Q=%d T=%d lo=%d b=%lld -> (%d,%d)", Q, T, lo,
                (long long)b, ti, tj);
          CHECK(seen.insert({ti, tj}).second, "duplicate unit Q=%d T=%d lo=%d b=%lld", Q, T, lo,
                (long long)b);
        }
        CHECK((int64_t)seen.size() == units, "coverage Q=%d T=%d lo=%d", Q, T, lo);
        ++cases;
      }
    }
  }
  std::printf("enumeration: %d (Q, T, tj_lo) cases bijective\n", cases);
}

// the side-CU helper's tail never holds a lead tile; the cap is the first unit past them
static void check_helper_clamp() {
  std::mt19937_64 rng(7);
  int cases = 0, capped = 0;
  for (int it = 0; it < 4000; ++it) {
    const int Q = (int)(rng() % 2) ? 6 : 1 + (int)(rng() % 4);
    const int T = 2 + (int)(rng() % 130);
    const int wn = 1 + (int)(rng() % 5);
    if (T - wn <= kBandMaxCols) continue;  // band enumeration: no helper (checked below)
    const int lead = 1 + (int)(rng() % 5);
    const int nr = (T - wn) * (T - wn + 1);
    const int64_t want = (int64_t)(rng() % (nr + 1));
    const int64_t hu = helper_clamp(want, nr, T, wn, lead, Q);
    CHECK(hu >= 0 && hu <= want, "hu out of range");
    for (int64_t b = nr - hu; b < nr; ++b) {
      int ti, tj;
      rest_unit_tile(b, T, wn, Q, &ti, &tj);
      CHECK(!(ti / 2 < wn + lead && tj < wn + lead), "lead tile in the helper's tail T=%d wn=%d "
            "lead=%d Q=%d b=%lld", T, wn, lead, Q, (long long)b);
    }
    capped += hu < want;
    ++cases;
  }
  // band-enumerated rest regions (<= 8 tile columns) never get a helper
  for (int T = 2; T <= 40; ++T)
    for (int wn = 1; wn < T && wn <= 5; ++wn)
      if (T - wn <= kBandMaxCols)
        CHECK(helper_clamp((T - wn) * (T - wn + 1) / 2, (T - wn) * (T - wn + 1), T, wn, 1, 6) == 0,
              "band region T=%d wn=%d got a helper", T, wn);
  CHECK(helper_units(640, 100, 5000, 200, 5, 128, 256, 32, 700, 1200) >= 0, "helper_units");
  CHECK(helper_units(640, 100, 5000, 200, 5, 128, 256, 32, 700, 1200) <= 2500, "helper half");
  CHECK(helper_units(640, 0, 10, 0, 5, 128, 256, 32, 700, 1200) == 0, "no helper for short");
  CHECK(helper_units(640, 100, 5000, 200, 5, 128, 256, 0, 700, 1200) == 0, "no side CUs");
  std::printf("helper clamp: %d cases (%d capped)\n", cases, capped);
}

static std::vector<double> grid_x(int G, int T, int R, const std::vector<int>& genes) {
  std::vector<double> x;
  for (int r = 0; r < R; ++r)
    for (int g = 0; g < G; ++g)
      for (int t = 0; t < T; ++t) {
        x.push_back(T > 1 ? 12.0 * t / (T - 1) : 0.0);
        x.push_back((double)genes[g]);
        x.push_back(1.0);
      }
  return x;
}

static void check_detect_grid() {
  std::vector<int> g8 = {0, 1, 2, 3, 4, 5, 6, 7};
  auto x = grid_x(8, 64, 1, g8);
  GridLayout L = detect_grid(x.data(), 8 * 64, 8);
  CHECK(L.ok && L.T == 64 && L.nblk == 8 && L.block_gene[7] == 7, "plain grid");
  auto x3 = grid_x(8, 16, 3, g8);  // replicate-major
  L = detect_grid(x3.data(), 3 * 8 * 16, 8);
  CHECK(L.ok && L.T == 16 && L.nblk == 24 && L.block_gene[8] == 0, "replicates");
  std::vector<int> shuf = {3, 1, 7, 0, 2, 6, 5, 4};
  auto xs = grid_x(8, 32, 1, shuf);
  L = detect_grid(xs.data(), 8 * 32, 8);
  CHECK(L.ok && L.block_gene[0] == 3 && L.block_gene[2] == 7, "shuffled genes");
  // negative / out-of-range / NaN gene indices follow the gather semantics
  std::vector<int> odd = {-1, 0, 9, 1};
  auto xo = grid_x(4, 8, 1, odd);
  L = detect_grid(xo.data(), 32, 4);
  CHECK(L.ok && L.block_gene[0] == 3 && L.block_gene[2] == 3, "wrapped / clamped genes");
  auto xn = x;
  xn[3 * 5 + 2] = 0.0;  // a latent (flag 0) row
  CHECK(!detect_grid(xn.data(), 8 * 64, 8).ok, "flag 0 row");
  xn = x;
  xn[3 * 70] += 1e-3;  // non-shared times in block 1
  CHECK(!detect_grid(xn.data(), 8 * 64, 8).ok, "times differ");
  xn = x;
  xn[3 * 10] = 100.0;  // non-uniform grid
  for (int b = 0; b < 8; ++b) xn[3 * (b * 64 + 10)] = 100.0;
  CHECK(!detect_grid(xn.data(), 8 * 64, 8).ok, "non-uniform");
  CHECK(!detect_grid(x.data(), 8 * 64 - 3, 8).ok, "ragged n");
  xn = x;
  xn[3 * 70 + 1] = std::nan("");  // NaN gathers gene 0: not block 1's gene
  CHECK(!detect_grid(xn.data(), 8 * 64, 8).ok, "NaN gene inside a block");
  xn = x;
  xn[3 * 3 + 1] = std::nan("");  // ... but block 0's
  CHECK(detect_grid(xn.data(), 8 * 64, 8).ok, "NaN gene gathers gene 0");
  CHECK(!detect_grid(nullptr, 0, 8).ok && !detect_grid(x.data(), 0, 8).ok, "empty");
  L = detect_grid(x.data(), 1, 8);
  CHECK(L.ok && L.T == 1 && L.nblk == 1, "single row");
  std::printf("detect_grid: ok\n");
}

static void check_plan() {
  int cases = 0;
  for (bool s3 : {false, true})
    for (bool bordered : {false, true})
      for (int64_t nblk : {1, 2, 3, 5, 9, 17, 33, 65, 129, 130}) {
        const int64_t Mp = nblk * 128;
        auto st = plan_steps(nblk, Mp, 128, bordered, s3, 5, 6144, 5120);
        int64_t k = 0;
        for (size_t i = 0; i < st.size(); ++i) {
          CHECK(st[i].first == k, "contiguous");
          CHECK(st[i].second == 1 || st[i].second == 2 || st[i].second == 4 ||
                    st[i].second == 5, "width");
          if (s3 && i == 0) CHECK(st[i].second == 1, "schedule 3 starts at width 1");
          k += st[i].second;
        }
        CHECK(k == nblk, "covers every block column");
        ++cases;
      }
  std::printf("plan_steps: %d cases\n", cases);
}

static void check_oracle() {
  const int G = 4, T = 24, n = G * T;
  std::vector<int> g4 = {0, 1, 2, 3};
  auto x = grid_x(G, T, 1, g4);
  std::vector<double> D = {0.3, 0.5, 0.7, 0.9}, S = {1.0, 0.8, 1.2, 0.9}, B = {0.05, 0.02, 0.07, 0.1};
  std::vector<double> y(n);
  std::mt19937_64 rng(3);
  std::normal_distribution<double> nd(0, 0.5);
  for (int i = 0; i < n; ++i) y[i] = B[i / T] / D[i / T] + nd(rng);
  std::vector<double> info(8), work((size_t)n * n);
  const double v1 = lfm_cpu_mll(x.data(), y.data(), n, G, D.data(), S.data(), B.data(), 2.5, 1.0,
                                1e-4, 0, 2, nullptr, info.data());
  const double v2 = lfm_cpu_mll(x.data(), y.data(), n, G, D.data(), S.data(), B.data(), 2.5, 1.0,
                                1e-4, 1, 2, work.data(), nullptr);
  CHECK(std::isfinite(v1) && v2 == -v1, "mll / negative");
  std::vector<double> K((size_t)n * n, 0.0);
  CHECK(lfm_cpu_gram(x.data(), n, G, D.data(), S.data(), 2.5, 0.0, K.data(), n, 2) == 0, "gram");
  std::vector<int64_t> rows = {0, 5, n - 1};
  std::vector<float> R(rows.size() * n, 0.0f);
  CHECK(lfm_cpu_gram_rows_f32(x.data(), n, G, D.data(), S.data(), 2.5, 0.0, rows.data(),
                              (int64_t)rows.size(), R.data(), 2) == 0, "gram rows");
  for (size_t q = 0; q < rows.size(); ++q)
    for (int64_t j = 0; j <= rows[q]; ++j)
      CHECK(R[q * n + j] == (float)K[rows[q] * n + j], "rows vs gram");
  int64_t bad = n;
  CHECK(lfm_cpu_gram_rows_f32(x.data(), n, G, D.data(), S.data(), 2.5, 0.0, &bad, 1, R.data(),
                              1) == 1, "row out of range refused");
  for (int i = 0; i < n; ++i) K[(size_t)i * n + i] += 1.0;
  CHECK(lfm_cpu_potrf(K.data(), n, n, 2) == -1, "potrf of K + I");
  std::printf("oracle: mll %.10f\n", v1);
}

// The device tenancy lock (TenancyLock, lfm_api.hip DeviceTenancy). Two objects on one path
// stand for two processes (flock is per open file description).
static void check_tenancy() {
  using clk = std::chrono::steady_clock;
  auto ms_since = [](clk::time_point t) {
    return std::chrono::duration<double, std::milli>(clk::now() - t).count();
  };
  char dir[] = "/tmp/lfm_tenancy_XXXXXX";
  CHECK(mkdtemp(dir) != nullptr, "mkdtemp");
  const std::string path = std::string(dir) + "/lfm_gpu_test.lock";
  TenancyLock a, b;
  CHECK(a.open(path) && b.open(path), "open");
  CHECK(a.path() == path, "path");
  TenancyLock bad;
  CHECK(!bad.open(std::string(dir) + "/no_suffix"), "a path without .lock is refused");

  // exclusive: mutual exclusion over threads
  {
    int counter = 0;
    std::vector<std::thread> ts;
    for (int t = 0; t < 4; ++t)
      ts.emplace_back([&] {
        for (int i = 0; i < 2000; ++i) {
          a.lock_exclusive();
          const int v = counter;
          counter = v + 1;
          a.unlock_exclusive();
        }
      });
    for (auto& t : ts) t.join();
    CHECK(counter == 8000, "exclusive sections overlapped: %d", counter);
  }
  // shared: two readers inside at once
  {
    std::atomic<int> inside{0};
    std::atomic<bool> both{false};
    auto reader = [&] {
      a.lock_shared();
      ++inside;
      const auto t0 = clk::now();
      while (inside.load() < 2 && ms_since(t0) < 2000) std::this_thread::yield();
      if (inside.load() == 2) both = true;
      a.unlock_shared();
    };
    std::thread r1(reader), r2(reader);
    r1.join();
    r2.join();
    CHECK(both.load(), "two shared holders were not admitted together");
  }
  // another "process" holding it exclusively: a shared request waits for the release
  {
    std::atomic<bool> held{false};
    std::thread w([&] {
      b.lock_exclusive();
      held = true;
      std::this_thread::sleep_for(std::chrono::milliseconds(200));
      b.unlock_exclusive();
    });
    while (!held.load()) std::this_thread::yield();
    const auto t0 = clk::now();
    a.lock_shared();
    const double waited = ms_since(t0);
    a.unlock_shared();
    w.join();
    CHECK(waited >= 150.0, "shared request did not wait for the other writer (%.1f ms)", waited);
  }
  // turnstile: while a writer of another "process" waits for this process's reader, a second
  // reader of this process queues behind the writer instead of joining the first reader
  {
    std::atomic<bool> r1_in{false}, w_waiting{false};
    std::atomic<double> w_at{0.0}, r2_at{0.0};
    const auto t0 = clk::now();
    std::thread r1([&] {
      a.lock_shared();
      r1_in = true;
      std::this_thread::sleep_for(std::chrono::milliseconds(300));
      a.unlock_shared();
    });
    while (!r1_in.load()) std::this_thread::yield();
    std::thread w([&] {
      w_waiting = true;
      b.lock_exclusive();
      w_at = ms_since(t0);
      std::this_thread::sleep_for(std::chrono::milliseconds(100));
      b.unlock_exclusive();
    });
    while (!w_waiting.load()) std::this_thread::yield();
    std::this_thread::sleep_for(std::chrono::milliseconds(80));  // the writer is queued now
    std::thread r2([&] {
      a.lock_shared();
      r2_at = ms_since(t0);
      a.unlock_shared();
    });
    r1.join();
    w.join();
    r2.join();
    CHECK(w_at.load() >= 250.0, "writer got in before the reader left (%.1f ms)", w_at.load());
    CHECK(r2_at.load() >= w_at.load() + 80.0,
          "second reader overtook the waiting writer (writer %.1f, reader %.1f ms)", w_at.load(),
          r2_at.load());
  }
  // a flock failure (here EBADF: the lock file's descriptor swapped for an O_PATH one, which
  // flock refuses) is recorded, not ignored: the lock turns in-process only and says so once,
  // and the in-process part still excludes
  {
    const std::string p2 = std::string(dir) + "/lfm_gpu_fail.lock";
    TenancyLock c;
    CHECK(c.open(p2), "open p2");
    int lock_fd = -1;
    for (int fd = 0; fd < 1024; ++fd) {
      char link[64], target[512];
      std::snprintf(link, sizeof(link), "/proc/self/fd/%d", fd);
      const ssize_t k = readlink(link, target, sizeof(target) - 1);
      if (k <= 0) continue;
      target[k] = 0;
      if (p2 == target) lock_fd = fd;
    }
    CHECK(lock_fd >= 0, "lock file descriptor not found");
    const int op = ::open(p2.c_str(), O_PATH | O_CLOEXEC);
    CHECK(op >= 0 && dup2(op, lock_fd) == lock_fd, "dup2 O_PATH");
    ::close(op);
    CHECK(c.error() == 0, "no error before the first lock");
    c.lock_exclusive();
    CHECK(c.error() == EBADF, "flock failure not recorded (%d)", c.error());
    c.unlock_exclusive();
    int counter = 0;
    std::vector<std::thread> ts;
    for (int t = 0; t < 4; ++t)
      ts.emplace_back([&] {
        for (int i = 0; i < 500; ++i) {
          if (i & 1) {
            c.lock_shared();
            c.unlock_shared();
          }
          c.lock_exclusive();
          const int v = counter;
          counter = v + 1;
          c.unlock_exclusive();
        }
      });
    for (auto& t : ts) t.join();
    CHECK(counter == 2000, "in-process exclusion lost after the flock failure: %d", counter);
    unlink(p2.c_str());
    unlink((p2.substr(0, p2.size() - 5) + ".turn").c_str());
  }
  std::string turn = path.substr(0, path.size() - 5) + ".turn";
  unlink(path.c_str());
  unlink(turn.c_str());
  rmdir(dir);
  std::printf("tenancy lock: ok\n");
}

int main() {
  check_tenancy();
  check_enumeration();
  check_helper_clamp();
  check_detect_grid();
  check_plan();
  check_oracle();
  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::printf("host_check: all passed\n");
  return 0;
}
