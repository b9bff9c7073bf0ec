// Host round trip of one small launch on gfx950: the host launches a one-workgroup kernel and
// spins until the kernel's store of a flag into coherent pinned memory lands — the C5 batch
// call's shape (lfm_batch_mll_f64) without its arithmetic. Variants: the kernel argument size
// (64 B against the 4 KB SmallArgs-sized struct), an event record after the launch and an event
// query before it (batch_prev_ok), and a 15-workgroup grid.
//   hipcc -O2 --offload-arch=gfx950 launch_rt.hip -o launch_rt && ./launch_rt
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

struct Small {
  int* flag;
  int seq;
};
struct Big {
  double pad[496];
  int* flag;
  int seq;
};

__global__ void k_small(Small a) {
  if (threadIdx.x == 0) {
    __threadfence_system();
    a.flag[blockIdx.x] = a.seq;
  }
}
__global__ void k_big(Big a) {
  if (threadIdx.x == 0) {
    __threadfence_system();
    a.flag[blockIdx.x] = a.seq + (int)(a.pad[blockIdx.x] * 0.0);
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int main() {
  int* flag;
  if (hipHostMalloc((void**)&flag, 64 * sizeof(int), hipHostMallocCoherent) != hipSuccess) return 1;
  hipStream_t s;
  hipStreamCreate(&s);
  hipEvent_t ev;
  hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  const int reps = 4000;
  int seq = 0;
  auto run = [&](const char* name, bool big, int grid, bool rec, bool query) {
    std::vector<double> t;
    for (int i = 0; i < reps + 200; ++i) {
      ++seq;
      for (int b = 0; b < grid; ++b) __atomic_store_n(&flag[b], -1, __ATOMIC_RELEASE);
      const double t0 = now_us();
      if (query) (void)hipEventQuery(ev);
      if (big) {
        Big a{};
        a.flag = flag;
        a.seq = seq;
        hipLaunchKernelGGL(k_big, dim3(grid), dim3(256), 0, s, a);
      } else {
        hipLaunchKernelGGL(k_small, dim3(grid), dim3(256), 0, s, Small{flag, seq});
      }
      const double t1 = now_us();
      if (rec) hipEventRecord(ev, s);
      const double t2 = now_us();
      for (int b = 0; b < grid; ++b)
        while (__atomic_load_n(&flag[b], __ATOMIC_ACQUIRE) != seq) __builtin_ia32_pause();
      const double t3 = now_us();
      if (i >= 200) {
        t.push_back(t3 - t0);
        t.push_back(t1 - t0);
        t.push_back(t2 - t1);
      }
    }
    std::vector<double> tot, lau, rc;
    for (size_t k = 0; k < t.size(); k += 3) {
      tot.push_back(t[k]);
      lau.push_back(t[k + 1]);
      rc.push_back(t[k + 2]);
    }
    auto med = [](std::vector<double> v) {
      std::sort(v.begin(), v.end());
      return v[v.size() / 2];
    };
    hipStreamSynchronize(s);
    std::printf("%-40s round trip %6.2f us  (launch call %5.2f, event record %5.2f)\n", name,
                med(tot), med(lau), med(rc));
  };
  for (int pass = 0; pass < 2; ++pass) {
    run("64 B args, 1 WG", false, 1, false, false);
    run("4 KB args, 1 WG", true, 1, false, false);
    run("64 B args, 15 WG", false, 15, false, false);
    run("4 KB args, 15 WG", true, 15, false, false);
    run("4 KB args, 15 WG, +event record", true, 15, true, false);
    run("4 KB args, 15 WG, +record +query", true, 15, true, true);
  }
  hipStreamSynchronize(s);
  hipEventDestroy(ev);
  hipStreamDestroy(s);
  hipHostFree(flag);
  return 0;
}
