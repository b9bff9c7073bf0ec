// One-wave latency chains behind the small kernels' per-column step (lfm_small.hip): cycles per
// iteration (s_memtime) of a dependent chain through
//   0 ds_write_b64 -> ds_read_b64 of another lane's slot -> v_add_f64 (the column round trip)
//   1 variant 0 plus 15 ds_read2_b64 of the column issued behind the dependent read
//   2 variant 1 with the reads waited on before the next store (the factor's shape)
//   3 v_readlane_b32 x 2 -> v_rcp_f64 -> two Newton steps (the pivot's reciprocal)
//   4 v_fma_f64 chain, 8 dependent
//   5 variant 2 plus 30 independent v_fma_f64 (the window update) after the reads
//   6 variant 2 with the column as 15 ds_read_b128 (16-B aligned)
//   7 variant 6 with 8 ds_read_b128 (half the column: the two-lane rows)
// Build: hipcc -O3 --offload-arch=gfx950 scripts/ubench/lds_chain.hip -o scripts/ubench/lds_chain
#include <hip/hip_runtime.h>
#include <cstdio>

template <int V>
__global__ __launch_bounds__(64) void chain(double* out, unsigned long long* cyc, int iters) {
  __shared__ __attribute__((aligned(16))) double buf[256];
  const int l = threadIdx.x;
  buf[l] = 1.0 + l;
  buf[64 + l] = 0.0;
  __syncthreads();
  double x = 1.0 + 1e-3 * l, acc[32];
  for (int q = 0; q < 32; ++q) acc[q] = q;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int it = 0; it < iters; ++it) {
    if constexpr (V >= 6) {
      using dbl2 = double __attribute__((ext_vector_type(2)));
      constexpr int NR = V == 6 ? 15 : 8;
      buf[l] = x;
      asm volatile("" ::: "memory");
      const int k = it & 31;
      double y = buf[k];
      dbl2 col[15];
      const dbl2* src = reinterpret_cast<const dbl2*>(buf + 2 * ((k + 1) >> 1));
#pragma unroll
      for (int q = 0; q < NR; ++q) col[q] = src[q];
      __builtin_amdgcn_sched_barrier(0);
      x = x * 0.5 + y * 1e-9;
#pragma unroll
      for (int q = 0; q < NR; ++q) asm volatile("" : "+v"(col[q]));
#pragma unroll
      for (int q = 0; q < NR; ++q) acc[q] += col[q].x + col[q].y;
    } else if constexpr (V <= 2 || V == 5) {
      buf[l] = x;
      asm volatile("" ::: "memory");
      const int k = it & 31;
      double y = buf[k];
      double col[30];
      if constexpr (V >= 1) {
#pragma unroll
        for (int q = 0; q < 30; ++q) col[q] = buf[k + 1 + q];
      }
      __builtin_amdgcn_sched_barrier(0);
      x = x * 0.5 + y * 1e-9;
      if constexpr (V >= 2) {
#pragma unroll
        for (int q = 0; q < 30; ++q) asm volatile("" : "+v"(col[q]));
      }
      if constexpr (V == 5) {
#pragma unroll
        for (int q = 0; q < 30; ++q) acc[q] = fma(-x, col[q], acc[q + 1]);
      } else if constexpr (V >= 1) {
#pragma unroll
        for (int q = 0; q < 30; ++q) acc[q] += col[q];
      }
    } else if constexpr (V == 3) {
      const int lo = __builtin_amdgcn_readlane((int)__double2loint(x), it & 63);
      const int hi = __builtin_amdgcn_readlane((int)__double2hiint(x), it & 63);
      const double d = __hiloint2double(hi, lo) + 1.0;
      double v = __builtin_amdgcn_rcp(d);
      v = fma(v, fma(-d, v, 1.0), v);
      v = fma(v, fma(-d, v, 1.0), v);
      x = 0.5 * x + v * 1e-9;
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) x = fma(x, 0.999, 1e-9);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = x;
  for (int q = 0; q < 32; ++q) s += acc[q];
  out[l] = s;
  if (l == 0) cyc[0] = t1 - t0;
}

int main() {
  double* out;
  unsigned long long* cyc;
  if (hipMalloc(&out, 64 * sizeof(double)) != hipSuccess) return 1;
  if (hipMalloc(&cyc, sizeof(unsigned long long)) != hipSuccess) return 1;
  const int iters = 4096;
  const char* names[] = {"write -> dependent read -> add (round trip)",
                         "  + 15 ds_read2_b64 of the column behind it",
                         "  + those reads waited on before the next store",
                         "readlane x2 -> rcp_f64 + 2 Newton",
                         "8 dependent v_fma_f64",
                         "round trip + column reads + 30 v_fma_f64 update",
                         "round trip + 15 ds_read_b128, waited on",
                         "round trip + 8 ds_read_b128, waited on"};
  void (*ks[])(double*, unsigned long long*, int) = {chain<0>, chain<1>, chain<2>, chain<3>,
                                                     chain<4>, chain<5>, chain<6>, chain<7>};
  for (int v = 0; v < 8; ++v) {
    unsigned long long best = ~0ull;
    for (int rep = 0; rep < 5; ++rep) {
      hipLaunchKernelGGL(ks[v], dim3(1), dim3(64), 0, 0, out, cyc, iters);
      unsigned long long c = 0;
      if (hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost) != hipSuccess) return 1;
      if (c < best) best = c;
    }
    printf("%-52s %7.1f cycles / iteration\n", names[v], (double)best / iters);
  }
  return hipFree(out) != hipSuccess || hipFree(cyc) != hipSuccess;
}
