// Four-wave column step (a sketch of the small factor with the window split over the waves):
// per iteration one half-wave stores its 32 entries into a parity buffer, a workgroup barrier,
// then every thread reads the pivot, its row's entry and its slice's 4 entries, forms the
// multiplier through v_rcp_f64 + 2 Newton steps and updates 4 slots. Cycles per iteration.
// Build: hipcc -O3 --offload-arch=gfx950 scripts/ubench/quad_col.hip -o scripts/ubench/quad_col
#include <hip/hip_runtime.h>
#include <cstdio>

template <int WAVES>
__global__ __launch_bounds__(256) void quad(double* out, unsigned long long* cyc, int iters) {
  __shared__ __attribute__((aligned(16))) double ub[2][64];
  const int t = threadIdx.x, i = t & 31, s = t >> 5;
  double a[4] = {1.0 + i, 2.0, 3.0, 4.0};
  if (t < 128) ub[t >> 6][t & 63] = 1.0 + (t & 31);
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int c = 0; c < iters; ++c) {
    const int p = c & 1, so = (c >> 2) & (2 * WAVES - 1);
    if (s == so) ub[p][i] = 1.0 + 1e-9 * a[c & 3];
    __syncthreads();
    const double d = ub[p][c & 31], ui = ub[p][i];
    using dbl2 = double __attribute__((ext_vector_type(2)));
    const dbl2 u01 = *reinterpret_cast<const dbl2*>(&ub[p][(4 * s) & 31]);
    const dbl2 u23 = *reinterpret_cast<const dbl2*>(&ub[p][((4 * s) & 31) + 2]);
    double v = __builtin_amdgcn_rcp(d);
    v = fma(v, fma(-d, v, 1.0), v);
    v = fma(v, fma(-d, v, 1.0), v);
    const double l = ui * v * 1e-3;
    a[0] = fma(-l, u01.x, a[0]);
    a[1] = fma(-l, u01.y, a[1]);
    a[2] = fma(-l, u23.x, a[2]);
    a[3] = fma(-l, u23.y, a[3]);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[t] = a[0] + a[1] + a[2] + a[3];
  if (t == 0) cyc[0] = t1 - t0;
}

int main() {
  double* out;
  unsigned long long* cyc;
  if (hipMalloc(&out, 256 * sizeof(double)) != hipSuccess) return 1;
  if (hipMalloc(&cyc, sizeof(unsigned long long)) != hipSuccess) return 1;
  const int iters = 4096;
  for (int rep = 0; rep < 2; ++rep) {
    for (int w = 1; w <= 4; w *= 2) {
      unsigned long long best = ~0ull;
      for (int k = 0; k < 5; ++k) {
        if (w == 1) hipLaunchKernelGGL(quad<1>, dim3(1), dim3(64), 0, 0, out, cyc, iters);
        if (w == 2) hipLaunchKernelGGL(quad<2>, dim3(1), dim3(128), 0, 0, out, cyc, iters);
        if (w == 4) hipLaunchKernelGGL(quad<4>, dim3(1), dim3(256), 0, 0, out, cyc, iters);
        unsigned long long c = 0;
        if (hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost) != hipSuccess) return 1;
        if (c < best) best = c;
      }
      printf("%d wave(s): store, barrier, 4 reads, rcp + 2 Newton, 4 fma: %6.1f cycles / column\n", w,
             (double)best / iters);
    }
  }
  return hipFree(out) != hipSuccess || hipFree(cyc) != hipSuccess;
}
