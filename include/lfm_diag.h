/*
 * lfm_diag.h — diagnostics, exported by liblfm_diag.so (dis_project_amd/csrc/lfm_diag.hip),
 * a library of its own beside the product liblfm.so (include/lfm.h), which it links against
 * and whose contexts it takes.
 *
 * Hardware probes (MFMA lane maps and issue rates, the trailing-update kernel alone), phase
 * timestamps of the schedule-3 factor chain and the schedule-3 tenancy state. They back the
 * measurements quoted in DESIGN.md and the layout / pivot / tenancy tests; no product call
 * path loads this library. Same conventions as lfm.h (LFM_OK / LFM_E_* return codes,
 * synchronous at return).
 */
#ifndef LFM_DIAG_H
#define LFM_DIAG_H

#include <stdint.h>

#include "lfm.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Timestamps (s_memrealtime, 100 MHz) of the schedule-3 factorisation: 256 rows of 16
 * chain-phase stamps per super-panel step, then 256 rows of 8 per main-stream step launch s
 * (s's update + the tall solve of s + 1): [0] bitwise NOT of the first unit's start,
 * [1] the last update unit's end, [2] the last tall unit's wait end (the chain's factor
 * landed), [3] the last unit's end, [4] / [5] the sums over the update ('rest') units of
 * their shader-clock (s_memtime) / 100 MHz (s_memrealtime) durations: the in-kernel clock
 * is [4] / [5] x 100 MHz. enable = 1 arms them; enable = 0 copies up to max (<= 256 * 24)
 * values out and disarms. */
int lfm_debug_stamps(lfm_ctx* ctx, int enable, unsigned long long* out, int max);

/* Per-workgroup trace of the schedule-3 step and helper launches. cap > 0 arms it for the next
 * cap workgroups (later launches untraced); cap = 0 copies min(written, max) records of four
 * words out — entry and exit s_memrealtime (100 MHz), HW_ID | XCC_ID << 32, and launch tag
 * << 40 | role << 32 | unit (tag: launch count, bit 23 set on helper launches; role 1 ahead,
 * 2 rest, 3 tall, 0 padding) — stores the count written in *written and disarms. */
int lfm_debug_trace(lfm_ctx* ctx, int64_t cap, unsigned long long* out, int64_t max,
                    int64_t* written);

/* The schedule (1 or 3) the context's last factorisation ran; 0 before the first. A schedule-3
 * context runs schedule 1 for a call while another process holds the device's tenancy lock. */
int lfm_debug_last_schedule(const lfm_ctx* ctx, int* out);

/* The advisory lock file of the context's device (schedule-3 tenancy across processes). */
int lfm_debug_lock_path(const lfm_ctx* ctx, char* buf, int len);

/* The diagonal factor's pivot reciprocal square root (v_rsq_f64 + one Newton step) on x[n]. */
int lfm_probe_rsq(lfm_ctx* ctx, const double* x, int64_t n, double* y);

/* The small-problem kernel's gram entries two ways, for every pair of x[n x 3] (n, num_genes
 * <= 63): out[0, n^2) by the reference restatement kernel_ref, out[n^2, 2 n^2) by the per-row /
 * per-gene tables small_mll_kernel uses for gene-gene pairs (KxxTab, lfm_math.h). */
int lfm_probe_kxx_tab(lfm_ctx* ctx, const double* x, int64_t n, const lfm_hyp* hyp, double* out);

/* Layout probe: D = A(16x4) * B(4x16) on one wave through v_mfma_f64_16x16x4_f64;
 * A, B, D row-major host arrays. */
int lfm_probe_mfma_f64_layout(lfm_ctx* ctx, const double* a, const double* b, double* d);

/* v_mfma_f64_4x4x4_4b_f64 on one wave: per-lane a, b, c [64] -> d[5][64] for
 * (CBSZ, ABID) = (0,0), (2,0), (2,1), (2,2), (2,3). */
int lfm_probe_mfma4_layout(lfm_ctx* ctx, const double* a, const double* b, const double* c,
                           double* d);

/* Throughput of v_mfma_f64_16x16x4_f64 over a grid of nblocks x 256 threads. */
int lfm_probe_mfma_f64(lfm_ctx* ctx, int nblocks, int iters, double* tflops, double* ms);

/* Shader cycles per v_mfma_f64_16x16x4_f64 per wave (8 chains) and the shader clock (MHz)
 * seen by block 0 of an nblocks x 256 grid. */
int lfm_probe_mfma_f64_cycles(lfm_ctx* ctx, int nblocks, int iters, double* cyc_per_mfma,
                              double* mhz);

/* fp64 rate probes (TFLOP/s): which = 0 VALU v_fma_f64, 1 v_mfma_f64_4x4x4_4b_f64,
 * 2 / 3 the 16x16x4 / 4x4x4_4b MFMA on pseudo-random register operands. */
int lfm_probe_rate(lfm_ctx* ctx, int which, int nblocks, int iters, double* tflops);

/* The trailing-update kernel alone (64-row slabs) on a T x T grid of 128-tiles, depth kd:
 * average us per launch. cio bit 0: C tile I/O (else MFMAs only), bit 3: random operands,
 * bit 4: on schedule 3's CU-masked bulk stream, bit 6: the step kernel's rest role (the other
 * bits: lfm_chol.hip probe_update_launch). */
int lfm_probe_syrk(lfm_ctx* ctx, int T, int kd, int cio, int reps, double* us);

#ifdef __cplusplus
}
#endif
#endif /* LFM_DIAG_H */
