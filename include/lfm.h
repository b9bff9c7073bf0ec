/*
 * lfm.h — C-ABI of the MI355X-native SIM latent-force-model hot path.
 *
 * This is the drop-in boundary for the GPJax hot path of wejpurvis/DIS_project:
 * the SIM multi-output covariance (src/model.py:152-414) and the Cholesky-based
 * log marginal likelihood (src/objectives.py:21-78 -> gpjax 0.8.2
 * GaussianDistribution.log_prob). The reference is pure Python/JAX and has no
 * FFI of its own; each entry point below names the reference interface it
 * replaces. Plain pointers and sizes only (no framework types).
 *
 * Conventions
 *   - x arrays are N x 3 row-major fp64: (time, gene index, flag), the layout of
 *     dataset_3d (src/dataset.py:358-399).
 *   - All host buffers are owned by the caller and are not retained after return.
 *     Every call is synchronous at return unless its name ends in _async.
 *   - Device workspace (the Mp x Mp factor, tables, scratch) is owned by the ctx,
 *     grown on demand and reused. A ctx is bound to one device and is NOT
 *     thread-safe: create one ctx per device per host thread.
 *   - Return value: LFM_OK (0) or an LFM_E_* code; lfm_last_error() has the text.
 *     LFM_E_NOT_PD mirrors JAX's silent NaN on a failed Cholesky: the scalar
 *     output is set to NaN and the failing pivot index is in lfm_last_error().
 *     LFM_E_TIMEOUT is NOT a property of the input: a bounded device-side wait of the
 *     factorisation's cross-stream hand-off ran out (e.g. a tool serialised the two
 *     streams' dispatches) and the in-call schedule-1 re-run (lfm_ctx_fallbacks) was
 *     disabled or ran out too. The result is invalid; callers must raise, never map it to NaN.
 *   - Diagnostics (rate / layout probes, phase stamps) are declared in lfm_diag.h.
 */
#ifndef LFM_H
#define LFM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LFM_ABI_VERSION 5

enum {
  LFM_OK = 0,
  LFM_E_ARG = 1,    /* bad shape / pointer / value                        */
  LFM_E_HIP = 2,    /* HIP runtime error (text in lfm_last_error)          */
  LFM_E_NOT_PD = 3, /* Cholesky pivot <= 0 or NaN; scalar result is NaN    */
  LFM_E_OOM = 4,    /* device allocation failed                            */
  LFM_E_RCCL = 5,   /* RCCL not loadable / collective failed               */
  LFM_E_STATE = 6,  /* call out of order (e.g. farm not initialised)       */
  LFM_E_TIMEOUT = 7 /* device-side wait ran out: result invalid (not NaN)  */
};

/* gram / cross-covariance output selection */
enum { LFM_UPLO_FULL = 0, LFM_UPLO_LOWER = 1 };

typedef struct lfm_ctx lfm_ctx;

/*
 * Constrained hyperparameters of ExactLFM (src/model.py:64-121).
 *   true_d / true_s / true_b : [num_genes] decay D, sensitivity S, basal B
 *   l                        : lengthscale (model.py:111-121)
 *   obs_stddev               : observation std-dev; sigma^2 = obs_stddev^2 (objectives.py:66)
 *   jitter                   : static jitter added to the gram diagonal (objectives.py:71)
 * Gene indices read from x[:,1] are truncated toward zero, negative ones wrap by
 * +num_genes and the result is clamped to [0, num_genes-1] (JAX gather semantics).
 */
typedef struct {
  int64_t num_genes;
  const double* true_d;
  const double* true_s;
  const double* true_b;
  double l;
  double obs_stddev;
  double jitter;
} lfm_hyp;

/* One independent marginal-likelihood problem of a batch (restart / ablation). */
typedef struct {
  const double* x; /* [n x 3] host */
  const double* y; /* [n]     host */
  int64_t n;
  lfm_hyp hyp;
} lfm_problem;

/* Per-kernel-class timing, filled when profiling is on (HIP events on the stream each
 * launch runs on). flops / bytes are ALGORITHMIC: the blocked Cholesky's work on the
 * unpadded (n + 1)-row augmented matrix (N^3 / 3 over a factorisation), not what the
 * padded tiles issue; issued_flops is the MFMA work the launches actually issue. */
typedef struct {
  char name[32];
  int64_t launches;
  double total_ms;     /* sum of per-launch HIP-event durations              */
  double flops;        /* algorithmic flops over all launches                */
  double bytes;        /* algorithmic HBM bytes over all launches            */
  double issued_flops; /* flops issued (padded tiles, inverse-based solves)  */
} lfm_kstat;

/* ---------------------------------------------------------------- context */
int lfm_abi_version(void);
int lfm_device_count(int* out);
int lfm_ctx_create(int device, lfm_ctx** out);
void lfm_ctx_destroy(lfm_ctx* ctx);
const char* lfm_last_error(const lfm_ctx* ctx);
int lfm_ctx_synchronize(lfm_ctx* ctx);
/* Block size of the blocked Cholesky: 128 (the only size built; 0 restores it). */
int lfm_ctx_set_block(lfm_ctx* ctx, int nb);
/* Factorisation schedule of this context's MLL / gradient:
 *   3  CU-partitioned stream pair: the factor chain on LFM_SIDE_CUS reserved CUs, the bulk on
 *      the rest. Lowest latency of ONE evaluation. Single tenant: the chain needs all of its
 *      workgroups resident, so a schedule-3 factorisation holds the device's lock exclusively
 *      (threads and processes: a per-device readers-writer lock plus flock on
 *      $TMPDIR/lfm_gpu_<PCI bus id>.lock); other GPU work of the library holds it shared.
 *      Concurrent callers wait their turn; results do not depend on it.
 *   1  look-ahead on every CU. Several schedule-1 contexts driven from separate host threads
 *      share one GPU (shared holders): the throughput mode of a restart farm
 *      (farm.ConcurrentEvaluator).
 *   0  the process default (LFM_SCHED, else 3).
 * Schedule 3 on a context without a CU partition -> LFM_E_ARG. Replaces no reference call:
 * the reference's XLA executable has no schedule (src/objectives.py:43-46 is the whole MLL). */
int lfm_ctx_set_schedule(lfm_ctx* ctx, int schedule);
/* The schedule the next factorisation will run (1 or 3). */
int lfm_ctx_get_schedule(const lfm_ctx* ctx, int* out);
/* Schedule-3 calls of this context (MLL, gradient, log_prob) whose device-side waits ran past
 * their time bound (LFM_DEVICE_WAIT_MS, default 2000: e.g. another tenant of the GPU starved
 * the factor chain's co-resident workgroups) and that were therefore re-run on schedule 1
 * inside the same call. Their results are valid (LFM_OK); lfm_last_error names the stall after
 * such a call. LFM_S3_FALLBACK=0 disables the re-run (the call then returns LFM_E_TIMEOUT).
 * Reference behaviour preserved: trainer.py:126 never fails for scheduling reasons. */
int lfm_ctx_fallbacks(const lfm_ctx* ctx, int64_t* out);

/* --------------------------------------------- ExactLFM surface (model.py) */
/* mean_function (model.py:124-149): out[i] = (B/D)[i / (n / num_genes)] * int(x[i,2]). */
int lfm_mean_function_f64(lfm_ctx* ctx, const double* x, int64_t n, const lfm_hyp* hyp,
                          double* out);

/* cross_covariance(kernel, x, x2) (model.py:372-394): out[i*ldo + j] = kernel(x[i], x2[j]),
 * the flag-switched kernel of model.py:152-195 (kxx / kff / kxf / kfx). */
int lfm_cross_covariance_f64(lfm_ctx* ctx, const double* x, int64_t n, const double* x2,
                             int64_t m, const lfm_hyp* hyp, double* out, int64_t ldo);

/* h(j, k, t1, t2) of model.py:315-365 element-wise over n tuples (gene indices clamped
 * as above); exposes the convolution term on its own for known-answer tests. */
int lfm_h_f64(lfm_ctx* ctx, const lfm_hyp* hyp, const int64_t* j, const int64_t* k,
              const double* t1, const double* t2, int64_t n, double* out);

/* gram(kernel, x) (model.py:396-414) plus diag_add on the diagonal; uplo = LFM_UPLO_FULL
 * writes the dense n x n, LFM_UPLO_LOWER computes only j <= i (the upper part of a host
 * output is zero-filled, of a device output left untouched). */
int lfm_gram_f64(lfm_ctx* ctx, const double* x, int64_t n, const lfm_hyp* hyp, double diag_add,
                 int uplo, double* out, int64_t ldo);
/* fp32 gram (arithmetic and output in fp32; per-gene tables built in fp64). */
int lfm_gram_f32(lfm_ctx* ctx, const double* x, int64_t n, const lfm_hyp* hyp, double diag_add,
                 int uplo, float* out, int64_t ldo);

/* --------------------------------- CustomConjMLL.step (objectives.py:21-78) */
/* out = constant * log N(y; m, K + jitter I + obs_stddev^2 I), constant = -1 if negative.
 * n >= 1 and n % num_genes == 0 (mean_function's broadcast, model.py:145-149), else
 * LFM_E_ARG; the same holds for lfm_mll_batch_f64's problems and lfm_mll_grad_f64. */
int lfm_mll_f64(lfm_ctx* ctx, const double* x, const double* y, int64_t n, const lfm_hyp* hyp,
                int negative, double* out);
/* nprob independent problems; out[p] per problem (NaN where not PD); status[p] optional. */
int lfm_mll_batch_f64(lfm_ctx* ctx, int64_t nprob, const lfm_problem* probs, int negative,
                      double* out, int* status);

/* A batch of small problems registered once and evaluated many times — the replicate x
 * leave-one-gene-out ablation farm of src/notebook.py:33-75, each problem the MLL of
 * src/objectives.py:64-78. x / y of every problem (probs[p].x, .y, .n; n <= 128, n % num_genes
 * == 0) go to HBM here, once; of probs[p].hyp only num_genes is read (it fixes the layout of the
 * packed hyperparameters). The caller's x / y may be freed after the call. A batch belongs to
 * the device of the ctx that created it and, like a ctx, to one host thread at a time (its
 * pinned hyperparameter / result buffer is reused by every call). */
typedef struct lfm_batch lfm_batch;
int lfm_batch_create(lfm_ctx* ctx, int64_t nprob, const lfm_problem* probs, lfm_batch** out);
int lfm_batch_destroy(lfm_batch* batch);
/* Doubles in the packed hyperparameter array: sum_p (3 G_p + 3). */
int lfm_batch_hyp_size(const lfm_batch* batch, int64_t* out);
/* Every problem's MLL (constant -1 if negative) in ONE launch, one workgroup per problem.
 * hyp packed: first, for each problem in order, true_d[G_p] true_s[G_p] true_b[G_p]; then, for
 * each problem in order, l, obs_stddev, jitter. out[p] per problem (NaN where not PD, with
 * status[p] = LFM_E_NOT_PD; status may be NULL); returns LFM_E_NOT_PD if any problem was.
 * Returns once every problem's result has landed in host memory (the kernel may still be
 * retiring: later work on the ctx's stream is ordered after it, lfm_batch_destroy waits for the
 * batch's last launch before it frees, and a fault that launch hits after the return is
 * reported as LFM_E_HIP by the batch's next value / gradient call). */
int lfm_batch_mll_f64(lfm_ctx* ctx, lfm_batch* batch, const double* hyp, int negative,
                      double* out, int* status);
/* Value and gradient of every problem's CustomConjMLL(negative).step in ONE launch, one
 * workgroup per problem — jax.value_and_grad(loss) at src/trainer.py:126 (before the
 * bijectors' chain rule, trainer.py:103), batched over the ablation problems of
 * src/notebook.py:33-75 / the p53 fit of src/main.py:59. Every problem needs n <= 127 and its
 * workgroup's LDS map (Sigma, x, y, and on the dataset_3d grid the gram and derivative tables)
 * within 160 KB, else LFM_E_ARG (lfm_mll_grad_f64 takes any n). hyp as lfm_batch_mll_f64; value[p] as its out[p] (the
 * same bits); grad packed in hyp's layout: for each problem dD[G_p] dS[G_p] dB[G_p] in order,
 * then for each problem d l, d obs_stddev, 0 (jitter is static, model.py:64). Not PD: value and
 * that problem's gradient NaN, status[p] = LFM_E_NOT_PD, returns LFM_E_NOT_PD. Deterministic (no
 * atomics: the same inputs give the same bits). */
int lfm_batch_mll_grad_f64(lfm_ctx* ctx, lfm_batch* batch, const double* hyp, int negative,
                           double* value, double* grad, int* status);

/* optax.adam(learning_rate, b1, b2, eps, eps_root) and JaxTrainer.fit's epoch handling
 * (src/trainer.py:162-228; src/main.py:45 and notebook.py:55 use adam(0.01)). */
typedef struct {
  double learning_rate, b1, b2, eps, eps_root;
  int64_t num_steps_per_epoch; /* after_epoch every this many steps, step 0 included (>= 1) */
  int fix_params;              /* after_epoch sets true_s[3] = 1.0, true_d[3] = 0.8          */
} lfm_adam;
/* JaxTrainer.fit of every problem of the batch at once, on the device: nsteps training steps
 * (trainer.py:105-132 under vscan, :198-216) in ONE launch, one workgroup per problem, no host
 * round trip between steps. Per step and problem: constrain (softplus for true_d / true_s /
 * true_b / obs_stddev, 0.5 + 3 sigmoid for l: model.py:66-121), value and gradient (as
 * lfm_batch_mll_grad_f64), the bijectors' chain rule, one Adam update of the unconstrained
 * parameters, then after_epoch on them when (step0 + s) % num_steps_per_epoch == 0 and
 * fix_params (the reference's index-3 quirk; nothing for G <= 3, as JAX drops the update).
 *   raw    [nhyp] in/out: the UNCONSTRAINED parameters in hyp's packed layout (the jitter slots
 *          hold the static jitter itself and are never changed)
 *   mu, nu [nhyp] in/out: Adam's moments (zeros to start; resumable across calls with step0)
 *   step0  steps already taken (Adam's count is step0 + s + 1)
 *   history [nsteps x nprob], step-major: each step's loss value before its update
 *   status [nprob] optional: 0, or 1 + the first step whose Cholesky failed (its loss and the
 *          parameters are NaN from there on, as under JAX); returns LFM_E_NOT_PD if any did.
 * The final constrain and after_epoch on the constrained model (trainer.py:218-222) are the
 * caller's (dis_project_amd.trainer.BatchTrainer). Problem sizes as lfm_batch_mll_grad_f64. */
int lfm_batch_fit_f64(lfm_ctx* ctx, lfm_batch* batch, const lfm_adam* opt, int negative,
                      int64_t step0, int64_t nsteps, double* raw, double* mu, double* nu,
                      double* history, int* status);

/* Value and gradient of CustomConjMLL(negative).step — what jax.value_and_grad(loss)
 * differentiates at trainer.py:126, before the bijectors' chain rule (trainer.py:103) —
 * with respect to the constrained parameters. grad[3G + 2]:
 *   [0,G) true_d   [G,2G) true_s   [2G,3G) true_b   [3G] l   [3G+1] obs_stddev.
 * jitter is a static field (model.py:64) and gets no gradient. Not PD: LFM_E_NOT_PD,
 * value and grad NaN. */
int lfm_mll_grad_f64(lfm_ctx* ctx, const double* x, const double* y, int64_t n,
                     const lfm_hyp* hyp, int negative, double* value, double* grad);

/* ------------- posterior at test inputs (latent_predict / multi_gene_predict) */
/* mean[m] = m(t) + K(t,x) S^{-1} (y - m(x)),  cov[m x m] = K(t,t) - K(t,x) S^{-1} K(x,t),
 * S = K(x,x) + diag(diag_vec) + diag_add I (diag_vec [n] may be NULL); model.py:420-514.
 * n and m must be multiples of num_genes (mean_function, model.py:145-149). The callers'
 * jitter / diagonalisation is applied by the shim. Not PD: LFM_E_NOT_PD, outputs NaN. */
int lfm_posterior_f64(lfm_ctx* ctx, const double* x, const double* y, int64_t n,
                      const double* diag_vec, double diag_add, const double* t, int64_t m,
                      const lfm_hyp* hyp, double* mean, double* cov);

/* ------------------- GaussianDistribution(loc, scale).log_prob(y) (gpjax 0.8.2) */
/* scale is a dense SPD n x n (row-major, leading dim lds; lower triangle read). */
int lfm_log_prob_f64(lfm_ctx* ctx, const double* loc, const double* scale, int64_t n,
                     int64_t lds, const double* y, double* out);

/* ----------------------- device-resident variants (inputs already in HBM) */
int lfm_dev_alloc(lfm_ctx* ctx, size_t bytes, void** out);
int lfm_dev_free(lfm_ctx* ctx, void* p);
int lfm_memcpy_h2d(lfm_ctx* ctx, void* dst, const void* src, size_t bytes);
int lfm_memcpy_d2h(lfm_ctx* ctx, void* dst, const void* src, size_t bytes);
/* Sets `bytes` bytes of device memory at dst to the byte `value` (e.g. sentinel fills). */
int lfm_memset_dev(lfm_ctx* ctx, void* dst, int value, size_t bytes);
/* As lfm_mll_f64 with x / y already on the ctx's device. */
int lfm_mll_f64_dev(lfm_ctx* ctx, const double* d_x, const double* d_y, int64_t n,
                    const lfm_hyp* hyp, int negative, double* out);
/* A device-resident dataset evaluated many times (training steps, random restarts): x (and y
 * when n is small) is read back and analysed once, here, instead of on every call. The caller
 * keeps d_x / d_y allocated and unmodified until lfm_data_destroy — the reference's Dataset is
 * an immutable JAX array pair (gpjax Dataset, objectives.py:21 / trainer.py:126) likewise. */
typedef struct lfm_data lfm_data;
int lfm_data_create(lfm_ctx* ctx, const double* d_x, const double* d_y, int64_t n,
                    lfm_data** out);
int lfm_data_destroy(lfm_data* data);
/* As lfm_mll_f64_dev on a dataset handle. */
int lfm_mll_f64_data(lfm_ctx* ctx, lfm_data* data, const lfm_hyp* hyp, int negative,
                     double* out);
/* nsets hyperparameter sets on one dataset (the random restarts of BASELINE.json configs[2]:
 * CustomConjMLL.step of each model in src/notebook.py:33-75's loop over one Dataset) ->
 * out[nsets], status[nsets] (optional: LFM_OK / LFM_E_NOT_PD per set; not PD -> NaN). The
 * values are lfm_mll_f64_data's, bit for bit. On schedule 3 the evaluations are pipelined: the
 * next set's prologue runs while the previous set's factorisation is in its chain-bound tail
 * (LFM_OVERLAP, default 1). Returns LFM_E_NOT_PD if any set failed. (ABI 5) */
int lfm_mll_multi_f64(lfm_ctx* ctx, lfm_data* data, int64_t nsets, const lfm_hyp* hyps,
                      int negative, double* out, int* status);
/* As lfm_gram_f64 / _f32 with x and out on the device. */
int lfm_gram_f64_dev(lfm_ctx* ctx, const double* d_x, int64_t n, const lfm_hyp* hyp,
                     double diag_add, int uplo, double* d_out, int64_t ldo);
int lfm_gram_f32_dev(lfm_ctx* ctx, const double* d_x, int64_t n, const lfm_hyp* hyp,
                     double diag_add, int uplo, float* d_out, int64_t ldo);

/* ------------------------------------------------------------- profiling */
int lfm_profile_enable(lfm_ctx* ctx, int on);
/* Restrict event timing to kernel classes whose bit is set (bit i = entry i of
 * lfm_profile_read's list; default all): fewer events inside a timed region. */
int lfm_profile_classes(lfm_ctx* ctx, unsigned mask);
int lfm_profile_reset(lfm_ctx* ctx);
/* Copies up to max entries; *count = number of kernel classes seen. */
int lfm_profile_read(lfm_ctx* ctx, lfm_kstat* stats, int max, int* count);

/* -------------------------------- multi-GPU farm: RCCL all-gather over xGMI */
/* Rank 0 creates the 128-byte unique id; the caller ships it to every rank. */
int lfm_farm_unique_id(lfm_ctx* ctx, unsigned char id[128]);
int lfm_farm_init(lfm_ctx* ctx, const unsigned char id[128], int nranks, int rank);
/* All-gather count fp64 per rank (host in, host out: recv holds nranks*count). */
int lfm_farm_allgather_f64(lfm_ctx* ctx, const double* send, int64_t count, double* recv);
/* One farm round of a resident batch — the replicate x ablation problems of
 * src/notebook.py:33-75, each rank holding its block of them (lfm_batch_create) — with the
 * exchange on the device: the batch's kernel writes every problem's MLL straight into this rank's
 * `slots` send slots (NaN past nprob), ncclAllGather runs on the ctx's stream behind it, and a
 * publish kernel copies the gathered nranks x slots values to pinned host memory and signals the
 * host: one launch chain, one bounded wait (LFM_RCCL_TIMEOUT_S), recv[nranks * slots] filled.
 * hyp / negative / status as lfm_batch_mll_f64 (status: this rank's problems). A failed or timed-
 * out exchange aborts the communicator (LFM_E_RCCL; recv untouched; later calls LFM_E_STATE until
 * lfm_farm_init). slots >= nprob, else LFM_E_ARG. */
int lfm_farm_batch_mll_f64(lfm_ctx* ctx, lfm_batch* batch, const double* hyp, int negative,
                           int64_t slots, double* recv, int* status);
int lfm_farm_destroy(lfm_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* LFM_H */
