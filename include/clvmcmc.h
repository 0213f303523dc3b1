/*
 * clvmcmc.h — C ABI of the MI355X-native Gibbs/MH sampler for the Abe (2009/2015)
 * hierarchical Pareto/NBD model (libclvmcmc.so, built from mcmc_clv_model_amd/csrc/).
 *
 * The reference (lucagem29/mcmc_clv_model) is pure Python and has no FFI of its own;
 * its drop-in boundary is the Python function pair
 *     src/models/bivariate/mcmc.py:437   mcmc_draw_parameters(...)
 *     src/models/trivariate/mcmc.py:580  mcmc_draw_parameters_rfm_m(...)
 * The Python host (mcmc_clv_model_amd/bivariate.py, trivariate.py) keeps those
 * signatures and binds the entry points below with ctypes.
 * Each entry point names the reference code it replaces.
 *
 * Conventions
 *  - Every function returns 0 on success or a negative CLV_E* code; the message of the
 *    last failure on the calling thread is available from clv_last_error().
 *  - Inputs are copied to device memory by clv_create(); outputs are written into
 *    caller-owned, contiguous, preallocated host buffers (float64, C order).
 *  - A sampler handle belongs to one host thread and one HIP device.
 *  - Customer data is struct-of-arrays: one contiguous array per CBS column.
 *  - State, log posteriors and the level-2 draw are float64, like the reference.  In Philox mode
 *    the MH proposal noise t3 is generated in float32 (fp32 hardware transcendentals), and the
 *    accept test compares in float64 against cur + ln2 * log2(U) with log2(U) an fp32 v_log_f32
 *    (DESIGN.md §5); replay mode (tests) takes the reference's own float64 variates.
 */
#ifndef CLVMCMC_H
#define CLVMCMC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CLV_ABI_VERSION 2

/* Customers per workgroup == the sufficient-statistic block size. Shards must begin on a
 * multiple of it so block partial sums are identical for every GPU count. */
#define CLV_BLOCK 256
#define CLV_MAX_K 9
#define CLV_MAX_D 3

enum { CLV_OK = 0, CLV_EINVAL = -1, CLV_EHIP = -2, CLV_ESTATE = -3, CLV_ENOMEM = -4 };
enum { CLV_RNG_PHILOX = 0, CLV_RNG_REPLAY = 1 };
/* CLV_SINK_SUMMARY_PCT: the summary sums plus every stored (lambda, mu) as a float32 pair,
 * [chain][draw][n] (8 B per customer and stored sweep instead of the full sink's 8 (D+2)), from
 * which clv_level1_summary_sampler forms the per-customer 2.5 / 97.5 percentiles of Table 4
 * (analysis_bi_helpers.py:95-96, 116-117): exact order statistics of the float32-rounded draws. */
enum { CLV_SINK_FULL = 0, CLV_SINK_SUMMARY = 1, CLV_SINK_NONE = 2, CLV_SINK_SUMMARY_PCT = 3 };

/* Per-customer running sums kept on device by CLV_SINK_SUMMARY / _PCT, accumulated over stored
 * draws. Layout of clv_read_summary(): [chain][stat][n].  CLV_SUM_MU_CAPPED sums
 * min(mu, CLV_SUMMARY_MU_CAP): Table 4's capped posterior mean of mu (analysis_bi_helpers.py:88-93). */
#define CLV_SUMMARY_MU_CAP 0.05
enum {
  CLV_SUM_LAMBDA = 0, CLV_SUM_MU, CLV_SUM_Z, CLV_SUM_LOG_LAMBDA, CLV_SUM_LOG_MU,
  CLV_SUM_LAMBDA2, CLV_SUM_MU2, CLV_SUM_ETA, CLV_SUM_LOG_ETA, CLV_SUM_MU_CAPPED, CLV_SUM_TAU,
  CLV_N_SUM_STATS
};

typedef struct clv_config {
  int32_t abi_version;   /* must equal CLV_ABI_VERSION */
  int32_t D;             /* 2 = bivariate (bivariate/mcmc.py), 3 = trivariate (trivariate/mcmc.py) */
  int32_t K;             /* design-matrix columns incl. the intercept, 1..CLV_MAX_K (bi:467-470) */
  int32_t n_mh_steps;    /* MH steps per sweep (bi:278, default 20) */
  int32_t burnin, mcmc, thin;          /* bi:437-447 semantics */
  int32_t n_chains;      /* chains batched into one launch (reference: sequential, bi:485) */
  int32_t chain_first;   /* global index of chain 0 of this handle: Philox key = seed + chain */
  int32_t rng_mode;      /* CLV_RNG_PHILOX or CLV_RNG_REPLAY (test mode, clv_set_replay_tape) */
  int32_t draw_sink;     /* CLV_SINK_* */
  int32_t device;        /* HIP device ordinal, -1 = current device */
  uint64_t seed;         /* Philox key base (reference: default_rng(seed + chain), bi:486) */
  int64_t n_global;      /* customers in the whole problem (nu_n and the log-lik mean use it) */
  int64_t shard_begin;   /* global index of this shard's first customer, multiple of CLV_BLOCK */
  int32_t world_size;    /* shards (one process per GPU); 1 = unsharded */
  int32_t rank;          /* this shard */
  int32_t blocks_per_rank; /* blocks of CLV_BLOCK customers per shard (last shard may be short);
                              0 = derive (unsharded only) */
  int32_t blocks_per_unit; /* blocks whose partials are summed into one exchanged unit (power of
                              two, a function of n_global only so every world size sums alike);
                              0 = derive with clv_default_blocks_per_unit(n_global) */
  uint64_t stream;       /* hipStream_t to launch on; 0 = a stream owned by the sampler */
} clv_config;

typedef struct clv_data {
  int64_t n;                 /* customers in this shard */
  const int32_t* x;          /* repeat transactions (bi:280) */
  const double* t_x;         /* recency (bi:194) */
  const double* T_cal;       /* calibration length (bi:194) */
  const double* covariates;  /* (K-1) arrays of n doubles, one per non-intercept column; NULL if K==1 */
  const double* log_s;       /* log average spend, D==3 only (tri:329) */
} clv_data;

/* Host-computed constants; the reference computes the same quantities on the host. */
typedef struct clv_prior {
  double lam_init;           /* bi:368 */
  double V[CLV_MAX_K * CLV_MAX_K];       /* inv(X'X + A0), K x K row-major (bi:248-249; constant) */
  double chol_V[CLV_MAX_K * CLV_MAX_K];  /* lower Cholesky factor of V */
  double A0B0[CLV_MAX_K * CLV_MAX_D];    /* A0 @ B0, K x D row-major (bi:250) */
  double S0_B0A0B0[CLV_MAX_D * CLV_MAX_D]; /* S0 + B0' A0 B0, D x D (bi:255 after expansion) */
  double nu_n;               /* nu0 + n_global (bi:256) */
  double beta_init[CLV_MAX_K * CLV_MAX_D]; /* tri: beta used by sweep 1 = beta_0 (tri:504) */
  double sigma_init[CLV_MAX_D * CLV_MAX_D];/* tri: Sigma used by sweep 1 = gamma_00 (tri:504) */
  double omega2;             /* tri: var(log_s, ddof=1) (tri:494) */
} clv_prior;

typedef struct clv_sampler clv_sampler;

int32_t clv_abi_version(void);
int32_t clv_default_blocks_per_unit(int64_t n_global);
/* sizeof(clv_config), sizeof(clv_data), sizeof(clv_prior) for which = 0, 1, 2 (binding checks). */
int64_t clv_sizeof(int32_t which);
const char* clv_last_error(void);
int clv_device_count(int32_t* count);

/* Allocate device state, upload the shard, initialise lambda/mu (bi:367-379, tri:488-504) and,
 * for D==2, the block partial sums the first level-2 draw needs. Replaces the setup half of
 * _run_chain (bi:346-382, tri:465-507). */
int clv_create(const clv_config* cfg, const clv_data* data, const clv_prior* prior,
               clv_sampler** out);
void clv_destroy(clv_sampler* s);

/* Test mode (CLV_RNG_REPLAY): variates recorded from the reference's numpy Generator.
 * Per chain, per sweep: [u_z n][v_tau n][S x (t_l n, t_m n, u_acc n)][eta_z n if D==3]
 * [hyper 40: iw_normal(3) iw_chi2(3) mvn_noise(<=27) pad]; chains back to back. */
int clv_set_replay_tape(clv_sampler* s, const double* tape, int64_t n_sweeps);
int64_t clv_replay_sweep_stride(const clv_sampler* s);

/* Run n sweeps (world_size == 1, or sharded after clv_p2p_connect). One sweep = a6's loop body: z (bi:388),
 * tau (bi:390), level-2 (bi:393), level-1 MH (bi:396), eta (tri:524-526), storage (bi:402-428).
 * Synchronous; chunks of sweeps are replayed from a captured hipGraph.  The persistent path at
 * world size 1 leaves the level-2 draw that follows its last sweep pending (CLV_DEFER, default on):
 * the next clv_run draws it first, and clv_get_state / clv_set_state / clv_read_draws (level 2) /
 * clv_sweep / clv_hyper draw it before they read or replace the state — the same draw either way,
 * so results never depend on how a run is cut into clv_run calls. */
int clv_run(clv_sampler* s, int64_t n_sweeps);
/* Persistent path only: undo the last completed clv_run (state, sweep count, summary sums) — a
 * sharded step whose persistent launch failed on another rank is redone by every rank from the
 * same point.  A clv_run that fails (a wait timed out) already leaves the state unchanged. */
int clv_rollback(clv_sampler* s);

/* Sharded stepping (one process per GPU; the caller exchanges the unit partials over RCCL):
 *   after clv_create, bivariate only: [exchange] clv_hyper   (initial draw, bi:393 of sweep 1)
 *   per sweep:                        clv_sweep, [exchange] clv_hyper
 * (bivariate: the hyper after sweep s is bi:393 of sweep s+1; trivariate: tri:529 of sweep s).
 * clv_partials() exposes this shard's unit partials, [chain][stride][units_per_rank] doubles;
 * clv_hyper() reads the gathered buffer [world][chain][stride][units_per_rank]
 * (NULL = the local buffer, world_size == 1) and sums it in global unit order. */
int clv_sweep(clv_sampler* s);
int clv_hyper(clv_sampler* s, const double* gathered_device_ptr);
int clv_partials(clv_sampler* s, double** device_ptr, int64_t* n_doubles, int32_t* stride);
/* Device-to-device copy of this shard's unit partials into dst (on the sampler's stream). */
int clv_copy_partials(clv_sampler* s, void* dst_device_ptr);
int clv_synchronize(clv_sampler* s);
int64_t clv_sweeps_done(const clv_sampler* s);

/* Average shader clock (GHz) of the device over the last clv_run: s_memtime against s_memrealtime
 * (100 MHz) over its sweeps but the last (at most the last 1024), each sweep's interval measured on
 * one CU by chain 0's level-2 workgroup of the persistent kernel (s_memtime counts per XCD).  *ghz = 0
 * when the run had fewer than 2 sweeps or ran without the persistent kernel (the launch-per-sweep
 * kernel keeps no record: it measured 1-1.5% slower with one).  Measurement
 * only — the reference has no counterpart; bench.py reports it beside every timed line, because
 * MI355X boxes of one pool were measured to run the same cycles at clocks ~13% apart (DESIGN.md §8
 * round 5).  Synchronizes the sampler's stream. */
int clv_clock_ghz(clv_sampler* s, double* ghz);
/* Shader clock (GHz) read by a probe kernel enqueued on the sampler's stream behind whatever it runs
 * (csrc/probe.hip): one 64-lane workgroup per CU busy for `us` microseconds (1..1e5) of s_memrealtime,
 * s_memtime against s_memrealtime on each CU.  For legs whose kernel keeps no record of its own (the
 * launch-per-sweep kernel): called right after the timed launches, it reads the clock they ran at
 * (the governor moves on a millisecond scale).  Measurement only.  Synchronizes the stream. */
int clv_clock_probe(clv_sampler* s, double us, double* ghz);
/* How clv_run launches: out[6] = (persistent 0/1, persistent-kernel workgroups per CU, CUs,
 * workgroups per sweep, reserved (0), reserved (0)).
 * Persistent = one launch for all of a clv_run's sweeps with every customer block resident, chosen
 * at create when world_size == 1, Philox mode, every workgroup fits at once (with a residency
 * margin) and few enough CUs hold two of them for it to pay (clv_debug_persist_choice), unless
 * CLV_PERSISTENT is "0" ("1": wherever it fits).  Otherwise one launch of the sweep kernel per
 * sweep (fused level-2 tail), replayed from captured hipGraph chunks. */
int clv_launch_info(const clv_sampler* s, int64_t* out);
/* Sharded runs without a host collective per sweep (world_size > 1, Philox mode): the persistent
 * kernel's level-2 workgroup of each chain writes this rank's unit partials of sweep s straight into
 * EVERY rank's mail buffer (device stores over xGMI into IPC-mapped peer memory), waits until its
 * own mail holds all ranks' units, and sums them in the same global unit order as clv_hyper — so
 * results are bitwise those of clv_sweep/clv_hyper with an all-gather (and of world size 1).
 * Replaces, per sweep, the all-gather of bi:243-255's statistics.
 *   clv_p2p_info:    out[6] = (capable 0/1, connected 0/1, mail bytes, mail device pointer,
 *                    persistent 0/1, mail memory: 0 uncached / 1 fine-grained / 2 device default /
 *                    -1 none); persistent = every workgroup of the persistent grid fits at
 *                    once on this GPU.  Otherwise (any shard size) clv_run launches the sweep
 *                    kernel once per sweep and its fused level-2 tail exchanges the same way: the
 *                    chain's unit-last workgroups store this rank's unit partials into every rank's
 *                    mail, the chain's last one waits for all ranks' units in its own mail, sums
 *                    them in global order and draws — no host collective, no separate launches.
 *   clv_p2p_export:  this rank's mail buffer as a hipIpcMemHandle (CLV_IPC_HANDLE_BYTES bytes).
 *   clv_p2p_connect: every rank's mail: handles = [world][CLV_IPC_HANDLE_BYTES] (opened with
 *                    hipIpcOpenMemHandle; this rank's entry ignored) or ptrs = [world] device
 *                    pointers valid in this process (ranks sharing one process).  Collective in
 *                    effect: call it on every rank, then barrier, before the first clv_run.
 * After connecting, clv_run(n) runs n sweeps (bivariate: after the initial clv_hyper); every rank
 * must call it with the same n.  A rank that waits longer than the bound (10 s by default,
 * CLV_WAIT_TIMEOUT_MS) for its peers fails with CLV_EHIP and keeps its state from before the call;
 * ranks whose call completed undo it with clv_rollback, and clv_p2p_connect may be called again
 * (it refills this rank's mail) to resume the peer exchange. */
#define CLV_IPC_HANDLE_BYTES 64
int clv_p2p_info(const clv_sampler* s, int64_t* out);
int clv_p2p_export(clv_sampler* s, void* handle);
int clv_p2p_connect(clv_sampler* s, const void* handles, const uint64_t* ptrs);
/* Drop the peer connection (closes opened IPC mappings, forgets the peers' mail pointers): a sharded
 * clv_run then fails with CLV_ESTATE until clv_p2p_connect is called again.  Idempotent. */
int clv_p2p_disconnect(clv_sampler* s);
/* Which peer exchange clv_run takes on this shard: on = 1 the persistent kernel (only where its grid
 * fits: clv_p2p_info out[4] as created), 0 the fused exchange (one sweep launch per sweep).  Both
 * write the same mail with the same protocol and give the same bits; ShardedSampler falls back from
 * the first to the second (then to RCCL) when the verification against RCCL fails. */
int clv_p2p_set_persistent(clv_sampler* s, int32_t on);
/* Bound of every wait in the persistent / fused-exchange kernels, in ms (default 2000 at world size
 * 1, 10000 with peers; the CLV_WAIT_TIMEOUT_MS environment variable sets the default at create).
 * A short bound makes a failed peer-exchange check cheap (distributed.ShardedSampler's verification
 * runs under 500 ms). */
int clv_set_wait_timeout(clv_sampler* s, double ms);
/* Launch on another stream from now on (e.g. a stream under hipGraph capture by the caller,
 * who then replays the captured sweeps), and adjust the host's sweep count by n (+chunk per
 * replay; -chunk after a capture, which records launches without executing them). */
int clv_set_stream(clv_sampler* s, uint64_t stream);
int clv_note_sweeps(clv_sampler* s, int64_t n);

/* Outputs. level1: [chain][draw][n][D+2] (lambda, mu, tau, z, [eta]) — bi:407-410, tri:544-548;
 * level2: [chain][draw][D*K + D(D+1)/2] — bi:411-412, tri:549-554;
 * loglik: [chain][draw] per-draw mean of the likelihood term — bi:423-428.
 * Any pointer may be NULL. level1 requires draw_sink == CLV_SINK_FULL. */
int clv_read_draws(clv_sampler* s, double* level1, double* level2, double* loglik);
/* Stream the level-1 draws into the caller's host buffer while the sampler runs (world_size 1,
 * CLV_SINK_FULL) — the drop-in's end-to-end time, run_mcmc_abe.py:60-77 around bi:437-504, instead
 * of one pageable copy of every stored draw after the run.  level1: [chain][n_draws][n][D+2]
 * doubles, caller-owned, valid until clv_read_draws with the same pointer (or NULL here, or
 * clv_destroy).  Host threads of a process-wide copy pool first fault its pages in (madvise
 * MADV_POPULATE_WRITE), then each clv_run (its stored sweeps in sub-runs of >= 256 sweeps and ~64 MB
 * of draws) hands the draws it completed to the pool (pinned staging, DMA on the device's null
 * stream, which the sampler's non-blocking stream does not wait for) and goes on sampling;
 * clv_read_draws(s, level1, ...) waits for the copies in flight and copies what is left.  Same
 * launches, same sweeps, same bits.  NULL stops streaming (after the copies in flight). */
int clv_stream_draws(clv_sampler* s, double* level1);
/* [chain][CLV_N_SUM_STATS][n] running sums over stored draws, and the number of stored draws. */
int clv_read_summary(clv_sampler* s, double* sums, int64_t* n_stored);

/* Current state: lambda, mu [chain][n]; hyper [chain][beta K*D, Sigma D*D]. Setting the state
 * is exact resume (the Philox counter is the sweep index); lambdas and mus must be positive,
 * normal and finite (CLV_EINVAL otherwise: the sweep takes their logs, bi:286-287). */
int clv_get_state(clv_sampler* s, double* lambdas, double* mus, double* hyper);
int clv_set_state(clv_sampler* s, const double* lambdas, const double* mus, const double* hyper,
                  int64_t sweeps_done);

/* Per-launch timing of the sweep kernel with HIP events on the launch stream. */
int clv_set_timing(clv_sampler* s, int32_t enable);
int clv_kernel_time(clv_sampler* s, double* sweep_kernel_ms_total, int64_t* sweep_launches,
                    double* hyper_kernel_ms_total, int64_t* hyper_launches);

/* ---- test hooks (run the device code paths on caller data) ---- */
/* Host clock (steady_clock ns) at the steps of the last persistent clv_run at world size 1:
 * out[0] entry, [1] after hipSetDevice, [2] before the launch call, [3] after it, [4] launch
 * enqueued (end event recorded), [5] end seen, [6] return; 0 where not reached. */
int clv_debug_host_times(const clv_sampler* s, int64_t* out);
/* Philox4x32-10 on device: ctr/out are n x 4 words. */
int clv_debug_philox(uint32_t k0, uint32_t k1, const uint32_t* ctr, int64_t n, uint32_t* out);
/* The Philox-mode variates of one sweep for customers [0, n): t_l/t_m/u_acc are S x n;
 * log2_u_acc (S x n, may be NULL) is the accept threshold's log2 U exactly as the sweep kernels
 * form it (v_log_f32 of the fp32 uniform; bi:329-330 compares exp(lp' - lp) with U). */
int clv_debug_variates(uint64_t seed, int32_t chain, uint32_t sweep, int64_t n, int32_t n_steps,
                       float* t_l, float* t_m, float* u_acc, double* u_z, double* u_tau,
                       double* e_alive, double* eta_z, float* log2_u_acc);
/* The accept threshold's log2 U over the Philox words [w_begin, w_end) (<= 2^32), against float64
 * log2 of the same fp32 uniform: out[4] = max error in fp32 ulps of the exact value, max absolute
 * error, the word with the largest ulp error, max ulp error where U <= 1/2. */
int clv_debug_log2u_scan(uint64_t w_begin, uint64_t w_end, double* out);
/* The MH proposal's Student-t(3) transforms on caller words (n x 3 uint32: radius word of t_l,
 * radius word of t_m, angle word: t_l takes its high 16 bits, t_m its low 16 bits), as the sweep
 * kernels form them (packed 0: t3_f32, 1: the trivariate launch-per-sweep kernels' t3_pair).
 * Pins the proposal's symmetry (bi:316-317 draws Sigma[0,0] * standard_t(3)). */
int clv_debug_t3(const uint32_t* words, int64_t n, int32_t packed, float* t_l, float* t_m);
/* Level-2 draw from given sufficient statistics and variates (replaces bi:233-262 given rng):
 * xty K*D, yty D*D, iw_normal n_tril, iw_chi2 D, z D*K (standard normals) -> beta, Sigma. */
int clv_debug_level2(int32_t D, int32_t K, const clv_prior* prior, const double* xty,
                     const double* yty, const double* iw_normal, const double* iw_chi2,
                     const double* z, double* beta, double* sigma);
/* Diagnostic build only (make STAMPS=1 -> libclvmcmc_stamps.so): per-sweep s_memrealtime stamps
 * [1024][8] (slot = sweep % 1024); CLV_ESTATE in the shipped library. */
int clv_debug_stamps(clv_sampler* s, uint64_t* out);
/* Diagnostic build only: per workgroup of the latest sweep launch, [chain * n_blocks + 1 per chain]
 * records of 12 u64 (sweep kernel: start / end of customer work (s_memrealtime), HW_ID, XCC_ID,
 * s_memtime phase stamps; persistent kernel: s_memrealtime phase stamps of one sweep, see
 * kernels.hip CLV_P_STAMP); out must hold 12 * n_chains * (n_blocks + 1) values; CLV_ESTATE in
 * the shipped library. */
int clv_debug_wg_stamps(clv_sampler* s, uint64_t* out);
/* Philox-mode chi-square and normal draws of the hyper stream (n of each). */
int clv_debug_hyper_variates(uint64_t seed, int32_t chain, uint32_t sweep, double df, int64_t n,
                             double* chi2, double* normals);
/* The Philox-mode MH step's fp64 exp (csrc/fastmath.h, |x| <= 700) on n values. */
int clv_debug_exp(const double* x, int64_t n, double* out);
/* The Philox-mode fp64 log (csrc/fastmath.h log_fast, x > 0 normal) on n values: the z/tau
 * draw's logs (bi:200-225) and the eta normal's radius. */
int clv_debug_log(const double* x, int64_t n, double* out);
/* One Philox-mode MH step exactly as the sweep kernels run it (bi:291-335: log posterior with the
 * Q3 cap, fma + clip proposal, accept iff pm <= 5 and plp > cur + ln2 log2 U), on n independent
 * lanes.  Per lane: x, z, T_cal, tau, mean [n][2] (X @ beta), cur_pt [n][2] (log lambda, log mu),
 * t3 [n][2] (fp32 t3 noise), log_u = log2 U (fp32, as the sweeps draw it; +inf = a padded step);
 * shared prec3 = inv(Sigma)[0:2,0:2] as (p00, p01, p11) and scale2 = (Sigma00, Sigma11) (Q2).
 * out [n][7] = current log posterior (up to a per-customer constant), the proposal's (before the
 * Q3 cap), the proposal (pl, pm; pm clipped below only: one above 5 is rejected whatever it is),
 * the new log lambda, log mu and log posterior. */
int clv_debug_mh_step(int64_t n, const int32_t* x, const uint8_t* z, const double* T_cal, const double* tau,
                      const double* mean, const double* prec3, const double* cur_pt, const float* t3,
                      const double* scale2, const float* log_u, double* out);
/* Host only (no device): the persistent grid's placement map for n_chains chains of nb customer
 * workgroups (+1 level-2 workgroup each) on n_cu CUs — out[linear workgroup] = chain << 16 | block. */
int clv_debug_wg_map(int32_t n_chains, int32_t nb, int32_t n_cu, int32_t* out);
/* Host only: 1 if a persistent grid of grid_wgs workgroups is taken as resident at once on n_cu CUs
 * admitting blocks_per_cu of them each: min(blocks_per_cu, 8, the SGPR rule at 102 SGPRs) per CU,
 * less one slot per 32 CUs (MI355X guide, residency of 256-thread blocks), else 0. */
int clv_debug_persist_fits(int64_t grid_wgs, int32_t blocks_per_cu, int32_t n_cu);
/* Host only: 1 if clv_create runs a grid of grid_wgs persistent workgroups (n_chains chains of a
 * D / K model) on n_cu CUs: it fits (clv_debug_persist_fits) and few enough CUs hold two of its
 * workgroups for it to beat the launch-per-sweep kernel (capi.hip persist_worth, measured
 * crossover); CLV_PERSISTENT=1 forces it wherever it fits, =0 never. */
int clv_debug_persist_choice(int32_t D, int32_t K, int32_t n_chains, int64_t grid_wgs, int32_t blocks_per_cu,
                             int32_t n_cu);

/* ---- In-process multi-device runs (SURVEY.md §8b devices=, §8e) ----
 * A group drives the n shards of one problem from one host thread: shards[r] = the sampler of rank
 * r of a world of n (clv_create with world_size n, blocks_per_rank / blocks_per_unit of the shard
 * plan, each on its own device or sharing one), all at the same sweep.  Per sweep the shards
 * exchange their unit partials (the all-gather of bi:243-255's statistics) either
 *   CLV_EXCHANGE_P2P:  every shard's persistent grid fits at once (on shared devices: together) and
 *                      distinct devices have peer access — clv_p2p_connect by device pointers, one
 *                      persistent launch per shard and call, all in flight before any is awaited;
 *   CLV_EXCHANGE_COPY: per sweep the sweep kernels, device-to-device copies of each shard's unit
 *                      partials into every shard's gathered buffer (stream-ordered by events), and
 *                      every shard's level-2 draw.
 * CLV_EXCHANGE_AUTO picks P2P where possible and no two shards share a device (their persistent
 * kernels would have to run concurrently from different streams, which HIP does not promise); the
 * group disconnects the shards it connected when destroyed.  Results are bitwise those of the unsharded run.  A
 * P2P call that times out on any shard is undone on the others and redone by copies (kept).
 * clv_group_run is synchronous; the bivariate initial draw (bi:393 of sweep 1) is its first
 * exchange.  The group does not own the shards (destroy the group first). */
enum { CLV_EXCHANGE_AUTO = 0, CLV_EXCHANGE_P2P = 1, CLV_EXCHANGE_COPY = 2 };
typedef struct clv_group clv_group;
int clv_group_create(clv_sampler* const* shards, int32_t n, int32_t exchange, clv_group** out);
int clv_group_run(clv_group* g, int64_t n_sweeps);
int32_t clv_group_exchange(const clv_group* g);
void clv_group_destroy(clv_group* g);

/* ---- Posterior analysis on device ----
 * Inputs are level-1 draws [n_draws][n][width] in the reference's layout, chains stacked
 * (np.vstack of draws["level_1"]); width 4 = (lambda, mu, tau, z), 5 = (+ eta).  The plain
 * variants take host arrays (uploaded, device = ordinal or -1 for the current one); the
 * *_sampler variants use the draws a CLV_SINK_FULL sampler holds in HBM after its run. */
enum {
  CLV_L1_MEAN_LAMBDA = 0, CLV_L1_LAMBDA_P025, CLV_L1_LAMBDA_P975, CLV_L1_MEAN_MU, CLV_L1_MEAN_MU_CAPPED,
  CLV_L1_MU_P025, CLV_L1_MU_P975, CLV_L1_MEAN_Z, CLV_L1_MEAN_TAU, CLV_L1_MEAN_ETA, CLV_N_L1_STATS
};
/* Posterior predictive future transactions: bivariate/mcmc.py:506-546 (draw_future_transactions)
 * and, with simulate_spend = 1 (width 5), the lognormal spend totals of trivariate/mcmc.py:660-749.
 * x_future int64 [n_draws][n]; spend_future float64 [n_draws][n] or NULL. */
int clv_predict(int32_t device, const double* level1, int64_t n_draws, int64_t n, int32_t width,
                const double* T_cal, double T_star, uint64_t seed, int32_t simulate_spend, double sigma_s,
                int64_t* x_future, double* spend_future);
int clv_predict_sampler(clv_sampler* s, double T_star, uint64_t seed, int32_t simulate_spend,
                        double sigma_s, int64_t* x_future, double* spend_future);
/* Weekly tracking curve of bivariate/analysis_abe.py:444-464: for each week t of `times`
 * (ascending), the mean over draws of the posterior-predictive number of repeat transactions of
 * the customers active in that week (birth_week < t <= birth_week + tau).  inc_weekly [n_times]. */
int clv_track(int32_t device, const double* level1, int64_t n_draws, int64_t n, int32_t width,
              const double* birth_week, const double* times, int32_t n_times, uint64_t seed,
              double* inc_weekly);
int clv_track_sampler(clv_sampler* s, const double* birth_week, const double* times, int32_t n_times,
                      uint64_t seed, double* inc_weekly);
/* Per-customer posterior statistics (out [n][CLV_N_L1_STATS]): means as numpy's axis-0 mean,
 * capped-mu mean min(mu, mu_cap) and numpy-'linear' 2.5/97.5 percentiles of lambda and mu —
 * utils/analysis_bi_helpers.py:15-27 (post_mean_*) and :75-107 (compute_table4). */
int clv_level1_summary(int32_t device, const double* level1, int64_t n_draws, int64_t n, int32_t width,
                       double mu_cap, double* out);
/* The _sampler variant also serves a CLV_SINK_SUMMARY_PCT sampler (no level-1 draws kept): means
 * from its running sums (pooled over chains), percentiles from its float32 (lambda, mu) store;
 * mu_cap must then be CLV_SUMMARY_MU_CAP. */
int clv_level1_summary_sampler(clv_sampler* s, double mu_cap, double* out);
/* Mean over draws of the total log-likelihood incl. -lgamma(x+1) (analysis_bi_helpers.py:52-72). */
int clv_chain_total_loglik(int32_t device, const double* level1, int64_t n_draws, int64_t n, int32_t width,
                           const int32_t* x, const double* T_cal, double* mean_total);
int clv_chain_total_loglik_sampler(clv_sampler* s, double* mean_total);

/* ---- Data preparation on device ----
 * Event log -> CBS (utils/elog2cbs2param.py:33-94): events (cust, date in ns since the epoch,
 * sales or NULL = 1) -> one row per customer with calibration events, sorted by cust.  Output
 * buffers hold n_events rows (upper bound); *n_customers rows are written.  Hold-out columns
 * (T_star, x_star, sales_star) are meaningful when T_cal_ns < T_tot_ns. */
int clv_elog2cbs(int32_t device, int64_t n_events, const int64_t* cust, const int64_t* date_ns, const double* sales,
                 int64_t unit_ns, int64_t T_cal_ns, int64_t T_tot_ns, int64_t* n_customers, int64_t* cust_out,
                 int64_t* x, double* t_x, double* litt, double* sales_out, double* sales_x, int64_t* first_ns,
                 double* T_cal, double* T_star, int64_t* x_star, double* sales_star);
/* Synthetic Abe (2009) data (bivariate/mcmc.py:95-187): covariates [1, U(-1,1)...] (or the
 * caller's [n][K] incl. intercept), theta = exp(X beta + MVN(0, gamma)), tau ~ Exp(mu), purchases
 * as a Poisson process until min(T_cal + max T_star, tau); CBS of bi:75-89 and hold-out counts
 * x_star[n_star][n].  beta K x 2 row-major, gamma 2 x 2, T_cal[n].  n_events = elog rows per
 * customer; with elog_offsets (exclusive prefix sum of n_events from a first call) a second call
 * also writes the elog (cust 1-based, t). */
int clv_generate_pareto_abe(int32_t device, int64_t n, int32_t K, const double* beta, const double* gamma,
                            const double* covars, const double* T_cal, int32_t n_star, const double* T_star,
                            uint64_t seed, int64_t* x, double* t_x, double* lambda_true, double* mu_true,
                            double* tau_true, uint8_t* alive_true, int64_t* x_star, double* covars_out,
                            int64_t* n_events, const int64_t* elog_offsets, int64_t elog_rows, int64_t* elog_cust,
                            double* elog_t);

#ifdef __cplusplus
}
#endif
#endif /* CLVMCMC_H */
