// Shared declarations between the HIP kernels (kernels.hip) and the C ABI (capi.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/clvmcmc.h"

namespace clv {

constexpr int BLOCK = CLV_BLOCK;       // customers (lanes) per sweep workgroup
constexpr int HS = 64;                 // doubles of hyper state per chain
constexpr int H_TAG = 63;              // stride kernel: the sweep a published (beta, Sigma) belongs to
constexpr int TAPE_HYPER = 40;         // doubles of hyper variates per recorded sweep
constexpr int MAX_WORLD = 64;             // peer exchange: ranks (mail pointers staged in LDS)
constexpr int UMAIL = 2048;            // persistent kernel, world size > 1: LDS doubles for this rank's
                                       // unit partials (stride * local units must fit)
constexpr int HV = 40;                 // precomputed Philox hyper variates per chain: iw normals [0,3),
                                       // chi2 [3,6), beta normals [8,35)
constexpr int MAIL_TAIL = MAX_WORLD;   // peer mail: after the [2][world][chain][unit][stat] slots, one
                                       // progress word per rank (the sweep its level-2 side last polled for)
constexpr int CLK_RING = 1024;         // shader-clock record (SweepArgs::clk): sweeps kept
constexpr int DIAG_WORDS = 16;         // wait-timeout record (SweepArgs::diag, see kernels.hip report_wait)
enum : int { WAIT_HYPER = 1, WAIT_BLOCKS = 2, WAIT_P2P_MAIL = 3, WAIT_FX_MAIL = 4 };

// Doubles of peer-mail slots before the progress words.
__host__ __device__ inline int64_t mail_slots(int world, int chains, int stride, int units_per_rank) {
  return 2LL * world * chains * stride * units_per_rank;
}

// Hyper-state layout (per chain, HS doubles).
enum : int {
  H_BETA = 0,        // K x D row-major, beta[k][d] at k*D + d   (<= 27)
  H_SIGMA = 27,      // 3 x 3 row-major (D x D used)
  H_P00 = 36, H_P01 = 37, H_P11 = 38,  // inv(Sigma)[0:2,0:2] (bi:283, tri:402 quirk Q4)
  H_S00 = 39, H_S11 = 40,              // proposal scales Sigma[0,0], Sigma[1,1] (quirk Q2)
  H_S22 = 41, H_POSTVAR = 42, H_SQRT_POSTVAR = 43, H_OMEGA2 = 44,  // draw_eta (tri:321-333)
  H_INV_OMEGA2 = 45, H_INV_S22 = 46,   // 1 / omega2, 1 / Sigma[2,2] (Philox-mode draw_eta)
};

struct Ctrl {
  int64_t cur;        // sweeps completed; the next sweep kernel runs sweep cur + 1
  uint32_t arrive;    // arrival counter of the hyper kernel's workgroups
  uint32_t abort;     // persistent kernel: a wait timed out (host checks and clears it)
};

struct Geometry {
  int D, K, S;               // S = n_mh_steps
  int n_chains;
  int64_t n;                 // local customers
  int64_t n_global;
  int64_t shard_begin;
  int nb_local;              // ceil(n / BLOCK)
  int blocks_per_rank;
  int blocks_per_unit;       // G_b: blocks summed into one exchanged unit (power of two)
  int units_per_rank;
  int64_t n_units_global;
  int world_size;
  int stride;                // doubles per partial: K*D + D(D+1)/2 + 1
  int burnin, mcmc, thin, n_draws;
  int l2w;                   // level-2 record width: D*K + D(D+1)/2
};

struct Rng {
  uint64_t seed;
  int chain_first;
  const double* tape;        // replay tape (device), [chain][sweep][tape_sweep_stride]
  int64_t tape_sweep_stride;
  int64_t tape_sweeps;
};

struct HyperArgs {
  Geometry g;
  Rng r;
  const double* units;       // [world][chain][stride][units_per_rank] (statistic-major: coalesced reads)
  double* hyper;             // [chain][HS]
  Ctrl* ctrl;
  double* level2;            // [chain][n_draws][l2w]
  double* loglik;            // [chain][n_draws]
  const double* V;           // K x K
  const double* cholV;       // K x K lower
  const double* A0B0;        // K x D
  const double* S0B;         // D x D: S0 + B0'A0B0
  double nu_n;
  double omega2;
  int mode;                  // 0: after sweep (cur+1); 1: bivariate initial draw (sweep 1)
  const double* hvar;        // [chain][HV] Philox variates precomputed by the sweep kernel, or null
  unsigned long long* stamps; // diagnostic build only (CLV_STAMPS)
};

struct SweepArgs {
  Geometry g;
  Rng r;
  const int32_t* x;
  const double* tx;
  const double* T;
  const double* cov;         // (K-1) x n
  const double* log_s;
  double* lam;               // [chain][n]
  double* mu;
  const double* hyper;       // [chain][HS]
  double* blockpart;         // [chain][stride][blocks_per_rank]
  double* pblock;            // persistent kernel: [chain][nb_local][stride] hand-off slots
  const Ctrl* ctrl;
  Ctrl* ctrl_rw;             // persistent kernel: writes cur and abort
  double* hyp2;              // persistent kernel: [2][chain][HS] (beta, Sigma) hand-off slots by sweep parity
  double* level1;            // [chain][n_draws][n][D+2] or null
  double* sums;              // [chain][CLV_N_SUM_STATS][n] or null
  float2* qstore;            // CLV_SINK_SUMMARY_PCT: [chain][n_draws][n] (lambda, mu) float32, or null
  int64_t* n_stored;         // device counter of stored draws (chain 0 block 0 bumps it)
  double lam_init;
  int init;                  // 1: initialisation pass (bi:367-370), no sweep
  int fuse;                  // 1: the chain's last-arriving workgroup performs the level-2 draw
  uint32_t* chain_arrive;    // [chain] arrival counters of the fused tail (zero between launches)
  uint32_t* unit_arrive;     // [chain][units_per_rank] per-unit arrival counters (blocks_per_unit > 1)
  double* unitpart;          // [chain][stride][units_per_rank] unit partials (blocks_per_unit > 1)
  double* hvar_out;          // [chain][HV]: the chain's last workgroup precomputes the next level-2
                             // draw's Philox variates at its start (off the critical path), or null
  // persistent kernel at world size > 1 (peer exchange over xGMI): unit partials of sweep s go
  // straight into every rank's mail buffer, [2 (sweep parity)][world][chain][units_per_rank][stride]
  double* mail;              // this rank's mail buffer (device memory, polled by its level-2 workgroups)
  double* const* peers;      // [world] device pointers to every rank's mail buffer (peers[rank] = mail)
  int rank;
  const int32_t* wg_map;     // persistent kernel: linear workgroup -> (chain << 16 | block), or null
  // persistent kernel: the carried state at the end of a launch goes to these (the host swaps them
  // with lam / mu / hyper only if no wave aborted), the bound on every wait (s_memrealtime ticks,
  // 100 MHz) and a host-mapped copy of ctrl->abort (read by the host after the launch, no D2H copy)
  double* lam_out;
  double* mu_out;
  double* hyper_out;
  // persistent kernel, world size 1 (clv_create CLV_DEFER): the level-2 draw that follows a
  // launch's last sweep is deferred to the next launch (or a flush).  pend_out: the last sweep's
  // fixed-order statistics [chain][stride] go here instead of being drawn from; pend_in: such
  // statistics of the sweep before s_first, drawn from first (while the customer workgroups load
  // and draw their first sweep's variates).  Null: no deferral on that side.
  const double* pend_in;
  double* pend_out;
  uint64_t wait_ticks;
  uint32_t* abort_host;
  // wait-timeout record (device memory, DIAG_WORDS, zero when none): the first wave whose bounded
  // wait expires claims word 0 and writes what it was waiting for (kernels.hip report_wait); the
  // host formats it into clv_last_error()
  unsigned long long* diag;
  // shader-clock record [CLK_RING][2] (device memory, or null): chain 0's level-2 side writes
  // (s_memtime, s_memrealtime) when it publishes sweep s's draw, slot s % CLK_RING — clv_clock_ghz
  // reads the run's first and last slots (the average clock the sweeps ran at)
  unsigned long long* clk;
  HyperArgs h;               // level-2 arguments of the fused tail
  unsigned long long* stamps; // diagnostic build only (CLV_STAMPS): [1024][8] s_memrealtime stamps
};

struct GroupArgs {
  Geometry g;
  const double* blockpart;
  double* unitpart;          // [chain][stride][units_per_rank]
};


// Launchers (kernels.hip).
hipError_t launch_sweep(const SweepArgs& a, bool replay, hipStream_t st, hipEvent_t e0 = nullptr,
                        hipEvent_t e1 = nullptr);
hipError_t launch_group(const GroupArgs& a, hipStream_t st);
hipError_t launch_persist(const SweepArgs& a, int64_t s_first, int64_t n_sweeps, hipStream_t st,
                          hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);
hipError_t persist_occupancy(int D, int K, bool p2p, int* blocks_per_cu);
hipError_t persist_scratch_bytes(int D, int K, bool p2p, size_t* bytes);  // spilled instances: > 0
// The deferred level-2 draw alone (a.pend_in, no sweeps): one level-2 workgroup per chain.
hipError_t launch_persist_flush(const SweepArgs& a, int64_t s_first, hipStream_t st);
hipError_t launch_hyper(const HyperArgs& a, bool replay, hipStream_t st);
hipError_t launch_set_hyper(int D, int K, int n_chains, double* hyper, const double* beta_sigma,
                            double omega2, bool replay, hipStream_t st);
hipError_t launch_debug_philox(uint32_t k0, uint32_t k1, const uint32_t* ctr, int64_t n, uint32_t* out,
                               hipStream_t st);
hipError_t launch_debug_variates(uint64_t seed, int chain, uint32_t sweep, int64_t n, int S, float* tl,
                                 float* tm, float* ua, float* l2u, double* uz, double* ut, double* ea, double* ez,
                                 hipStream_t st);
hipError_t launch_debug_log2u_scan(uint64_t w_begin, uint64_t w_end, int n_blocks, double* out, hipStream_t st);
hipError_t launch_debug_t3(const uint32_t* w, int64_t n, int packed, float* tl, float* tm, hipStream_t st);
hipError_t launch_debug_level2(int D, int K, const double* prior_dev, const double* in, double* out,
                               hipStream_t st);
hipError_t launch_debug_hyper_variates(uint64_t seed, int chain, uint32_t sweep, double df, int64_t n,
                                       double* chi2, double* normals, hipStream_t st);
hipError_t launch_debug_exp(const double* x, int64_t n, double* out, hipStream_t st, bool log_fn = false);
hipError_t launch_debug_mh(const int32_t* x, const uint8_t* z, const double* T, const double* tau, const double* m,
                           const double* prec, const double* cur_pt, const float* t3, const double* scale,
                           const float* log_u, int64_t n, double* out, hipStream_t st);

}  // namespace clv
