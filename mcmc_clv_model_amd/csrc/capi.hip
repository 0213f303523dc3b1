// C ABI of libclvmcmc.so (declared in include/clvmcmc.h): device memory, the sweep pipeline,
// hipGraph capture of sweep chunks, and outputs.  Host-side replacement of _run_chain /
// mcmc_draw_parameters (src/models/bivariate/mcmc.py:346-504, trivariate/mcmc.py:465-657).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "internal.h"
#include "kernels.h"
#include "philox.h"

using namespace clv;

namespace {

thread_local std::string g_err;

constexpr int PRIOR_DOUBLES = 81 + 81 + 27 + 9;  // V, cholV, A0B0, S0B
constexpr int GRAPH_CHUNK = 64;                  // sweeps per captured graph
constexpr int TIMING_EVENTS = 256;               // sweep launches timed per harvest

}  // namespace

int clv::fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

namespace {

HyperArgs hyper_args(clv_sampler* s, const double* units, int mode);

SweepArgs sweep_args(clv_sampler* s, int init, int fuse = 0) {
  SweepArgs a{};
  a.g = s->g;
  a.r.seed = s->cfg.seed;
  a.r.chain_first = s->cfg.chain_first;
  a.r.tape = s->d_tape;
  a.r.tape_sweep_stride = clv_replay_sweep_stride(s);
  a.r.tape_sweeps = s->tape_sweeps;
  a.x = s->d_x;
  a.tx = s->d_tx;
  a.T = s->d_T;
  a.cov = s->d_cov;
  a.log_s = s->d_logs;
  a.lam = s->d_lam;
  a.mu = s->d_mu;
  a.hyper = s->d_hyper;
  a.blockpart = s->d_block;
  a.pblock = s->d_pblock;
  a.ctrl = s->d_ctrl;
  a.level1 = s->d_level1;
  a.sums = s->d_sums;
  a.qstore = s->d_qstore;
  a.n_stored = nullptr;
  a.lam_init = s->prior.lam_init;
  a.init = init;
  a.fuse = fuse;
  a.chain_arrive = s->d_arrive;
  a.unit_arrive = s->d_arrive + s->g.n_chains;
  a.ctrl_rw = s->d_ctrl;
  a.hyp2 = s->d_hyp2;
  a.unitpart = s->d_unit;
  a.hvar_out = s->d_hvar;
  a.stamps = s->d_stamps;
  a.mail = s->d_mail;
  a.peers = s->d_peers;
  a.wg_map = s->d_wgmap;
  a.rank = s->cfg.rank;
  a.lam_out = s->d_lam_alt ? s->d_lam_alt : s->d_lam;
  a.mu_out = s->d_mu_alt ? s->d_mu_alt : s->d_mu;
  a.hyper_out = s->d_hyper_alt ? s->d_hyper_alt : s->d_hyper;
  a.wait_ticks = s->wait_ticks;
  a.abort_host = s->d_h_abort;
  a.diag = s->d_diag;
  a.clk = s->d_clk;
  a.h = hyper_args(s, nullptr, 0);
  if (fuse) a.h.hvar = s->replay ? nullptr : s->d_hvar;
  return a;
}

HyperArgs hyper_args(clv_sampler* s, const double* units, int mode) {
  HyperArgs a{};
  a.g = s->g;
  a.r.seed = s->cfg.seed;
  a.r.chain_first = s->cfg.chain_first;
  a.r.tape = s->d_tape;
  a.r.tape_sweep_stride = clv_replay_sweep_stride(s);
  a.r.tape_sweeps = s->tape_sweeps;
  a.units = units ? units : s->d_unit;
  a.hyper = s->d_hyper;
  a.ctrl = s->d_ctrl;
  a.level2 = s->d_level2;
  a.loglik = s->d_loglik;
  a.V = s->d_prior;
  a.cholV = s->d_prior + 81;
  a.A0B0 = s->d_prior + 162;
  a.S0B = s->d_prior + 189;
  a.nu_n = s->prior.nu_n;
  a.omega2 = s->prior.omega2;
  a.mode = mode;
  a.stamps = s->d_stamps;
  // mode 0 follows a sweep kernel, which precomputed the draw's variates (if it had workgroups)
  a.hvar = (mode == 0 && !s->replay && s->g.nb_local > 0) ? s->d_hvar : nullptr;
  return a;
}

int enqueue_sweep(clv_sampler* s, hipEvent_t e0, hipEvent_t e1) {
  s->last_persist_n = 0;
  CLV_HIP(launch_sweep(sweep_args(s, 0), s->replay, s->stream, e0, e1));
  if (s->g.blocks_per_unit > 1) {
    GroupArgs ga{};
    ga.g = s->g;
    ga.blockpart = s->d_block;
    ga.unitpart = s->d_unit;
    CLV_HIP(launch_group(ga, s->stream));
  }
  return CLV_OK;
}

// world_size == 1: one launch per sweep (the level-2 draw runs in the sweep kernel's tail)
int enqueue_fused(clv_sampler* s, hipEvent_t e0, hipEvent_t e1) {
  s->last_persist_n = 0;
  CLV_HIP(launch_sweep(sweep_args(s, 0, 1), s->replay, s->stream, e0, e1));
  return CLV_OK;
}

int enqueue_hyper(clv_sampler* s, const double* units, int mode, hipEvent_t e0, hipEvent_t e1) {
  s->last_persist_n = 0;
  if (e0) CLV_HIP(hipEventRecord(e0, s->stream));
  CLV_HIP(launch_hyper(hyper_args(s, units, mode), s->replay, s->stream));
  if (e1) CLV_HIP(hipEventRecord(e1, s->stream));
  return CLV_OK;
}

int check_replay_range(clv_sampler* s, int64_t n_more) {
  if (!s->replay) return CLV_OK;
  const int64_t need = s->sweeps_done + n_more + (s->g.D == 2 ? 1 : 0);
  if (!s->d_tape || need > s->tape_sweeps)
    return fail(CLV_ESTATE, "replay tape too short: need " + std::to_string(need) + " sweeps, have " +
                                std::to_string(s->tape_sweeps));
  return CLV_OK;
}

int harvest_timing(clv_sampler* s) {
  if (s->ev_used == 0) return CLV_OK;
  CLV_HIP(hipEventSynchronize(s->ev[4 * (s->ev_used - 1) + 1]));
  for (int k = 0; k < s->ev_used; ++k) {
    float ms = 0.f;
    CLV_HIP(hipEventElapsedTime(&ms, s->ev[4 * k], s->ev[4 * k + 1]));
    s->t_sweep_ms += ms;  // fused: the level-2 draw is inside the timed launch
    s->n_sweep_timed += s->ev_sweeps.empty() ? 1 : s->ev_sweeps[k];  // persistent: many sweeps
  }
  s->ev_used = 0;
  return CLV_OK;
}

int ensure_events(clv_sampler* s) {
  if (s->ev.empty()) {
    s->ev.resize(4 * TIMING_EVENTS);
    for (auto& e : s->ev) CLV_HIP(hipEventCreate(&e));
  }
  return CLV_OK;
}

int build_graph(clv_sampler* s, int n) {
  if (s->graph_exec && s->graph_sweeps == n) return CLV_OK;
  if (s->graph_exec) {
    CLV_HIP(hipGraphExecDestroy(s->graph_exec));
    s->graph_exec = nullptr;
  }
  hipGraph_t graph;
  CLV_HIP(hipStreamBeginCapture(s->stream, hipStreamCaptureModeThreadLocal));
  for (int k = 0; k < n; ++k) {
    int rc = enqueue_fused(s, nullptr, nullptr);
    if (rc != CLV_OK) {
      hipGraph_t dummy;
      (void)hipStreamEndCapture(s->stream, &dummy);
      return rc;
    }
  }
  CLV_HIP(hipStreamEndCapture(s->stream, &graph));
  CLV_HIP(hipGraphInstantiate(&s->graph_exec, graph, nullptr, nullptr, 0));
  CLV_HIP(hipGraphDestroy(graph));
  s->graph_sweeps = n;
  return CLV_OK;
}

bool is_pow2(int v) { return v > 0 && (v & (v - 1)) == 0; }

// Draws stored by the first `sweeps` sweeps (per chain): bi:402's condition, capped at n_draws.
int64_t stored_count(const clv_sampler* s, int64_t sweeps) {
  const Geometry& g = s->g;
  if (sweeps <= g.burnin || g.n_draws <= 0) return 0;
  return std::min<int64_t>((sweeps - 1 - g.burnin) / g.thin + 1, g.n_draws);
}

// Hand the level-1 draws completed since the last call to the copy pool (clv_stream_draws).
void stream_enqueue(clv_sampler* s) {
  if (!s->ds_dest || !s->d_level1) return;
  const Geometry& g = s->g;
  const int64_t k = stored_count(s, s->sweeps_done);
  if (k <= s->ds_next) return;
  const int64_t row = g.n * (g.D + 2);  // doubles per draw and chain
  for (int c = 0; c < g.n_chains; ++c) {
    const int64_t off = ((int64_t)c * g.n_draws + s->ds_next) * row;
    stream_copy(s->ds, s->device, s->d_level1 + off, s->ds_dest + off, sizeof(double) * (size_t)((k - s->ds_next) * row));
  }
  s->ds_next = k;
}

// Before the draws already streamed may be rewritten (the state is set back): wait for the copies in
// flight and stream again from the first draw the new sweep count has not stored.
void stream_rewind(clv_sampler* s) {
  if (!s->ds_dest) return;
  stream_wait(s->ds);
  s->ds_next = std::min(s->ds_next, stored_count(s, s->sweeps_done));
}

// The wait-timeout record of the last failed launch (kernels.hip report_wait) as text, and cleared
// for the next one; "" if no wave recorded one.
std::string take_wait_diag(clv_sampler* s) {
  if (!s->d_diag) return "";
  unsigned long long d[DIAG_WORDS] = {};
  if (hipMemcpy(d, s->d_diag, sizeof(d), hipMemcpyDeviceToHost) != hipSuccess) return "";
  (void)hipMemset(s->d_diag, 0, sizeof(d));
  if (!d[0]) return "";
  const Geometry& g = s->g;
  const char* what = d[1] == WAIT_HYPER ? "(beta, Sigma) hand-off slot"
                     : d[1] == WAIT_BLOCKS ? "block partial"
                     : d[1] == WAIT_P2P_MAIL ? "peer unit partial (persistent)" : "peer unit partial (fused)";
  std::string m = std::string(" [wait record: sweep ") + std::to_string((long long)d[2]) + ", chain " +
                  std::to_string(d[3]) + ", rank " + std::to_string(d[4]) + ": " + what + " ";
  const long long unit = (long long)d[5];
  if ((d[1] == WAIT_P2P_MAIL || d[1] == WAIT_FX_MAIL) && g.units_per_rank > 0 && unit >= 0)
    m += "unit " + std::to_string(unit) + " (rank " + std::to_string(unit / g.units_per_rank) + ", local unit " +
         std::to_string(unit % g.units_per_rank) + ")";
  else
    m += (d[1] == WAIT_HYPER ? "of block " : "") + std::to_string(unit);
  char bits[32];
  std::snprintf(bits, sizeof(bits), "%016llx", d[7]);
  m += " statistic " + std::to_string((long long)d[6]) + " still empty (bits " + bits + ") after " +
       std::to_string(d[8]) + " polls, " + std::to_string(d[9] / 100000.0) + " ms; " + std::to_string(d[10]) +
       " lanes of the wave missing";
  if (d[1] == WAIT_P2P_MAIL || d[1] == WAIT_FX_MAIL) {
    m += "; progress (sweep each rank's level-2 side last polled for):";
    for (int q = 0; q < std::min(g.world_size, 5); ++q)
      m += " " + std::to_string(q) + ":" + (d[11 + q] == ~0ull ? std::string("none") : std::to_string((long long)d[11 + q]));
  }
  return m + "]";
}

// CLV_WAIT_TIMEOUT_MS: a finite decimal number (surrounding blanks allowed; no hex, inf or nan),
// clamped to the range clv_set_wait_timeout accepts, [1 ms, 1 h].  distributed.run_wait_ms applies
// the same rule in Python.
bool parse_wait_ms(const char* txt, double* ms) {
  for (const char* c = txt; *c; ++c)
    if (*c == 'x' || *c == 'X' || *c == 'n' || *c == 'N' || *c == 'i' || *c == 'I') return false;
  char* end = nullptr;
  const double v = std::strtod(txt, &end);
  if (end == txt) return false;
  while (*end == ' ' || *end == '\t' || *end == '\n') ++end;
  if (*end || !(v == v) || v > 1e300 || v < -1e300) return false;
  *ms = std::min(3.6e6, std::max(1.0, v));
  return true;
}

}  // namespace

extern "C" {

int32_t clv_abi_version(void) { return CLV_ABI_VERSION; }

int32_t clv_default_blocks_per_unit(int64_t n_global) {
  // Keep the number of exchanged/reduced units <= 512 (one hyper workgroup sums them).
  const int64_t nb = (n_global + BLOCK - 1) / BLOCK;
  int32_t g = 1;
  while ((nb + g - 1) / g > 512) g *= 2;
  return g;
}

const char* clv_last_error(void) { return g_err.c_str(); }

int64_t clv_sizeof(int32_t which) {
  switch (which) {
    case 0: return (int64_t)sizeof(clv_config);
    case 1: return (int64_t)sizeof(clv_data);
    case 2: return (int64_t)sizeof(clv_prior);
    default: return -1;
  }
}

int clv_device_count(int32_t* count) {
  int n = 0;
  CLV_HIP(hipGetDeviceCount(&n));
  *count = n;
  return CLV_OK;
}

int64_t clv_replay_sweep_stride(const clv_sampler* s) {
  const int64_t n = s->g.n;
  return n * (2 + 3 * (int64_t)s->g.S + (s->g.D == 3 ? 1 : 0)) + TAPE_HYPER;
}

}  // extern "C"

// The persistent kernels spin on other workgroups of their grid, so every workgroup must be
// resident at once.  Admitted 256-thread blocks per CU (MI355X guide, "Residency and cooperative
// launch") = min(occupancy API, 8, floor(800 / (ceil(sgpr/16)*16 + 16))); the API answer is one
// high only where the SGPR term binds.  The persistent instances are VGPR-bound at 2 blocks per CU
// (129-256 VGPRs: 2 waves per SIMD) and their SGPR term is >= 6 even at the architectural maximum
// of 102 SGPRs, so it is applied at that maximum (never binding here) and a margin of one slot per
// 32 CUs guards against another kernel of the process holding slots.  c2 / c3: 376 of 512 slots;
// c4 at 8 ranks: 497 of 512 (504 allowed).  Every wait is bounded regardless.
bool clv::persist_grid_fits(int64_t grid_wgs, int blocks_per_cu, int n_cu) {
  constexpr int SGPR_MAX = 102;
  const int sgpr_term = 800 / (((SGPR_MAX + 15) / 16) * 16 + 16);
  const int64_t per_cu = std::min({blocks_per_cu, 8, sgpr_term});
  const int64_t slots = per_cu * n_cu;
  const int64_t margin = std::max(1, n_cu / 32);
  return grid_wgs > 0 && slots > 0 && grid_wgs <= slots - margin;
}

// Whether the persistent kernel is worth running a resident grid of grid_wgs workgroups (world size
// 1 and the peer exchange).  Round 4 measured it losing to the launch-per-sweep kernel once most CUs
// held two of its workgroups (c4's 8-rank shard, 1 chain x 497 workgroups: 43.8 vs 22.4 us per sweep)
// and capped it by density.  The cause was not the doubled SIMDs: the level-2 workgroup emptied its
// chain's hand-off slots lane-per-block (one double of a different line per lane and instruction), and
// at ~500 blocks those ~7k partial-line write-throughs queued ahead of its draw (the draw measured 9.2
// us of a 20 us sweep, profiles/r06_c4shard8_stamps_*.txt).  With coalesced resets (round 6) the
// persistent kernel wins at every measured point (tools/persist_crossover.py,
// profiles/r06_persist_crossover*.jsonl; us per sweep persistent / launch-per-sweep, workgroups per CU):
//   bivariate, 4 chains  K=2: 1.25 10.1 / 17.1, 1.61 9.8 / 18.2, 1.73 9.9 / 18.3, 1.86 10.3 / 19.0
//                        K=5: 1.25 10.4 / 18.5, 1.61 10.1 / 19.5
//   bivariate, 1-2 chains K=2: 0.92 7.2 / 15.2, 1.38 10.1 / 17.6, 1.68 10.3 / 18.3, 2 chains 1.84
//                        10.6 / 19.0; K=5: 0.92 9.2 / 16.6, 1.38 12.6 / 18.7, 1.68 13.8 / 19.6,
//                        1.91 14.1 / 20.3 (c4 at 8 ranks); K=9: 0.92 12.8 / 18.4, 1.38 16.9 / 22.5
//   trivariate, 4 chains K=3: 1.25 10.8 / 19.7, 1.61 11.5 / 20.7; 1 chain K=3: 1.38 14.6 / 19.6,
//                        1.68 15.6 / 20.6; K=9 (its persistent instance spills): 0.92 20.1 / 20.8
// So: wherever the grid fits (persist_grid_fits).  Kept as a function: the CPU test pins the choice.
// Instances whose private segment (spills) exceeds this many bytes per lane are never run
// persistently: the trivariate K = 9 peer instance (768 B per lane) at world 2 on one card left 39 of
// a chain's 40 customer workgroups undispatched until its 10 s wait bound (round 6) — the runtime
// provisions scratch for a limited number of waves, and a persistent grid must be resident whole.
// Every instance a BASELINE configuration selects is at or below it: world size 1 0 B (bivariate K <=
// 8, trivariate K <= 4), peer c2-tiled <2,2> 0 B, c4 at 8 ranks <2,5> 56 B, <3,3> 48 B (the tests'
// world-3 trivariate run).  (llvm-readelf --notes: .private_segment_fixed_size.)
constexpr size_t PERSIST_SCRATCH_MAX = 64;

bool clv::persist_worth(int D, int K, int n_chains, int64_t grid_wgs, int n_cu) {
  (void)D, (void)K, (void)n_chains;
  return n_cu > 0 && grid_wgs > 0;
}

namespace {

// Persistent grid: which (chain, block) each dispatched workgroup runs.  The grid has more
// workgroups (T = chains x (blocks + 1)) than CUs, and the dispatcher fills every CU once before
// doubling up: linear workgroup i < T - n_cu shares its CU with workgroup i + n_cu (measured,
// tools/placement.py).  A SIMD holding two customer waves runs each at ~0.68 of its solo speed,
// and the hardware favours the older wave; pairing two waves of DIFFERENT chains lets the older
// chain run ahead while the younger one crawls, and the run lasts until the slowest chain ends.
// So shared CUs pair workgroups of the SAME chain (every chain then paces at its pairs' rate), each
// chain's level-2 workgroup (asleep most of the time) shares a CU with one of its own customer
// workgroups, and the pairs are spread evenly over the chains.  Pure placement: every workgroup
// still runs one logical (chain, block), so results do not depend on it.
// Chains of at least CLV_L2_ALONE_MIN_NB blocks (the level-2 workgroup's lanes then poll two blocks
// each) place their level-2 workgroup on a CU of its own: c4's 8-rank shard (496 blocks, 1 chain)
// 13.54 -> 12.88 us per sweep; c2 (93 blocks per chain) 9.86 -> 9.80, within the noise, so it keeps
// the pairing (profiles/r06_ab_l2alone.txt).
#ifndef CLV_L2_ALONE_MIN_NB
#define CLV_L2_ALONE_MIN_NB 256
#endif
std::vector<int32_t> persist_wg_map(int C, int nb, int n_cu) {
  const int per = nb + 1;  // workgroups per chain (block nb = the level-2 workgroup)
  const int T = C * per;
  std::vector<int32_t> map(T);
  for (int c = 0; c < C; ++c)  // identity: blockIdx = (b, c)
    for (int b = 0; b < per; ++b) map[c * per + b] = (c << 16) | b;
  const int P = T - n_cu;  // shared CUs
  if (P <= 0 || T > 2 * n_cu) return map;
  std::vector<std::vector<int>> todo(C);  // customer blocks of each chain still to place
  for (int c = 0; c < C; ++c)
    for (int b = nb - 1; b >= 0; --b) todo[c].push_back(b);
  std::vector<int32_t> first, second, single;
  int p = 0;
  const bool l2_alone = nb >= CLV_L2_ALONE_MIN_NB;
  for (int c = 0; !l2_alone && c < C && p < P; ++c, ++p) {  // level-2 workgroup + one own customer workgroup
    first.push_back((c << 16) | nb);
    if (todo[c].empty()) return map;
    second.push_back((c << 16) | todo[c].back());
    todo[c].pop_back();
  }
  const int n_l2_paired = (int)first.size();
  const bool l2_paired = n_l2_paired == C;
  for (int c = 0; p < P; c = (c + 1) % C) {  // same-chain customer pairs, round robin over chains
    bool any = false;
    for (int k = 0; k < C && !any; ++k) any = todo[(c + k) % C].size() >= 2;
    if (!any) return map;  // cannot pair within chains: keep the identity
    if (todo[c].size() < 2) continue;
    first.push_back((c << 16) | todo[c].back());
    todo[c].pop_back();
    second.push_back((c << 16) | todo[c].back());
    todo[c].pop_back();
    ++p;
  }
  for (int c = 0; c < C; ++c) {
    if (!l2_paired && c >= n_l2_paired) single.push_back((c << 16) | nb);
    while (!todo[c].empty()) {
      single.push_back((c << 16) | todo[c].back());
      todo[c].pop_back();
    }
  }
  // interleave the chains over the single slots (so that each chain spreads over all XCDs)
  std::vector<int32_t> sorted_single;
  for (size_t k = 0; sorted_single.size() < single.size(); ++k)
    for (int c = 0; c < C; ++c) {
      size_t seen = 0;
      for (int32_t v : single)
        if ((v >> 16) == c && seen++ == k) sorted_single.push_back(v);
    }
  if ((int)first.size() != P || (int)sorted_single.size() != n_cu - P) return map;
  for (int i = 0; i < P; ++i) {
    map[i] = first[i];
    map[n_cu + i] = second[i];
  }
  for (int i = 0; i < n_cu - P; ++i) map[P + i] = sorted_single[i];
  return map;
}

}  // namespace

extern "C" {

int clv_create(const clv_config* cfg, const clv_data* data, const clv_prior* prior, clv_sampler** out) {
  if (!cfg || !data || !prior || !out) return fail(CLV_EINVAL, "null argument");
  *out = nullptr;
  if (cfg->abi_version != CLV_ABI_VERSION) return fail(CLV_EINVAL, "ABI version mismatch");
  if (cfg->D != 2 && cfg->D != 3) return fail(CLV_EINVAL, "D must be 2 or 3");
  if (cfg->K < 1 || cfg->K > CLV_MAX_K) return fail(CLV_EINVAL, "K must be in 1..9");
  if (cfg->n_mh_steps < 0) return fail(CLV_EINVAL, "n_mh_steps must be >= 0");
  if (cfg->thin < 1) return fail(CLV_EINVAL, "thin must be >= 1");
  if (cfg->burnin < 0 || cfg->mcmc < 0) return fail(CLV_EINVAL, "burnin/mcmc must be >= 0");
  if (cfg->n_chains < 1) return fail(CLV_EINVAL, "n_chains must be >= 1");
  if (cfg->rng_mode != CLV_RNG_PHILOX && cfg->rng_mode != CLV_RNG_REPLAY) return fail(CLV_EINVAL, "bad rng_mode");
  if (cfg->draw_sink < CLV_SINK_FULL || cfg->draw_sink > CLV_SINK_SUMMARY_PCT) return fail(CLV_EINVAL, "bad draw_sink");
  if (data->n < 0) return fail(CLV_EINVAL, "n must be >= 0");
  if (cfg->n_global > 0xffffffffLL) return fail(CLV_EINVAL, "n_global must fit the 32-bit Philox customer counter");
  if (cfg->n_global < data->n || cfg->n_global < 1) return fail(CLV_EINVAL, "n_global must be >= n >= 0 and > 0");
  if (cfg->world_size < 1 || cfg->rank < 0 || cfg->rank >= cfg->world_size) return fail(CLV_EINVAL, "bad rank/world_size");
  if (cfg->D == 3 && data->n > 0 && !data->log_s) return fail(CLV_EINVAL, "D == 3 needs log_s");
  if (cfg->K > 1 && data->n > 0 && !data->covariates) return fail(CLV_EINVAL, "K > 1 needs covariates");
  if (data->n > 0 && (!data->x || !data->t_x || !data->T_cal)) return fail(CLV_EINVAL, "missing CBS column");
  if (cfg->rng_mode == CLV_RNG_REPLAY && cfg->world_size != 1) return fail(CLV_EINVAL, "replay needs world_size 1");

  const int32_t bpu = cfg->blocks_per_unit ? cfg->blocks_per_unit : clv_default_blocks_per_unit(cfg->n_global);
  if (!is_pow2(bpu)) return fail(CLV_EINVAL, "blocks_per_unit must be a power of two");
  const int nb_local = (int)((data->n + BLOCK - 1) / BLOCK);
  int32_t bpr = cfg->blocks_per_rank;
  if (bpr == 0) {
    if (cfg->world_size != 1) return fail(CLV_EINVAL, "blocks_per_rank required when sharded");
    bpr = ((std::max(nb_local, 1) + bpu - 1) / bpu) * bpu;
  }
  if (bpr % bpu) return fail(CLV_EINVAL, "blocks_per_rank must be a multiple of blocks_per_unit");
  if (nb_local > bpr) return fail(CLV_EINVAL, "shard larger than blocks_per_rank * CLV_BLOCK");
  if (cfg->shard_begin != (int64_t)cfg->rank * bpr * BLOCK) return fail(CLV_EINVAL, "shard_begin != rank * blocks_per_rank * CLV_BLOCK");
  const int64_t nb_global = (cfg->n_global + BLOCK - 1) / BLOCK;
  if ((int64_t)bpr * cfg->world_size < nb_global) return fail(CLV_EINVAL, "shards do not cover n_global");

  auto* s = new clv_sampler();
  s->cfg = *cfg;
  s->cfg.blocks_per_rank = bpr;
  s->cfg.blocks_per_unit = bpu;
  s->prior = *prior;
  s->replay = cfg->rng_mode == CLV_RNG_REPLAY;

  Geometry& g = s->g;
  g.D = cfg->D;
  g.K = cfg->K;
  g.S = cfg->n_mh_steps;
  g.n_chains = cfg->n_chains;
  g.n = data->n;
  g.n_global = cfg->n_global;
  g.shard_begin = cfg->shard_begin;
  g.nb_local = nb_local;
  g.blocks_per_rank = bpr;
  g.blocks_per_unit = bpu;
  g.units_per_rank = bpr / bpu;
  g.n_units_global = (nb_global + bpu - 1) / bpu;
  g.world_size = cfg->world_size;
  g.stride = cfg->K * cfg->D + cfg->D * (cfg->D + 1) / 2 + 1;
  g.burnin = cfg->burnin;
  g.mcmc = cfg->mcmc;
  g.thin = cfg->thin;
  g.n_draws = cfg->mcmc >= 1 ? (cfg->mcmc - 1) / cfg->thin + 1 : 0;
  g.l2w = cfg->D * cfg->K + cfg->D * (cfg->D + 1) / 2;

  auto cleanup_fail = [&](int rc) {
    clv_destroy(s);
    return rc;
  };
#define CLV_HIPC(expr)                                                                            \
  do {                                                                                            \
    hipError_t e_ = (expr);                                                                       \
    if (e_ != hipSuccess)                                                                         \
      return cleanup_fail(fail(CLV_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)));    \
  } while (0)

  if (cfg->device >= 0) CLV_HIPC(hipSetDevice(cfg->device));
  CLV_HIPC(hipGetDevice(&s->device));
  if (cfg->stream) {
    s->stream = (hipStream_t)(uintptr_t)cfg->stream;
  } else {
    CLV_HIPC(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
    s->own = s->stream;
    s->own_stream = true;
  }

  const int64_t n = g.n, C = g.n_chains;
  CLV_HIPC(dalloc(&s->d_x, std::max<int64_t>(n, 1)));
  CLV_HIPC(dalloc(&s->d_tx, std::max<int64_t>(n, 1)));
  CLV_HIPC(dalloc(&s->d_T, std::max<int64_t>(n, 1)));
  if (g.K > 1) CLV_HIPC(dalloc(&s->d_cov, (size_t)(g.K - 1) * std::max<int64_t>(n, 1)));
  if (g.D == 3) CLV_HIPC(dalloc(&s->d_logs, std::max<int64_t>(n, 1)));
  CLV_HIPC(dalloc(&s->d_clk, 2 * CLK_RING));
  CLV_HIPC(hipMemsetAsync(s->d_clk, 0, sizeof(unsigned long long) * 2 * CLK_RING, s->stream));
  CLV_HIPC(dalloc(&s->d_lam, C * std::max<int64_t>(n, 1)));
  CLV_HIPC(dalloc(&s->d_mu, C * std::max<int64_t>(n, 1)));
  CLV_HIPC(dalloc(&s->d_hyper, C * HS));
  CLV_HIPC(dalloc(&s->d_block, (size_t)C * bpr * g.stride));
  if (bpu > 1) CLV_HIPC(dalloc(&s->d_unit, (size_t)C * g.units_per_rank * g.stride));
  else s->d_unit = s->d_block;
  CLV_HIPC(dalloc(&s->d_prior, PRIOR_DOUBLES));
  CLV_HIPC(dalloc(&s->d_ctrl, 1));
  CLV_HIPC(dalloc(&s->d_arrive, C + C * (int64_t)g.units_per_rank));  // chain, then unit counters
  CLV_HIPC(dalloc(&s->d_hvar, 2 * C * HV));
  CLV_HIPC(dalloc(&s->d_hyp2, 2 * C * HS));
  // Persistent sweeps (one launch runs many sweeps) when every workgroup of the grid can be
  // resident at once — the chain hand-off spins on the other workgroups (CLV_PERSISTENT=0 opts out)
  if (!s->replay && cfg->world_size == 1 && nb_local > 0 && bpu == 1 && nb_local <= 2 * BLOCK) {
    const char* env = std::getenv("CLV_PERSISTENT");
    hipDeviceProp_t prop{};
    size_t scratch = SIZE_MAX;  // (a failed query: never persistent)
    if (persist_occupancy(g.D, g.K, false, &s->persist_bpc) == hipSuccess &&
        persist_scratch_bytes(g.D, g.K, false, &scratch) == hipSuccess &&
        hipGetDeviceProperties(&prop, s->device) == hipSuccess)
      s->n_cu = prop.multiProcessorCount;
    // CLV_PERSISTENT: "0" never, "1" whenever the grid fits (tests, A/B), unset: where it pays;
    // an instance that spills more than PERSIST_SCRATCH_MAX bytes per lane only when forced (tests)
    const int64_t grid = (int64_t)(nb_local + 1) * C;
    const bool force = env && std::string(env) == "1";
    if ((!env || std::string(env) != "0") && (force || scratch <= PERSIST_SCRATCH_MAX) && persist_grid_fits(grid, s->persist_bpc, s->n_cu) &&
        (force || persist_worth(g.D, g.K, (int)C, grid, s->n_cu)))
      s->persistent = true;
  }
  // World size > 1: the same persistent kernel exchanging unit partials with its peers over xGMI
  // (clv_p2p_connect) when the grid fits at once here, as above, and on every rank (the caller
  // checks that all ranks are capable before connecting).
  if (!s->replay && cfg->world_size > 1 && cfg->world_size <= MAX_WORLD && nb_local > 0 && nb_local <= 2 * BLOCK && g.n_units_global <= 2 * BLOCK &&
      bpu <= 64 && (int64_t)g.stride * ((nb_local + bpu - 1) / bpu) <= UMAIL) {
    hipDeviceProp_t prop{};
    size_t scratch = SIZE_MAX;  // (a failed query: never persistent)
    if (persist_occupancy(g.D, g.K, true, &s->persist_bpc) == hipSuccess &&
        persist_scratch_bytes(g.D, g.K, true, &scratch) == hipSuccess &&
        hipGetDeviceProperties(&prop, s->device) == hipSuccess)
      s->n_cu = prop.multiProcessorCount;
    const char* env = std::getenv("CLV_PERSISTENT");  // "0": the fused exchange below instead
    const int64_t grid = (int64_t)(nb_local + 1) * C;
    const bool force = env && std::string(env) == "1";
    if ((!env || std::string(env) != "0") && (force || scratch <= PERSIST_SCRATCH_MAX) && persist_grid_fits(grid, s->persist_bpc, s->n_cu) &&
        (force || persist_worth(g.D, g.K, (int)C, grid, s->n_cu)))
      s->p2p_capable = s->p2p_persist_fits = true;
  }
  // Any other shard: the sweep kernel's fused level-2 tail exchanges through the same mail (one
  // launch per sweep, no host collective; n_units_global <= 2 CLV_BLOCK as its readers assume)
  if (!s->replay && cfg->world_size > 1 && cfg->world_size <= MAX_WORLD && g.n_units_global <= 2 * BLOCK)
    s->fx_capable = true;
  if (s->p2p_capable || s->fx_capable) {
    // the slots, then one progress word per rank (MAIL_TAIL)
    const int64_t nm = mail_slots(g.world_size, (int)C, g.stride, g.units_per_rank) + MAIL_TAIL;
    // The mail is written by OTHER GPUs (system-scope write-through stores over xGMI) while this
    // GPU polls it.  Uncached device memory (MTYPE UC: every access of every agent goes to memory,
    // no L2 line of this GPU can hold a stale copy of a peer's store); fine-grained, then plain
    // device memory if the allocator refuses (CLV_MAIL_ALLOC = uncached | fine | default selects)
    {
      const char* env = std::getenv("CLV_MAIL_ALLOC");
      const std::string want = env ? env : "uncached";
      const unsigned flags[3] = {hipDeviceMallocUncached, hipDeviceMallocFinegrained, hipDeviceMallocDefault};
      const int first = want == "fine" ? 1 : want == "default" ? 2 : 0;
      for (int k = first; k < 3 && !s->d_mail; ++k) {
        void* p = nullptr;
        if (hipExtMallocWithFlags(&p, sizeof(double) * (size_t)nm, flags[k]) == hipSuccess && p) {
          s->d_mail = (double*)p;
          s->mail_kind = k;
        } else {
          (void)hipGetLastError();
        }
      }
      if (!s->d_mail) return cleanup_fail(fail(CLV_ENOMEM, "peer mail buffer"));
    }
    CLV_HIPC(hipMemsetAsync(s->d_mail, 0xFF, sizeof(double) * nm, s->stream));  // every slot empty
    CLV_HIPC(dalloc(&s->d_peers, g.world_size));
  }
  if (s->persistent || s->p2p_capable || s->fx_capable) {  // (fused exchange: the snapshot buffers)
    CLV_HIPC(dalloc(&s->d_pblock, (size_t)C * std::max(nb_local, 1) * g.stride));
    if (s->persistent) {  // deferred level-2 draws (CLV_DEFER=0: every launch draws its last one)
      const char* env = std::getenv("CLV_DEFER");
      s->defer = !(env && std::string(env) == "0");
      if (s->defer) CLV_HIPC(dalloc(&s->d_pend, (size_t)2 * C * g.stride));
    }
    CLV_HIPC(dalloc(&s->d_lam_alt, C * std::max<int64_t>(n, 1)));
    CLV_HIPC(dalloc(&s->d_mu_alt, C * std::max<int64_t>(n, 1)));
    CLV_HIPC(dalloc(&s->d_hyper_alt, C * HS));
    if ((cfg->draw_sink == CLV_SINK_SUMMARY || cfg->draw_sink == CLV_SINK_SUMMARY_PCT) && n > 0)
      CLV_HIPC(dalloc(&s->d_sums_prev, (size_t)C * CLV_N_SUM_STATS * n));
    CLV_HIPC(dalloc(&s->d_diag, DIAG_WORDS));
    CLV_HIPC(hipMemsetAsync(s->d_diag, 0, sizeof(unsigned long long) * DIAG_WORDS, s->stream));
    CLV_HIPC(hipHostMalloc((void**)&s->h_abort, sizeof(uint32_t), hipHostMallocMapped));
    *s->h_abort = 0;
    CLV_HIPC(hipHostGetDevicePointer((void**)&s->d_h_abort, s->h_abort, 0));
    // every wait of the persistent kernel is bounded: 2 s at world size 1 (all workgroups are
    // resident, so a wait that long means a fault), 10 s with peers (host-side launch skew between
    // ranks); CLV_WAIT_TIMEOUT_MS overrides
    double ms = cfg->world_size > 1 ? 10000.0 : 2000.0;
    if (const char* env = std::getenv("CLV_WAIT_TIMEOUT_MS")) {
      if (!parse_wait_ms(env, &ms))
        return cleanup_fail(fail(CLV_EINVAL, "CLV_WAIT_TIMEOUT_MS must be a finite decimal number of ms"));
    }
    s->wait_ticks = (uint64_t)(ms * 1e5);  // s_memrealtime: 100 MHz
  }
  if ((s->persistent || s->p2p_capable) && s->n_cu > 0) {
    // same-chain pairs on shared CUs, bivariate and trivariate: with the MH-phase wave priority
    // (kernels.hip persist_kernel) measured c2 10.70 -> 9.58 us per sweep against no map, c3 11.45 ->
    // 11.1 (chain pairs c / c + 2 instead: c2 10.16, c3 11.1; profiles/r05_ab_priority.txt)
    {
      std::vector<int32_t> map = persist_wg_map((int)C, (int)nb_local, s->n_cu);
      CLV_HIPC(dalloc(&s->d_wgmap, map.size()));
      CLV_HIPC(hipMemcpy(s->d_wgmap, map.data(), sizeof(int32_t) * map.size(), hipMemcpyHostToDevice));
    }
  }
#ifdef CLV_STAMPS
  {
    std::vector<unsigned long long> st(1024 * 8 + 12 * (size_t)C * (std::max(nb_local, 1) + 1), 0ull);
    for (int i = 0; i < 1024; ++i) st[i * 8 + 0] = st[i * 8 + 4] = ~0ull;
    CLV_HIPC(dalloc(&s->d_stamps, st.size()));
    CLV_HIPC(hipMemcpy(s->d_stamps, st.data(), st.size() * sizeof(unsigned long long), hipMemcpyHostToDevice));
  }
#endif
  CLV_HIPC(hipMemsetAsync(s->d_hvar, 0, sizeof(double) * 2 * C * HV, s->stream));
  CLV_HIPC(hipMemsetAsync(s->d_arrive, 0, sizeof(uint32_t) * (C + C * (int64_t)g.units_per_rank), s->stream));
  CLV_HIPC(dalloc(&s->d_bs, C * (CLV_MAX_K * CLV_MAX_D + CLV_MAX_D * CLV_MAX_D)));
  if (g.n_draws > 0) {
    CLV_HIPC(dalloc(&s->d_level2, (size_t)C * g.n_draws * g.l2w));
    CLV_HIPC(dalloc(&s->d_loglik, (size_t)C * g.n_draws));
    CLV_HIPC(hipMemsetAsync(s->d_level2, 0, sizeof(double) * C * g.n_draws * g.l2w, s->stream));
    CLV_HIPC(hipMemsetAsync(s->d_loglik, 0, sizeof(double) * C * g.n_draws, s->stream));
    if (cfg->draw_sink == CLV_SINK_FULL && n > 0) {
      const size_t bytes = sizeof(double) * (size_t)C * g.n_draws * n * (g.D + 2);
      CLV_HIPC(dalloc(&s->d_level1, bytes / sizeof(double)));
      CLV_HIPC(hipMemsetAsync(s->d_level1, 0, bytes, s->stream));
    }
  }
  if ((cfg->draw_sink == CLV_SINK_SUMMARY || cfg->draw_sink == CLV_SINK_SUMMARY_PCT) && n > 0) {
    CLV_HIPC(dalloc(&s->d_sums, (size_t)C * CLV_N_SUM_STATS * n));
    CLV_HIPC(hipMemsetAsync(s->d_sums, 0, sizeof(double) * C * CLV_N_SUM_STATS * n, s->stream));
  }
  if (cfg->draw_sink == CLV_SINK_SUMMARY_PCT && n > 0 && g.n_draws > 0) {
    const size_t nq = (size_t)C * g.n_draws * n;
    if (hipMalloc((void**)&s->d_qstore, sizeof(float2) * nq) != hipSuccess) {
      (void)hipGetLastError();
      s->d_qstore = nullptr;
      return cleanup_fail(fail(CLV_ENOMEM, "percentile store: " + std::to_string(sizeof(float2) * nq) +
                                               " bytes of device memory not available"));
    }
    CLV_HIPC(hipMemsetAsync(s->d_qstore, 0, sizeof(float2) * nq, s->stream));
  }
  CLV_HIPC(hipMemsetAsync(s->d_block, 0, sizeof(double) * C * bpr * g.stride, s->stream));
  if (bpu > 1) CLV_HIPC(hipMemsetAsync(s->d_unit, 0, sizeof(double) * C * g.units_per_rank * g.stride, s->stream));
  CLV_HIPC(hipMemsetAsync(s->d_ctrl, 0, sizeof(Ctrl), s->stream));
  CLV_HIPC(hipMemsetAsync(s->d_hyper, 0, sizeof(double) * C * HS, s->stream));

  if (n > 0) {
    CLV_HIPC(hipMemcpyAsync(s->d_x, data->x, sizeof(int32_t) * n, hipMemcpyHostToDevice, s->stream));
    CLV_HIPC(hipMemcpyAsync(s->d_tx, data->t_x, sizeof(double) * n, hipMemcpyHostToDevice, s->stream));
    CLV_HIPC(hipMemcpyAsync(s->d_T, data->T_cal, sizeof(double) * n, hipMemcpyHostToDevice, s->stream));
    if (g.K > 1)
      CLV_HIPC(hipMemcpyAsync(s->d_cov, data->covariates, sizeof(double) * (g.K - 1) * n, hipMemcpyHostToDevice, s->stream));
    if (g.D == 3)
      CLV_HIPC(hipMemcpyAsync(s->d_logs, data->log_s, sizeof(double) * n, hipMemcpyHostToDevice, s->stream));
  }
  {
    std::vector<double> pr(PRIOR_DOUBLES, 0.0);
    const int K = g.K, D = g.D;
    for (int i = 0; i < K * K; ++i) {
      pr[i] = prior->V[i];
      pr[81 + i] = prior->chol_V[i];
    }
    for (int i = 0; i < K * D; ++i) pr[162 + i] = prior->A0B0[i];
    for (int i = 0; i < D * D; ++i) pr[189 + i] = prior->S0_B0A0B0[i];
    CLV_HIPC(hipMemcpyAsync(s->d_prior, pr.data(), sizeof(double) * PRIOR_DOUBLES, hipMemcpyHostToDevice, s->stream));
    CLV_HIPC(hipStreamSynchronize(s->stream));
  }

  // Initial state (bi:367-379, tri:488-504) and, for D == 2, the statistics of the first draw.
  if (n > 0) CLV_HIPC(launch_sweep(sweep_args(s, 1), false, s->stream));
  else CLV_HIPC(hipMemsetAsync(s->d_block, 0, sizeof(double) * C * bpr * g.stride, s->stream));
  if (bpu > 1) {
    GroupArgs ga{};
    ga.g = g;
    ga.blockpart = s->d_block;
    ga.unitpart = s->d_unit;
    if (n > 0) CLV_HIPC(launch_group(ga, s->stream));
  }
  if (g.D == 3) {
    std::vector<double> bs(C * (g.K * g.D + g.D * g.D));
    for (int c = 0; c < C; ++c) {
      double* o = bs.data() + c * (g.K * g.D + g.D * g.D);
      for (int i = 0; i < g.K * g.D; ++i) o[i] = prior->beta_init[i];
      for (int i = 0; i < g.D * g.D; ++i) o[g.K * g.D + i] = prior->sigma_init[i];
    }
    CLV_HIPC(hipMemcpyAsync(s->d_bs, bs.data(), sizeof(double) * bs.size(), hipMemcpyHostToDevice, s->stream));
    CLV_HIPC(launch_set_hyper(g.D, g.K, (int)C, s->d_hyper, s->d_bs, prior->omega2, s->replay, s->stream));
  } else {
    s->pending_init_hyper = true;
  }
  CLV_HIPC(hipStreamSynchronize(s->stream));
#undef CLV_HIPC
  *out = s;
  return CLV_OK;
}

void clv_destroy(clv_sampler* s) {
  if (!s) return;
  (void)hipSetDevice(s->device);
  if (s->stream) (void)hipStreamSynchronize(s->stream);
  if (s->ds) {  // no copy may still read the draws freed below
    stream_wait(s->ds);
    delete s->ds;
  }
  if (s->graph_exec) (void)hipGraphExecDestroy(s->graph_exec);
  for (auto e : s->ev) (void)hipEventDestroy(e);
  if (s->done_ev) (void)hipEventDestroy(s->done_ev);
  void* ptrs[] = {s->d_x, s->d_tx, s->d_T, s->d_cov, s->d_logs, s->d_lam, s->d_mu, s->d_hyper,
                  s->d_block, s->d_prior, s->d_ctrl, s->d_level1, s->d_level2, s->d_loglik,
                  s->d_sums, s->d_tape, s->d_bs, s->d_arrive, s->d_hvar, s->d_stamps};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (s->d_unit && s->d_unit != s->d_block) (void)hipFree(s->d_unit);
  if (s->d_hyp2) (void)hipFree(s->d_hyp2);
  for (void* p : {(void*)s->d_lam_alt, (void*)s->d_mu_alt, (void*)s->d_hyper_alt, (void*)s->d_sums_prev,
                  (void*)s->d_pblock, (void*)s->d_qstore, (void*)s->d_pend, (void*)s->d_diag,
                  (void*)s->d_clk})
    if (p) (void)hipFree(p);
  if (s->h_abort) (void)hipHostFree(s->h_abort);
  for (void* p : s->ipc_opened) (void)hipIpcCloseMemHandle(p);
  if (s->d_mail) (void)hipFree(s->d_mail);
  if (s->d_peers) (void)hipFree(s->d_peers);
  if (s->d_wgmap) (void)hipFree(s->d_wgmap);
  if (s->own_stream && s->own) (void)hipStreamDestroy(s->own);
  delete s;
}

int clv_set_replay_tape(clv_sampler* s, const double* tape, int64_t n_sweeps) {
  if (!s || !tape || n_sweeps < 1) return fail(CLV_EINVAL, "bad replay tape arguments");
  if (!s->replay) return fail(CLV_ESTATE, "sampler not created in replay mode");
  CLV_HIP(hipSetDevice(s->device));
  if (s->d_tape) CLV_HIP(hipFree(s->d_tape));
  s->d_tape = nullptr;
  const size_t count = (size_t)s->g.n_chains * n_sweeps * clv_replay_sweep_stride(s);
  CLV_HIP(dalloc(&s->d_tape, count));
  CLV_HIP(hipMemcpy(s->d_tape, tape, count * sizeof(double), hipMemcpyHostToDevice));
  s->tape_sweeps = n_sweeps;
  if (s->graph_exec) {
    CLV_HIP(hipGraphExecDestroy(s->graph_exec));
    s->graph_exec = nullptr;
  }
  return CLV_OK;
}

int clv_hyper(clv_sampler* s, const double* gathered) {
  if (!s) return fail(CLV_EINVAL, "null sampler");
  if (s->g.world_size > 1 && !gathered) return fail(CLV_EINVAL, "sharded hyper needs the gathered buffer");
  CLV_HIP(hipSetDevice(s->device));
  {
    int rc = persist_flush(s);
    if (rc) return rc;
  }
  if (s->pending_init_hyper) {
    int rc = check_replay_range(s, 0);
    if (rc) return rc;
    rc = enqueue_hyper(s, gathered, 1, nullptr, nullptr);
    if (rc) return rc;
    s->pending_init_hyper = false;
    return CLV_OK;
  }
  return enqueue_hyper(s, gathered, 0, nullptr, nullptr);
}

int clv_sweep(clv_sampler* s) {
  if (!s) return fail(CLV_EINVAL, "null sampler");
  if (s->pending_init_hyper) return fail(CLV_ESTATE, "bivariate: call clv_hyper once before the first sweep");
  CLV_HIP(hipSetDevice(s->device));
  int rc = persist_flush(s);
  if (rc) return rc;
  rc = check_replay_range(s, 1);
  if (rc) return rc;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (s->timing) {
    rc = ensure_events(s);
    if (rc) return rc;
    e0 = s->ev[4 * s->ev_used];
    e1 = s->ev[4 * s->ev_used + 1];
  }
  rc = enqueue_sweep(s, e0, e1);
  if (rc) return rc;
  if (s->timing && ++s->ev_used == TIMING_EVENTS) {
    rc = harvest_timing(s);
    if (rc) return rc;
  }
  s->sweeps_done++;
  return CLV_OK;
}

int clv_partials(clv_sampler* s, double** ptr, int64_t* n_doubles, int32_t* stride) {
  if (!s) return fail(CLV_EINVAL, "null sampler");
  if (ptr) *ptr = s->d_unit;
  if (n_doubles) *n_doubles = (int64_t)s->g.n_chains * s->g.units_per_rank * s->g.stride;
  if (stride) *stride = s->g.stride;
  return CLV_OK;
}

int clv_copy_partials(clv_sampler* s, void* dst) {
  if (!s || !dst) return fail(CLV_EINVAL, "null argument");
  CLV_HIP(hipSetDevice(s->device));
  const size_t bytes = sizeof(double) * (size_t)s->g.n_chains * s->g.units_per_rank * s->g.stride;
  CLV_HIP(hipMemcpyAsync(dst, s->d_unit, bytes, hipMemcpyDeviceToDevice, s->stream));
  return CLV_OK;
}

int clv_synchronize(clv_sampler* s) {
  if (!s) return fail(CLV_EINVAL, "null sampler");
  CLV_HIP(hipSetDevice(s->device));
  CLV_HIP(hipStreamSynchronize(s->stream));
  return CLV_OK;
}

int64_t clv_sweeps_done(const clv_sampler* s) { return s ? s->sweeps_done : -1; }

int clv_clock_ghz(clv_sampler* s, double* ghz) {
  if (!s || !ghz) return fail(CLV_EINVAL, "null argument");
  *ghz = 0.0;
  // the last clv_run's sweeps [first, end]: each slot is one workgroup's (delta s_memtime, delta
  // s_memrealtime) up to that sweep's publish; the last sweep's draw may be deferred (persistent
  // kernel), so it is left out; at most the last CLK_RING sweeps are kept
  const int64_t end = s->sweeps_done - 1;
  const int64_t first = std::max<int64_t>(s->clk_first, end - (CLK_RING - 1));
  if (!s->d_clk || s->clk_first < 1 || end < first) return CLV_OK;
  CLV_HIP(hipSetDevice(s->device));
  CLV_HIP(hipStreamSynchronize(s->stream));
  std::vector<unsigned long long> ring(2 * CLK_RING);
  CLV_HIP(hipMemcpy(ring.data(), s->d_clk, sizeof(unsigned long long) * ring.size(), hipMemcpyDeviceToHost));
  double dm = 0.0, dr = 0.0;
  for (int64_t q = first; q <= end; ++q) {
    dm += (double)ring[2 * (q % CLK_RING)];
    dr += (double)ring[2 * (q % CLK_RING) + 1];
  }
  if (dr > 0.0) *ghz = 0.1 * dm / dr;  // s_memrealtime: 100 MHz
  return CLV_OK;
}

int clv_launch_info(const clv_sampler* s, int64_t* out) {
  if (!s || !out) return fail(CLV_EINVAL, "null argument");
  out[0] = s->persistent ? 1 : 0;
  out[1] = s->persist_bpc;
  out[2] = s->n_cu;
  out[3] = (int64_t)(s->g.nb_local + (s->persistent ? 1 : 0)) * s->g.n_chains;
  out[4] = 0;  // (reserved: was the MH-variate producer / consumer chunks, removed in round 4)
  out[5] = 0;  // (reserved: was the stride kernel's grid, removed)
  return CLV_OK;
}

int clv_p2p_info(const clv_sampler* s, int64_t* out) {
  if (!s || !out) return fail(CLV_EINVAL, "null argument");
  out[0] = (s->p2p_capable || s->fx_capable) ? 1 : 0;
  out[4] = s->p2p_capable ? 1 : 0;
  out[1] = s->p2p_ready ? 1 : 0;
  out[2] = s->d_mail ? (int64_t)sizeof(double) * 2 * s->g.world_size * s->g.n_chains * s->g.stride * s->g.units_per_rank : 0;
  out[3] = (int64_t)(uintptr_t)s->d_mail;
  out[5] = s->d_mail ? s->mail_kind : -1;
  return CLV_OK;
}

int clv_p2p_export(clv_sampler* s, void* handle) {
  if (!s || !handle) return fail(CLV_EINVAL, "null argument");
  if (!s->p2p_capable && !s->fx_capable) return fail(CLV_ESTATE, "no peer exchange for this sampler (world size 1 or replay mode)");
  CLV_HIP(hipSetDevice(s->device));
  hipIpcMemHandle_t h;
  CLV_HIP(hipIpcGetMemHandle(&h, s->d_mail));
  std::memcpy(handle, &h, sizeof(h));
  return CLV_OK;
}

int clv_p2p_connect(clv_sampler* s, const void* handles, const uint64_t* ptrs) {
  if (!s || (!handles && !ptrs)) return fail(CLV_EINVAL, "null argument");
  if (!s->p2p_capable && !s->fx_capable) return fail(CLV_ESTATE, "no peer exchange for this sampler (world size 1 or replay mode)");
  CLV_HIP(hipSetDevice(s->device));
  CLV_HIP(hipStreamSynchronize(s->stream));
  if (s->p2p_ready || !s->ipc_opened.empty()) {  // reconnect (after a failed step): drop the old mappings
    s->p2p_ready = false;
    for (void* p : s->ipc_opened) (void)hipIpcCloseMemHandle(p);
    s->ipc_opened.clear();
  }
  {  // every slot of this rank's mail empty (a failed step may have left units of any rank there);
     // the caller synchronises the ranks after connecting, before any rank runs
    const int64_t nm = mail_slots(s->g.world_size, s->g.n_chains, s->g.stride, s->g.units_per_rank) + MAIL_TAIL;
    CLV_HIP(hipMemsetAsync(s->d_mail, 0xFF, sizeof(double) * nm, s->stream));
  }
  const int W = s->g.world_size, r = s->cfg.rank;
  std::vector<double*> peers(W, nullptr);
  for (int q = 0; q < W; ++q) {
    if (q == r) {
      peers[q] = s->d_mail;
    } else if (handles) {
      hipIpcMemHandle_t h;
      std::memcpy(&h, (const char*)handles + (size_t)q * sizeof(h), sizeof(h));
      void* p = nullptr;
      CLV_HIP(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
      s->ipc_opened.push_back(p);
      peers[q] = (double*)p;
    } else {
      peers[q] = (double*)(uintptr_t)ptrs[q];
    }
    if (!peers[q]) return fail(CLV_EINVAL, "null peer mail pointer");
  }
  CLV_HIP(hipMemcpy(s->d_peers, peers.data(), sizeof(double*) * W, hipMemcpyHostToDevice));
  CLV_HIP(hipStreamSynchronize(s->stream));  // the mail's sentinel fill has landed
  s->p2p_ready = true;
  return CLV_OK;
}

int clv_p2p_set_persistent(clv_sampler* s, int32_t on) {
  if (!s) return fail(CLV_EINVAL, "null sampler");
  if (on && !s->p2p_persist_fits) return fail(CLV_ESTATE, "the persistent peer exchange does not fit this shard's grid");
  if (!on && !s->fx_capable) return fail(CLV_ESTATE, "no fused peer exchange for this sampler");
  CLV_HIP(hipSetDevice(s->device));
  CLV_HIP(hipStreamSynchronize(s->stream));
  s->p2p_capable = on != 0;
  s->last_persist_n = 0;  // (a rollback undoes a call of the path that ran it)
  return CLV_OK;
}

int clv_p2p_disconnect(clv_sampler* s) {
  if (!s) return fail(CLV_EINVAL, "null sampler");
  CLV_HIP(hipSetDevice(s->device));
  CLV_HIP(hipStreamSynchronize(s->stream));
  s->p2p_ready = false;
  for (void* p : s->ipc_opened) (void)hipIpcCloseMemHandle(p);
  s->ipc_opened.clear();
  if (s->d_peers) CLV_HIP(hipMemset(s->d_peers, 0, sizeof(double*) * s->g.world_size));
  return CLV_OK;
}

int clv_set_wait_timeout(clv_sampler* s, double ms) {
  if (!s || !(ms >= 1.0) || ms > 3.6e6) return fail(CLV_EINVAL, "wait timeout must be in [1 ms, 1 h]");
  s->wait_ticks = (uint64_t)(ms * 1e5);  // s_memrealtime: 100 MHz
  if (s->graph_exec) {  // captured with the previous bound (kernel arguments)
    CLV_HIP(hipGraphExecDestroy(s->graph_exec));
    s->graph_exec = nullptr;
  }
  return CLV_OK;
}

int clv_set_stream(clv_sampler* s, uint64_t stream) {
  if (!s || !stream) return fail(CLV_EINVAL, "bad arguments");
  if (s->graph_exec) {
    CLV_HIP(hipGraphExecDestroy(s->graph_exec));  // captured on the previous stream
    s->graph_exec = nullptr;
  }
  s->stream = (hipStream_t)(uintptr_t)stream;  // caller-owned from now on
  return CLV_OK;
}

int clv_note_sweeps(clv_sampler* s, int64_t n) {
  if (!s || s->sweeps_done + n < 0) return fail(CLV_EINVAL, "bad arguments");
  s->sweeps_done += n;
  s->last_persist_n = 0;
  return CLV_OK;
}

}  // extern "C"

// Persistent path: one launch of persist_kernel for all n sweeps (see kernels.hip), in two halves
// so that a group of shards in one process (group.hip) can have every shard's launch in flight
// before waiting for any.
static inline int64_t host_now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int clv::persist_launch(clv_sampler* s, int64_t n_sweeps) {
  const Geometry& g = s->g;
  s->last_persist_n = 0;
  s->inflight_n = 0;
  if (n_sweeps == 0) return CLV_OK;
  if (s->slots_dirty) {  // a completed launch leaves every hand-off slot empty; else fill them
    // every hand-off slot empty (all-ones bytes: the sentinel NaN)
    CLV_HIP(hipMemsetAsync(s->d_hyp2, 0xFF, sizeof(double) * 2 * g.n_chains * HS, s->stream));
    CLV_HIP(hipMemsetAsync(s->d_pblock, 0xFF, sizeof(double) * g.n_chains * g.nb_local * g.stride, s->stream));
    s->slots_dirty = false;
  }
  const size_t sums_bytes = sizeof(double) * (size_t)g.n_chains * CLV_N_SUM_STATS * g.n;
  if (s->d_sums_prev)  // an aborted (or rolled-back) launch restores the running sums from here
    CLV_HIP(hipMemcpyAsync(s->d_sums_prev, s->d_sums, sums_bytes, hipMemcpyDeviceToDevice, s->stream));
  SweepArgs a = sweep_args(s, 0, 1);
  const int64_t stride_c = (int64_t)g.n_chains * g.stride;
  a.pend_in = s->pend ? s->d_pend + s->pend_buf * stride_c : nullptr;
  a.pend_out = s->defer ? s->d_pend + (s->pend_buf ^ 1) * stride_c : nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (s->timing) {
    int rc = ensure_events(s);
    if (rc) return rc;
    e0 = s->ev[4 * s->ev_used];
    e1 = s->ev[4 * s->ev_used + 1];
    if (s->ev_sweeps.size() < TIMING_EVENTS) s->ev_sweeps.assign(TIMING_EVENTS, 1);
    s->ev_sweeps[s->ev_used] = n_sweeps;
  }
  // timed launches: events recorded around the launch (measured 0.4-0.7 us per step less host cost
  // on the driver's 20-sweep run than the dispatch's own timestamps, same duration to 0.2%)
  if (e0) CLV_HIP(hipEventRecord(e0, s->stream));
  s->host_ns[2] = host_now_ns();
  CLV_HIP(launch_persist(a, s->sweeps_done + 1, n_sweeps, s->stream, nullptr, nullptr));
  s->host_ns[3] = host_now_ns();
  if (e1) CLV_HIP(hipEventRecord(e1, s->stream));
  // the launch's end event; timed launches are harvested later (clv_kernel_time or a full slot set)
  s->inflight_done = e1;
  if (s->timing) {
    if (++s->ev_used == TIMING_EVENTS) {
      int rc = harvest_timing(s);
      if (rc) return rc;
    }
  } else {
    if (!s->done_ev) CLV_HIP(hipEventCreateWithFlags(&s->done_ev, hipEventDisableTiming));
    CLV_HIP(hipEventRecord(s->done_ev, s->stream));
    s->inflight_done = s->done_ev;
  }
  s->inflight_n = n_sweeps;
  s->host_ns[4] = host_now_ns();
  return CLV_OK;
}

int clv::persist_wait(clv_sampler* s) {
  const int64_t n_sweeps = s->inflight_n;
  if (n_sweeps == 0) return CLV_OK;
  s->inflight_n = 0;
  const Geometry& g = s->g;
  // the host polls the launch's end event (stream synchronize / event synchronize measured within
  // 0.3 us per step of it, profiles/r04_host_variants.jsonl)
  const hipEvent_t done = s->inflight_done;
  if (!done) {
    CLV_HIP(hipStreamSynchronize(s->stream));
  } else {
    hipError_t q;
    while ((q = hipEventQuery(done)) == hipErrorNotReady) {
    }
    CLV_HIP(q);
  }
  s->host_ns[5] = host_now_ns();
  if (__atomic_load_n(s->h_abort, __ATOMIC_ACQUIRE)) {
    // the carried state was written to the *_alt buffers only: lam / mu / hyper still hold the
    // state this launch started from; restore the counters, flags and running sums
    *s->h_abort = 0;
    Ctrl c{};
    c.cur = s->sweeps_done;
    CLV_HIP(hipMemcpy(s->d_ctrl, &c, sizeof(Ctrl), hipMemcpyHostToDevice));
    const size_t sums_bytes = sizeof(double) * (size_t)g.n_chains * CLV_N_SUM_STATS * g.n;
    if (s->d_sums_prev) CLV_HIP(hipMemcpy(s->d_sums, s->d_sums_prev, sums_bytes, hipMemcpyDeviceToDevice));
    s->slots_dirty = true;
    if (g.world_size > 1) s->p2p_ready = false;  // mail slots are in an unknown state now
    const std::string diag = take_wait_diag(s);
    return fail(CLV_EHIP, std::string(g.world_size > 1
                                          ? "persistent sweep kernel: a wait timed out (a peer rank not running, or not all "
                                            "resident?); state unchanged"
                                          : "persistent sweep kernel: a workgroup timed out waiting for its chain (not all "
                                            "resident?); state unchanged") + diag);
  }
  std::swap(s->d_lam, s->d_lam_alt);
  std::swap(s->d_mu, s->d_mu_alt);
  s->rb_pend = s->pend;  // (rollback: the hyper state this launch started from)
  s->rb_pend_buf = s->pend_buf;
  s->rb_hyper_swaps = 0;
  if (s->defer) {  // the launch's last draw is pending in the other buffer; hyper untouched
    s->pend = true;
    s->pend_buf ^= 1;
  } else {
    std::swap(s->d_hyper, s->d_hyper_alt);
    s->rb_hyper_swaps = 1;
    s->pend = false;
  }
  if (s->graph_exec) {  // captured with the previous state pointers
    CLV_HIP(hipGraphExecDestroy(s->graph_exec));
    s->graph_exec = nullptr;
  }
  s->sweeps_done += n_sweeps;
  s->last_persist_n = n_sweeps;
  return CLV_OK;
}

// The pending level-2 draw of the last launch's last sweep (CLV_DEFER), into hyper (and the
// level-2 record it belongs to): before anything reads the hyper state or the level-2 records, or
// runs a sweep that is not a persistent launch.  The same draw (statistics, variates, order) the
// next launch would make first, so results do not depend on where a run is cut into clv_run calls.
int clv::persist_flush(clv_sampler* s) {
  if (!s->pend) return CLV_OK;
  CLV_HIP(hipSetDevice(s->device));
  SweepArgs a = sweep_args(s, 0, 1);
  a.pend_in = s->d_pend + s->pend_buf * (int64_t)s->g.n_chains * s->g.stride;
  a.pend_out = nullptr;
  CLV_HIP(launch_persist_flush(a, s->sweeps_done + 1, s->stream));
  CLV_HIP(hipStreamSynchronize(s->stream));
  std::swap(s->d_hyper, s->d_hyper_alt);
  s->rb_hyper_swaps++;
  s->pend = false;
  if (s->graph_exec) {
    CLV_HIP(hipGraphExecDestroy(s->graph_exec));
    s->graph_exec = nullptr;
  }
  return CLV_OK;
}

namespace {
int run_persistent(clv_sampler* s, int64_t n_sweeps) {
  int rc = persist_launch(s, n_sweeps);
  if (rc) return rc;
  return persist_wait(s);
}

// n launches of the fused sweep kernel (world size 1, or sharded with the fused peer exchange):
// hipGraph chunks, or (timing) one event pair per launch.  Not waited for.
int enqueue_fused_sweeps(clv_sampler* s, int64_t n_sweeps) {
  int rc = CLV_OK;
  int64_t left = n_sweeps;
  if (s->timing) {
    rc = ensure_events(s);
    if (rc) return rc;
    while (left > 0) {
      const int k = s->ev_used;
      rc = enqueue_fused(s, s->ev[4 * k], s->ev[4 * k + 1]);
      if (rc) return rc;
      s->ev_used++;
      s->sweeps_done++;
      left--;
      if (s->ev_used == TIMING_EVENTS) {
        rc = harvest_timing(s);
        if (rc) return rc;
      }
    }
    return harvest_timing(s);
  }
  if (left >= GRAPH_CHUNK) {
    rc = build_graph(s, GRAPH_CHUNK);
    if (rc) return rc;
    while (left >= GRAPH_CHUNK) {
      CLV_HIP(hipGraphLaunch(s->graph_exec, s->stream));
      s->sweeps_done += GRAPH_CHUNK;
      left -= GRAPH_CHUNK;
    }
  }
  while (left > 0) {
    rc = enqueue_fused(s, nullptr, nullptr);
    if (rc) return rc;
    s->sweeps_done++;
    left--;
  }
  return CLV_OK;
}

// World size > 1 without a resident grid: n launches of the sweep kernel whose fused tail
// exchanges unit partials through the peers' mail (kernels.hip sweep_body, FX).  The state before
// the call is kept in the persistent path's *_alt buffers, so that a call in which a wait times out
// (a peer not running; the call's later launches then return at once) leaves it unchanged, and a
// completed call can be undone by clv_rollback (a step that failed on another rank).
int run_fused_exchange(clv_sampler* s, int64_t n_sweeps) {
  s->last_persist_n = 0;
  if (n_sweeps == 0) return CLV_OK;
  const Geometry& g = s->g;
  const size_t nl = sizeof(double) * (size_t)g.n_chains * std::max<int64_t>(g.n, 1);
  const size_t sums_bytes = sizeof(double) * (size_t)g.n_chains * CLV_N_SUM_STATS * g.n;
  CLV_HIP(hipMemcpyAsync(s->d_lam_alt, s->d_lam, nl, hipMemcpyDeviceToDevice, s->stream));
  CLV_HIP(hipMemcpyAsync(s->d_mu_alt, s->d_mu, nl, hipMemcpyDeviceToDevice, s->stream));
  CLV_HIP(hipMemcpyAsync(s->d_hyper_alt, s->d_hyper, sizeof(double) * g.n_chains * HS, hipMemcpyDeviceToDevice,
                         s->stream));
  if (s->d_sums_prev) CLV_HIP(hipMemcpyAsync(s->d_sums_prev, s->d_sums, sums_bytes, hipMemcpyDeviceToDevice, s->stream));
  const int64_t before = s->sweeps_done;
  const int rc = enqueue_fused_sweeps(s, n_sweeps);
  CLV_HIP(hipStreamSynchronize(s->stream));
  const bool aborted = __atomic_load_n(s->h_abort, __ATOMIC_ACQUIRE) != 0;
  if (rc == CLV_OK && !aborted) {
    s->last_persist_n = n_sweeps;
    s->rb_pend = false;      // (rollback: the hyper state before the call is the copy in hyper_alt)
    s->rb_hyper_swaps = 1;
    return CLV_OK;
  }
  // back to the state before the call (copies: a captured graph keeps the buffer addresses)
  CLV_HIP(hipMemcpy(s->d_lam, s->d_lam_alt, nl, hipMemcpyDeviceToDevice));
  CLV_HIP(hipMemcpy(s->d_mu, s->d_mu_alt, nl, hipMemcpyDeviceToDevice));
  CLV_HIP(hipMemcpy(s->d_hyper, s->d_hyper_alt, sizeof(double) * g.n_chains * HS, hipMemcpyDeviceToDevice));
  if (s->d_sums_prev) CLV_HIP(hipMemcpy(s->d_sums, s->d_sums_prev, sums_bytes, hipMemcpyDeviceToDevice));
  *s->h_abort = 0;
  s->sweeps_done = before;
  Ctrl c{};
  c.cur = before;
  CLV_HIP(hipMemcpy(s->d_ctrl, &c, sizeof(Ctrl), hipMemcpyHostToDevice));
  CLV_HIP(hipMemset(s->d_arrive, 0, sizeof(uint32_t) * (g.n_chains + (int64_t)g.n_chains * g.units_per_rank)));
  s->p2p_ready = false;  // mail slots in an unknown state: clv_p2p_connect refills them
  if (rc) return rc;
  return fail(CLV_EHIP, "fused peer exchange: a wait timed out (a peer rank not running?); state unchanged" +
                            take_wait_diag(s));
}

// World size 1 with the draws streamed to the host (clv_stream_draws): the burn-in in one go, the
// stored sweeps in sub-runs of >= 256 sweeps and ~64 MB of draws, each sub-run's draws handed to the
// copy pool while the next one runs (the same launches' sweeps in the same order: the same bits).
int run_streaming(clv_sampler* s, int64_t n_sweeps) {
  const Geometry& g = s->g;
  const int64_t per_draw = (int64_t)g.n_chains * g.n * (g.D + 2) * (int64_t)sizeof(double);
  const int64_t chunk = std::max<int64_t>(256, std::max<int64_t>(1, (64LL << 20) / std::max<int64_t>(per_draw, 1)) * g.thin);
  int64_t left = n_sweeps;
  while (left > 0) {
    const int64_t k = s->sweeps_done < g.burnin ? std::min<int64_t>(left, g.burnin - s->sweeps_done)
                                                : std::min<int64_t>(left, chunk);
    int rc;
    if (s->persistent) {
      rc = run_persistent(s, k);
    } else {
      rc = enqueue_fused_sweeps(s, k);
      if (rc == CLV_OK && hipStreamSynchronize(s->stream) != hipSuccess) rc = fail(CLV_EHIP, "hipStreamSynchronize");
    }
    if (rc) return rc;
    stream_enqueue(s);
    left -= k;
  }
  return CLV_OK;
}
}  // namespace

extern "C" {

int clv_run(clv_sampler* s, int64_t n_sweeps) {
  if (!s) return fail(CLV_EINVAL, "null sampler");
  s->clk_first = s->sweeps_done + 1;
  if (s->g.world_size != 1) {
    if (!s->p2p_ready) return fail(CLV_ESTATE, "sharded clv_run needs clv_p2p_connect; else use clv_sweep/clv_hyper");
    if (s->pending_init_hyper) return fail(CLV_ESTATE, "bivariate: call clv_hyper once before the first sweep");
    if (n_sweeps < 0) return fail(CLV_EINVAL, "n_sweeps < 0");
    CLV_HIP(hipSetDevice(s->device));
    if (s->p2p_capable) return run_persistent(s, n_sweeps);
    return run_fused_exchange(s, n_sweeps);
  }
  if (n_sweeps < 0) return fail(CLV_EINVAL, "n_sweeps < 0");
  s->host_ns[0] = host_now_ns();
  CLV_HIP(hipSetDevice(s->device));
  s->host_ns[1] = host_now_ns();
  int rc = check_replay_range(s, n_sweeps);
  if (rc) return rc;
  if (s->pending_init_hyper) {
    rc = enqueue_hyper(s, nullptr, 1, nullptr, nullptr);
    if (rc) return rc;
    s->pending_init_hyper = false;
  }
  if (s->ds_dest) return run_streaming(s, n_sweeps);
  if (s->persistent) {
    rc = run_persistent(s, n_sweeps);
    s->host_ns[6] = host_now_ns();
    return rc;
  }
  rc = enqueue_fused_sweeps(s, n_sweeps);
  if (rc) return rc;
  CLV_HIP(hipStreamSynchronize(s->stream));
  return CLV_OK;
}

int clv_stream_draws(clv_sampler* s, double* level1) {
  if (!s) return fail(CLV_EINVAL, "null sampler");
  if (s->ds) {
    stream_wait(s->ds);
    // the old registration ends here; a new one streams every draw again from the first
    // (ds_next = 0), so a failure of the old pieces has nothing left to repair
    stream_clear_failed(s->ds);
  }
  if (!level1) {
    s->ds_dest = nullptr;
    return CLV_OK;
  }
  if (s->g.world_size != 1) return fail(CLV_ESTATE, "draw streaming needs world_size 1");
  if (!s->d_level1) return fail(CLV_ESTATE, "draw streaming needs draw_sink == CLV_SINK_FULL with draws to store");
  CLV_HIP(hipSetDevice(s->device));
  if (!s->ds) s->ds = new DrawStreamState();
  s->ds_dest = level1;
  s->ds_next = 0;
  const Geometry& g = s->g;
  stream_prefault(s->ds, s->device, level1, sizeof(double) * (size_t)g.n_chains * g.n_draws * g.n * (g.D + 2));
  // draws of sweeps already run: the pool copies on the null stream, which does not order against
  // the sampler's non-blocking stream, so the sweeps enqueued there must have completed
  CLV_HIP(hipStreamSynchronize(s->stream));
  stream_enqueue(s);
  return CLV_OK;
}

int clv_rollback(clv_sampler* s) {
  if (!s) return fail(CLV_EINVAL, "null sampler");
  if (s->ds_dest) return fail(CLV_ESTATE, "clv_rollback while the draws are streamed (clv_stream_draws)");
  if (s->last_persist_n <= 0) return fail(CLV_ESTATE, "nothing to roll back (the last call was not a completed persistent clv_run)");
  CLV_HIP(hipSetDevice(s->device));
  CLV_HIP(hipStreamSynchronize(s->stream));
  std::swap(s->d_lam, s->d_lam_alt);
  std::swap(s->d_mu, s->d_mu_alt);
  // the hyper state the launch started from: pending statistics (still in their buffer), or the
  // hyper buffer that was current then (in hyper_alt after an odd number of swaps since)
  if (s->rb_hyper_swaps & 1) std::swap(s->d_hyper, s->d_hyper_alt);
  s->pend = s->rb_pend;
  s->pend_buf = s->rb_pend_buf;
  s->rb_hyper_swaps = 0;
  s->sweeps_done -= s->last_persist_n;
  s->last_persist_n = 0;
  Ctrl c{};
  c.cur = s->sweeps_done;
  CLV_HIP(hipMemcpy(s->d_ctrl, &c, sizeof(Ctrl), hipMemcpyHostToDevice));
  if (s->d_sums_prev)
    CLV_HIP(hipMemcpy(s->d_sums, s->d_sums_prev, sizeof(double) * (size_t)s->g.n_chains * CLV_N_SUM_STATS * s->g.n,
                      hipMemcpyDeviceToDevice));
  if (s->graph_exec) {
    CLV_HIP(hipGraphExecDestroy(s->graph_exec));
    s->graph_exec = nullptr;
  }
  return CLV_OK;
}

int clv_read_draws(clv_sampler* s, double* level1, double* level2, double* loglik) {
  if (!s) return fail(CLV_EINVAL, "null sampler");
  CLV_HIP(hipSetDevice(s->device));
  CLV_HIP(hipStreamSynchronize(s->stream));
  if (level2) {
    int rc = persist_flush(s);  // the last level-2 record may still be pending
    if (rc) return rc;
  }
  const Geometry& g = s->g;
  const size_t C = g.n_chains;
  if (level1) {
    if (!s->d_level1 && g.n_draws > 0 && g.n > 0) return fail(CLV_ESTATE, "level-1 draws need draw_sink == CLV_SINK_FULL");
    bool done = false;
    if (s->ds_dest == level1) {  // streamed: the rest of the stored draws, then wait for every copy
      stream_enqueue(s);
      done = stream_wait(s->ds);
      // (draws beyond the stored ones are never written: zeros, as the device buffer holds)
      const int64_t k = stored_count(s, s->sweeps_done);
      if (done && k < g.n_draws)
        for (size_t c = 0; c < C; ++c)
          std::memset(level1 + ((int64_t)c * g.n_draws + k) * g.n * (g.D + 2), 0,
                      sizeof(double) * (size_t)((g.n_draws - k) * g.n * (g.D + 2)));
    } else if (s->ds) {
      stream_wait(s->ds);
    }
    if (s->d_level1 && !done) {
      CLV_HIP(hipMemcpy(level1, s->d_level1, sizeof(double) * C * g.n_draws * g.n * (g.D + 2), hipMemcpyDeviceToHost));
      if (s->ds && s->ds_dest == level1) stream_clear_failed(s->ds);  // the full copy repaired it
    }
  }
  if (level2 && s->d_level2)
    CLV_HIP(hipMemcpy(level2, s->d_level2, sizeof(double) * C * g.n_draws * g.l2w, hipMemcpyDeviceToHost));
  if (loglik && s->d_loglik)
    CLV_HIP(hipMemcpy(loglik, s->d_loglik, sizeof(double) * C * g.n_draws, hipMemcpyDeviceToHost));
  return CLV_OK;
}

int clv_read_summary(clv_sampler* s, double* sums, int64_t* n_stored) {
  if (!s) return fail(CLV_EINVAL, "null sampler");
  CLV_HIP(hipSetDevice(s->device));
  CLV_HIP(hipStreamSynchronize(s->stream));
  const Geometry& g = s->g;
  if (n_stored) {
    int64_t k = 0;
    if (s->sweeps_done > g.burnin) k = (s->sweeps_done - 1 - g.burnin) / g.thin + 1;
    *n_stored = std::min<int64_t>(k, g.n_draws);
  }
  if (sums) {
    if (!s->d_sums) return fail(CLV_ESTATE, "summaries need draw_sink == CLV_SINK_SUMMARY (or _PCT)");
    CLV_HIP(hipMemcpy(sums, s->d_sums, sizeof(double) * g.n_chains * CLV_N_SUM_STATS * g.n, hipMemcpyDeviceToHost));
  }
  return CLV_OK;
}

int clv_get_state(clv_sampler* s, double* lambdas, double* mus, double* hyper) {
  if (!s) return fail(CLV_EINVAL, "null sampler");
  CLV_HIP(hipSetDevice(s->device));
  CLV_HIP(hipStreamSynchronize(s->stream));
  if (hyper) {
    int rc = persist_flush(s);
    if (rc) return rc;
  }
  const Geometry& g = s->g;
  if (lambdas && g.n) CLV_HIP(hipMemcpy(lambdas, s->d_lam, sizeof(double) * g.n_chains * g.n, hipMemcpyDeviceToHost));
  if (mus && g.n) CLV_HIP(hipMemcpy(mus, s->d_mu, sizeof(double) * g.n_chains * g.n, hipMemcpyDeviceToHost));
  if (hyper) {
    std::vector<double> h((size_t)g.n_chains * HS);
    CLV_HIP(hipMemcpy(h.data(), s->d_hyper, sizeof(double) * h.size(), hipMemcpyDeviceToHost));
    const int w = g.K * g.D + g.D * g.D;
    for (int c = 0; c < g.n_chains; ++c) {
      for (int i = 0; i < g.K * g.D; ++i) hyper[c * w + i] = h[c * HS + H_BETA + i];
      for (int p = 0; p < g.D; ++p)
        for (int q = 0; q < g.D; ++q) hyper[c * w + g.K * g.D + p * g.D + q] = h[c * HS + H_SIGMA + p * 3 + q];
    }
  }
  return CLV_OK;
}

int clv_set_state(clv_sampler* s, const double* lambdas, const double* mus, const double* hyper, int64_t sweeps_done) {
  if (!s || sweeps_done < 0) return fail(CLV_EINVAL, "bad arguments");
  const Geometry& g = s->g;
  // the sampler takes logs of the state (bi:286-287; Philox mode: log_fast, defined for positive
  // normal doubles): reject what exp() of a log-scale state can never be
  for (const double* v : {lambdas, mus})
    if (v)
      for (int64_t i = 0; i < (int64_t)g.n_chains * g.n; ++i)
        if (!(v[i] >= 2.2250738585072014e-308 && v[i] <= 1.7976931348623157e308))
          return fail(CLV_EINVAL, "lambdas and mus must be positive, normal and finite");
  CLV_HIP(hipSetDevice(s->device));
  {  // a pending draw belongs to the state being replaced (its level-2 record too)
    int rc = persist_flush(s);
    if (rc) return rc;
  }
  if (lambdas && g.n) CLV_HIP(hipMemcpy(s->d_lam, lambdas, sizeof(double) * g.n_chains * g.n, hipMemcpyHostToDevice));
  if (mus && g.n) CLV_HIP(hipMemcpy(s->d_mu, mus, sizeof(double) * g.n_chains * g.n, hipMemcpyHostToDevice));
  if (hyper) {
    CLV_HIP(hipMemcpy(s->d_bs, hyper, sizeof(double) * g.n_chains * (g.K * g.D + g.D * g.D), hipMemcpyHostToDevice));
    CLV_HIP(launch_set_hyper(g.D, g.K, g.n_chains, s->d_hyper, s->d_bs, s->prior.omega2, s->replay, s->stream));
    s->pending_init_hyper = false;
  }
  Ctrl c{};
  c.cur = sweeps_done;
  CLV_HIP(hipMemcpyAsync(s->d_ctrl, &c, sizeof(Ctrl), hipMemcpyHostToDevice, s->stream));
  CLV_HIP(hipStreamSynchronize(s->stream));
  s->sweeps_done = sweeps_done;
  s->last_persist_n = 0;
  stream_rewind(s);
  return CLV_OK;
}

int clv_set_timing(clv_sampler* s, int32_t enable) {
  if (!s) return fail(CLV_EINVAL, "null sampler");
  int rc = harvest_timing(s);  // never drop pending timed launches
  if (rc) return rc;
  s->timing = enable != 0;
  if (s->timing) {  // created here, not inside the first timed clv_run
    CLV_HIP(hipSetDevice(s->device));
    rc = ensure_events(s);
    if (rc) return rc;
  }
  s->t_sweep_ms = s->t_hyper_ms = 0.0;
  s->n_sweep_timed = s->n_hyper_timed = 0;
  return CLV_OK;
}

int clv_kernel_time(clv_sampler* s, double* sweep_ms, int64_t* n_sweep, double* hyper_ms, int64_t* n_hyper) {
  if (!s) return fail(CLV_EINVAL, "null sampler");
  int rc = harvest_timing(s);
  if (rc) return rc;
  if (sweep_ms) *sweep_ms = s->t_sweep_ms;
  if (n_sweep) *n_sweep = s->n_sweep_timed;
  if (hyper_ms) *hyper_ms = s->t_hyper_ms;
  if (n_hyper) *n_hyper = s->n_hyper_timed;
  return CLV_OK;
}

// ---- test hooks ----
int clv_debug_stamps(clv_sampler* s, uint64_t* out) {
  if (!s || !out) return fail(CLV_EINVAL, "null argument");
  if (!s->d_stamps) return fail(CLV_ESTATE, "library not built with CLV_STAMPS (make STAMPS=1)");
  CLV_HIP(hipStreamSynchronize(s->stream));
  CLV_HIP(hipMemcpy(out, s->d_stamps, sizeof(uint64_t) * 1024 * 8, hipMemcpyDeviceToHost));
  return CLV_OK;
}

int clv_debug_wg_stamps(clv_sampler* s, uint64_t* out) {
  if (!s || !out) return fail(CLV_EINVAL, "null argument");
  if (!s->d_stamps) return fail(CLV_ESTATE, "library not built with CLV_STAMPS (make STAMPS=1)");
  CLV_HIP(hipStreamSynchronize(s->stream));
  CLV_HIP(hipMemcpy(out, s->d_stamps + 1024 * 8, sizeof(uint64_t) * 12 * s->g.n_chains * (s->g.nb_local + 1),
                    hipMemcpyDeviceToHost));
  return CLV_OK;
}

int clv_debug_host_times(const clv_sampler* s, int64_t* out) {
  if (!s || !out) return fail(CLV_EINVAL, "bad arguments");
  for (int k = 0; k < 8; ++k) out[k] = s->host_ns[k];
  return CLV_OK;
}

int clv_debug_philox(uint32_t k0, uint32_t k1, const uint32_t* ctr, int64_t n, uint32_t* out) {
  if (!ctr || !out || n < 0) return fail(CLV_EINVAL, "bad arguments");
  uint32_t *dc = nullptr, *dout = nullptr;
  CLV_HIP(dalloc(&dc, 4 * std::max<int64_t>(n, 1)));
  CLV_HIP(dalloc(&dout, 4 * std::max<int64_t>(n, 1)));
  CLV_HIP(hipMemcpy(dc, ctr, 16 * n, hipMemcpyHostToDevice));
  CLV_HIP(launch_debug_philox(k0, k1, dc, n, dout, nullptr));
  CLV_HIP(hipMemcpy(out, dout, 16 * n, hipMemcpyDeviceToHost));
  CLV_HIP(hipFree(dc));
  CLV_HIP(hipFree(dout));
  return CLV_OK;
}

int clv_debug_variates(uint64_t seed, int32_t chain, uint32_t sweep, int64_t n, int32_t S, float* tl, float* tm,
                       float* ua, double* uz, double* ut, double* ea, double* ez, float* l2u) {
  if (n < 1 || S < 0) return fail(CLV_EINVAL, "bad arguments");
  const int64_t nS = std::max<int64_t>(n * S, 1);
  float *dtl, *dtm, *dua, *dl2u;
  double *duz, *dut, *dea, *dez;
  CLV_HIP(dalloc(&dtl, nS));
  CLV_HIP(dalloc(&dtm, nS));
  CLV_HIP(dalloc(&dua, nS));
  CLV_HIP(dalloc(&dl2u, nS));
  CLV_HIP(dalloc(&duz, n));
  CLV_HIP(dalloc(&dut, n));
  CLV_HIP(dalloc(&dea, n));
  CLV_HIP(dalloc(&dez, n));
  CLV_HIP(launch_debug_variates(seed, chain, sweep, n, S, dtl, dtm, dua, dl2u, duz, dut, dea, dez, nullptr));
  if (S > 0) {
    CLV_HIP(hipMemcpy(tl, dtl, sizeof(float) * n * S, hipMemcpyDeviceToHost));
    CLV_HIP(hipMemcpy(tm, dtm, sizeof(float) * n * S, hipMemcpyDeviceToHost));
    CLV_HIP(hipMemcpy(ua, dua, sizeof(float) * n * S, hipMemcpyDeviceToHost));
    if (l2u) CLV_HIP(hipMemcpy(l2u, dl2u, sizeof(float) * n * S, hipMemcpyDeviceToHost));
  }
  CLV_HIP(hipMemcpy(uz, duz, sizeof(double) * n, hipMemcpyDeviceToHost));
  CLV_HIP(hipMemcpy(ut, dut, sizeof(double) * n, hipMemcpyDeviceToHost));
  CLV_HIP(hipMemcpy(ea, dea, sizeof(double) * n, hipMemcpyDeviceToHost));
  CLV_HIP(hipMemcpy(ez, dez, sizeof(double) * n, hipMemcpyDeviceToHost));
  for (void* p : {(void*)dtl, (void*)dtm, (void*)dua, (void*)dl2u, (void*)duz, (void*)dut, (void*)dea, (void*)dez})
    CLV_HIP(hipFree(p));
  return CLV_OK;
}

int clv_debug_log2u_scan(uint64_t w_begin, uint64_t w_end, double* out) {
  if (!out || w_end > (1ull << 32) || w_begin >= w_end) return fail(CLV_EINVAL, "bad arguments");
  constexpr int NB = 4096;
  double* dres = nullptr;
  CLV_HIP(dalloc(&dres, 4 * NB));
  CLV_HIP(launch_debug_log2u_scan(w_begin, w_end, NB, dres, nullptr));
  std::vector<double> r(4 * NB);
  CLV_HIP(hipMemcpy(r.data(), dres, sizeof(double) * r.size(), hipMemcpyDeviceToHost));
  CLV_HIP(hipFree(dres));
  double mu = 0.0, ma = 0.0, wu = 0.0, mu_far = 0.0;
  for (int b = 0; b < NB; ++b) {
    if (r[4 * b] > mu) {
      mu = r[4 * b];
      wu = r[4 * b + 2];
    }
    ma = std::max(ma, r[4 * b + 1]);
    mu_far = std::max(mu_far, r[4 * b + 3]);
  }
  out[0] = mu;      // max error in fp32 ulps of the exact log2
  out[1] = ma;      // max absolute error
  out[2] = wu;      // the word where the ulp error is largest
  out[3] = mu_far;  // max ulp error where U <= 1/2 (|log2 U| >= 1)
  return CLV_OK;
}

int clv_debug_t3(const uint32_t* words, int64_t n, int32_t packed, float* tl, float* tm) {
  if (!words || !tl || !tm || n < 1 || (packed != 0 && packed != 1)) return fail(CLV_EINVAL, "bad arguments");
  uint32_t* dw = nullptr;
  float *dl = nullptr, *dm = nullptr;
  CLV_HIP(dalloc(&dw, 3 * n));
  CLV_HIP(dalloc(&dl, n));
  CLV_HIP(dalloc(&dm, n));
  CLV_HIP(hipMemcpy(dw, words, 12 * n, hipMemcpyHostToDevice));
  CLV_HIP(launch_debug_t3(dw, n, packed, dl, dm, nullptr));
  CLV_HIP(hipMemcpy(tl, dl, sizeof(float) * n, hipMemcpyDeviceToHost));
  CLV_HIP(hipMemcpy(tm, dm, sizeof(float) * n, hipMemcpyDeviceToHost));
  for (void* p : {(void*)dw, (void*)dl, (void*)dm}) CLV_HIP(hipFree(p));
  return CLV_OK;
}

int clv_debug_level2(int32_t D, int32_t K, const clv_prior* prior, const double* xty, const double* yty,
                     const double* iwn, const double* chi2, const double* z, double* beta, double* sigma) {
  if ((D != 2 && D != 3) || K < 1 || K > CLV_MAX_K || !prior) return fail(CLV_EINVAL, "bad arguments");
  std::vector<double> pr(PRIOR_DOUBLES, 0.0);
  for (int i = 0; i < K * K; ++i) {
    pr[i] = prior->V[i];
    pr[81 + i] = prior->chol_V[i];
  }
  for (int i = 0; i < K * D; ++i) pr[162 + i] = prior->A0B0[i];
  for (int i = 0; i < D * D; ++i) pr[189 + i] = prior->S0_B0A0B0[i];
  std::vector<double> in(K * D + D * D + 6 + D * K, 0.0);
  for (int i = 0; i < K * D; ++i) in[i] = xty[i];
  for (int i = 0; i < D * D; ++i) in[K * D + i] = yty[i];
  for (int i = 0; i < D * (D - 1) / 2; ++i) in[K * D + D * D + i] = iwn[i];
  for (int i = 0; i < D; ++i) in[K * D + D * D + 3 + i] = chi2[i];
  for (int i = 0; i < D * K; ++i) in[K * D + D * D + 6 + i] = z[i];
  double *dpr, *din, *dout;
  CLV_HIP(dalloc(&dpr, pr.size()));
  CLV_HIP(dalloc(&din, in.size()));
  CLV_HIP(dalloc(&dout, K * D + D * D));
  CLV_HIP(hipMemcpy(dpr, pr.data(), sizeof(double) * pr.size(), hipMemcpyHostToDevice));
  CLV_HIP(hipMemcpy(din, in.data(), sizeof(double) * in.size(), hipMemcpyHostToDevice));
  CLV_HIP(launch_debug_level2(D, K, dpr, din, dout, nullptr));
  std::vector<double> o(K * D + D * D);
  CLV_HIP(hipMemcpy(o.data(), dout, sizeof(double) * o.size(), hipMemcpyDeviceToHost));
  for (int i = 0; i < K * D; ++i) beta[i] = o[i];
  for (int i = 0; i < D * D; ++i) sigma[i] = o[K * D + i];
  CLV_HIP(hipFree(dpr));
  CLV_HIP(hipFree(din));
  CLV_HIP(hipFree(dout));
  return CLV_OK;
}

int clv_debug_hyper_variates(uint64_t seed, int32_t chain, uint32_t sweep, double df, int64_t n, double* chi2,
                             double* normals) {
  if (n < 1 || df < 2.0) return fail(CLV_EINVAL, "bad arguments");
  double *dc, *dn;
  CLV_HIP(dalloc(&dc, n));
  CLV_HIP(dalloc(&dn, n));
  CLV_HIP(launch_debug_hyper_variates(seed, chain, sweep, df, n, dc, dn, nullptr));
  CLV_HIP(hipMemcpy(chi2, dc, sizeof(double) * n, hipMemcpyDeviceToHost));
  CLV_HIP(hipMemcpy(normals, dn, sizeof(double) * n, hipMemcpyDeviceToHost));
  CLV_HIP(hipFree(dc));
  CLV_HIP(hipFree(dn));
  return CLV_OK;
}

int clv_debug_persist_choice(int32_t D, int32_t K, int32_t n_chains, int64_t grid_wgs, int32_t blocks_per_cu,
                             int32_t n_cu) {
  return persist_grid_fits(grid_wgs, blocks_per_cu, n_cu) && persist_worth(D, K, n_chains, grid_wgs, n_cu) ? 1 : 0;
}

int clv_debug_persist_fits(int64_t grid_wgs, int32_t blocks_per_cu, int32_t n_cu) {
  return persist_grid_fits(grid_wgs, blocks_per_cu, n_cu) ? 1 : 0;
}

int clv_debug_wg_map(int32_t n_chains, int32_t nb, int32_t n_cu, int32_t* out) {
  if (!out || n_chains < 1 || nb < 0 || n_cu < 1 || n_chains >= (1 << 15) || nb >= (1 << 16))
    return fail(CLV_EINVAL, "bad arguments");
  const std::vector<int32_t> m = persist_wg_map(n_chains, nb, n_cu);
  std::copy(m.begin(), m.end(), out);
  return CLV_OK;
}

int clv_debug_mh_step(int64_t n, const int32_t* x, const uint8_t* z, const double* T_cal, const double* tau,
                      const double* mean, const double* prec3, const double* cur_pt, const float* t3,
                      const double* scale2, const float* log_u, double* out) {
  if (!x || !z || !T_cal || !tau || !mean || !prec3 || !cur_pt || !t3 || !scale2 || !log_u || !out || n < 1)
    return fail(CLV_EINVAL, "bad arguments");
  int32_t *dx;
  uint8_t* dz;
  double *dT, *dtau, *dm, *dp, *dc, *ds, *dout;
  float *dt3, *dlu;
  CLV_HIP(hipMalloc(&dx, sizeof(int32_t) * n));
  CLV_HIP(hipMalloc(&dz, n));
  CLV_HIP(dalloc(&dT, n));
  CLV_HIP(dalloc(&dtau, n));
  CLV_HIP(dalloc(&dm, 2 * n));
  CLV_HIP(dalloc(&dp, 3));
  CLV_HIP(dalloc(&dc, 2 * n));
  CLV_HIP(dalloc(&ds, 2));
  CLV_HIP(dalloc(&dout, 7 * n));
  CLV_HIP(hipMalloc(&dt3, sizeof(float) * 2 * n));
  CLV_HIP(hipMalloc(&dlu, sizeof(float) * n));
  CLV_HIP(hipMemcpy(dx, x, sizeof(int32_t) * n, hipMemcpyHostToDevice));
  CLV_HIP(hipMemcpy(dz, z, n, hipMemcpyHostToDevice));
  CLV_HIP(hipMemcpy(dT, T_cal, sizeof(double) * n, hipMemcpyHostToDevice));
  CLV_HIP(hipMemcpy(dtau, tau, sizeof(double) * n, hipMemcpyHostToDevice));
  CLV_HIP(hipMemcpy(dm, mean, sizeof(double) * 2 * n, hipMemcpyHostToDevice));
  CLV_HIP(hipMemcpy(dp, prec3, sizeof(double) * 3, hipMemcpyHostToDevice));
  CLV_HIP(hipMemcpy(dc, cur_pt, sizeof(double) * 2 * n, hipMemcpyHostToDevice));
  CLV_HIP(hipMemcpy(ds, scale2, sizeof(double) * 2, hipMemcpyHostToDevice));
  CLV_HIP(hipMemcpy(dt3, t3, sizeof(float) * 2 * n, hipMemcpyHostToDevice));
  CLV_HIP(hipMemcpy(dlu, log_u, sizeof(float) * n, hipMemcpyHostToDevice));
  CLV_HIP(launch_debug_mh(dx, dz, dT, dtau, dm, dp, dc, dt3, ds, dlu, n, dout, nullptr));
  CLV_HIP(hipMemcpy(out, dout, sizeof(double) * 7 * n, hipMemcpyDeviceToHost));
  for (void* p : {(void*)dx, (void*)dz, (void*)dT, (void*)dtau, (void*)dm, (void*)dp, (void*)dc, (void*)ds,
                  (void*)dout, (void*)dt3, (void*)dlu})
    CLV_HIP(hipFree(p));
  return CLV_OK;
}

}  // extern "C"
static int debug_fast_fn(const double* x, int64_t n, double* out, bool log_fn) {
  if (!x || !out || n < 1) return fail(CLV_EINVAL, "bad arguments");
  double *dx, *dout;
  CLV_HIP(dalloc(&dx, n));
  CLV_HIP(dalloc(&dout, n));
  CLV_HIP(hipMemcpy(dx, x, sizeof(double) * n, hipMemcpyHostToDevice));
  CLV_HIP(launch_debug_exp(dx, n, dout, nullptr, log_fn));
  CLV_HIP(hipMemcpy(out, dout, sizeof(double) * n, hipMemcpyDeviceToHost));
  CLV_HIP(hipFree(dx));
  CLV_HIP(hipFree(dout));
  return CLV_OK;
}
extern "C" {
int clv_debug_exp(const double* x, int64_t n, double* out) { return debug_fast_fn(x, n, out, false); }

int clv_debug_log(const double* x, int64_t n, double* out) { return debug_fast_fn(x, n, out, true); }

}  // extern "C"
