// In-process customer sharding over several devices (the drop-in's devices=
// extra; §8e).  One process drives the shards of one problem — clv_sampler handles with
// world_size = n and rank = their index, each on its own device (or sharing one) — with no
// torch.distributed / launcher.  The reference runs its chains one after another
// (bivariate/mcmc.py:481-488); the level-2 draw (bi:233-262) couples every customer of a chain, so
// the shards exchange their unit partials once per sweep, in one of two ways:
//
//   CLV_EXCHANGE_P2P   every shard's persistent grid fits its device at once: the shards' mail
//                      buffers are connected by device pointers (peer access enabled between
//                      distinct devices) and one clv_run-style persistent launch per shard runs all
//                      sweeps of a call — every launch is put in flight before any is waited for.
//   CLV_EXCHANGE_COPY  otherwise: per sweep, each shard's sweep kernels, then stream-ordered
//                      device-to-device copies of its unit partials into every shard's gathered
//                      buffer (pushed from the producer's stream, double-buffered by sweep parity),
//                      an event, and on every shard the level-2 draw after all shards' events.
//
// Both give the bits of the unsharded run (same block partials, same fixed-order sums).  A P2P
// call that times out on any shard is undone on the shards that completed it (clv_rollback) and
// redone through the copy exchange, which the group keeps from then on.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>
#include <vector>

#include "internal.h"

using namespace clv;

struct clv_group {
  std::vector<clv_sampler*> shards;
  int exchange = CLV_EXCHANGE_COPY;
  int64_t nd = 0;                         // doubles of one shard's unit partials
  std::vector<double*> gathered;          // [shard][parity] -> [world][nd] on the shard's device
  std::vector<hipEvent_t> ev;             // [shard] "this shard's partials pushed" (per exchange)
  int64_t n_exchanges = 0;                // exchanges so far (their parity alternates)
  std::vector<clv_sampler*> connected;    // shards this group connected (disconnected again by destroy)
};

namespace {

// One exchange: every shard pushes its unit partials (written by the kernels just enqueued on its
// stream) into every shard's gathered buffer of this parity, then every shard's level-2 draw
// waits for all pushes and reads its own gathered copy.  Reuse of a parity two exchanges later is
// ordered: a shard's push of exchange k + 2 follows its own level-2 draw of k + 1, which waited
// for every shard's push of k + 1 — each enqueued behind that shard's draw of k on its stream.
int exchange_and_hyper(clv_group* G) {
  const int W = (int)G->shards.size();
  const int par = (int)(G->n_exchanges & 1);
  const size_t bytes = sizeof(double) * (size_t)G->nd;
  for (int r = 0; r < W; ++r) {
    clv_sampler* s = G->shards[r];
    CLV_HIP(hipSetDevice(s->device));
    for (int q = 0; q < W; ++q) {
      clv_sampler* d = G->shards[q];
      CLV_HIP(hipMemcpyPeerAsync(G->gathered[2 * q + par] + (int64_t)r * G->nd, d->device, s->d_unit, s->device, bytes,
                                 s->stream));
    }
    CLV_HIP(hipEventRecord(G->ev[r], s->stream));
  }
  for (int q = 0; q < W; ++q) {
    clv_sampler* d = G->shards[q];
    CLV_HIP(hipSetDevice(d->device));
    for (int r = 0; r < W; ++r)
      if (r != q) CLV_HIP(hipStreamWaitEvent(d->stream, G->ev[r], 0));
    int rc = clv_hyper(d, G->gathered[2 * q + par]);
    if (rc) return rc;
  }
  G->n_exchanges++;
  return CLV_OK;
}

int run_copy(clv_group* G, int64_t n_sweeps) {
  for (int64_t k = 0; k < n_sweeps; ++k) {
    for (clv_sampler* s : G->shards) {
      int rc = clv_sweep(s);
      if (rc) return rc;
    }
    int rc = exchange_and_hyper(G);
    if (rc) return rc;
  }
  return CLV_OK;
}

int run_p2p(clv_group* G, int64_t n_sweeps) {
  const int W = (int)G->shards.size();
  std::vector<int> rc(W, CLV_OK);
  // test hook: CLV_TEST_P2P_STALL_RANK=r leaves shard r's launch out (a shard that never runs), so
  // the others wait out their bound and the group takes the fallback below (tests/test_gpu_multidevice)
  const char* stall_env = std::getenv("CLV_TEST_P2P_STALL_RANK");
  const int stall = stall_env ? std::atoi(stall_env) : -1;
  for (int r = 0; r < W; ++r) {  // every launch in flight first (each waits for the others' units)
    clv_sampler* s = G->shards[r];
    if (r == stall) {
      rc[r] = fail(CLV_EHIP, "test hook: shard launch withheld (CLV_TEST_P2P_STALL_RANK)");
      continue;
    }
    if (hipSetDevice(s->device) != hipSuccess) {
      rc[r] = fail(CLV_EHIP, "hipSetDevice");
      continue;
    }
    rc[r] = persist_launch(s, n_sweeps);
  }
  for (int r = 0; r < W; ++r) {
    clv_sampler* s = G->shards[r];
    if (rc[r] == CLV_OK) {
      (void)hipSetDevice(s->device);
      rc[r] = persist_wait(s);
    }
  }
  bool ok = true;
  for (int r = 0; r < W; ++r) ok = ok && rc[r] == CLV_OK;
  if (ok) return CLV_OK;
  // some shard timed out (its state is unchanged): the shards that completed undo the call, and
  // the sweeps are redone through the copy exchange (kept from now on)
  for (int r = 0; r < W; ++r)
    if (rc[r] == CLV_OK) {
      int e = clv_rollback(G->shards[r]);
      if (e) return e;
    }
  G->exchange = CLV_EXCHANGE_COPY;
  for (clv_sampler* s : G->connected) (void)clv_p2p_disconnect(s);  // no shard keeps stale peer pointers
  G->connected.clear();
  return run_copy(G, n_sweeps);
}

}  // namespace

extern "C" {

int clv_group_create(clv_sampler* const* shards, int32_t n, int32_t exchange, clv_group** out) {
  if (!shards || !out || n < 1) return fail(CLV_EINVAL, "null argument");
  if (exchange < CLV_EXCHANGE_AUTO || exchange > CLV_EXCHANGE_COPY) return fail(CLV_EINVAL, "bad exchange");
  *out = nullptr;
  for (int r = 0; r < n; ++r) {
    const clv_sampler* s = shards[r];
    if (!s) return fail(CLV_EINVAL, "null shard");
    for (int q = 0; q < r; ++q)
      if (shards[q] == s) return fail(CLV_EINVAL, "a shard appears twice");
    if (s->g.world_size != n || s->cfg.rank != r)
      return fail(CLV_EINVAL, "shard r must be the sampler of rank r of a world of n shards");
    const Geometry& a = s->g;
    const Geometry& b = shards[0]->g;
    if (a.D != b.D || a.K != b.K || a.S != b.S || a.n_chains != b.n_chains || a.n_global != b.n_global ||
        a.blocks_per_rank != b.blocks_per_rank || a.blocks_per_unit != b.blocks_per_unit || a.burnin != b.burnin ||
        a.mcmc != b.mcmc || a.thin != b.thin || s->cfg.seed != shards[0]->cfg.seed ||
        s->cfg.chain_first != shards[0]->cfg.chain_first)
      return fail(CLV_EINVAL, "shards of different problems or run settings");
    if (s->sweeps_done != shards[0]->sweeps_done) return fail(CLV_ESTATE, "shards at different sweeps");
    if (s->p2p_ready) return fail(CLV_ESTATE, "shard already connected to a peer exchange");
  }
  auto* G = new clv_group();
  G->shards.assign(shards, shards + n);
  G->nd = (int64_t)shards[0]->g.n_chains * shards[0]->g.units_per_rank * shards[0]->g.stride;
  auto cleanup = [&](int rc) {
    clv_group_destroy(G);
    return rc;
  };
  G->gathered.assign(2 * (size_t)n, nullptr);
  G->ev.assign(n, nullptr);
  for (int q = 0; q < n; ++q) {
    clv_sampler* s = shards[q];
    if (hipSetDevice(s->device) != hipSuccess) return cleanup(fail(CLV_EHIP, "hipSetDevice"));
    for (int p = 0; p < 2; ++p)
      if (hipMalloc((void**)&G->gathered[2 * q + p], sizeof(double) * (size_t)G->nd * n) != hipSuccess)
        return cleanup(fail(CLV_ENOMEM, "gathered unit-partial buffers"));
    if (hipEventCreateWithFlags(&G->ev[q], hipEventDisableTiming) != hipSuccess)
      return cleanup(fail(CLV_EHIP, "hipEventCreateWithFlags"));
  }
  // peer exchange: every shard's grid fits at once, and every pair of distinct devices can map
  // the other's memory (P2P stores from the level-2 workgroups)
  bool p2p = exchange != CLV_EXCHANGE_COPY && n > 1;
  for (int r = 0; r < n && p2p; ++r) p2p = shards[r]->p2p_capable;
  // shards sharing a device: their persistent kernels must run at the same time from different
  // streams, which HIP does not promise (more streams than hardware queues share a queue and then
  // run one after another: the first would wait out its bound for mail the second never sends).
  // AUTO takes the copy exchange there; CLV_EXCHANGE_P2P still tries it (and falls back if a wait
  // times out).
  for (int r = 0; r < n && p2p && exchange == CLV_EXCHANGE_AUTO; ++r)
    for (int q = 0; q < r && p2p; ++q)
      if (shards[q]->device == shards[r]->device) p2p = false;
  for (int r = 0; r < n && p2p; ++r) {  // shards sharing a device: their grids together
    int64_t wgs = 0;
    for (int q = 0; q < n; ++q)
      if (shards[q]->device == shards[r]->device) wgs += (int64_t)(shards[q]->g.nb_local + 1) * shards[q]->g.n_chains;
    p2p = persist_grid_fits(wgs, shards[r]->persist_bpc, shards[r]->n_cu);
  }
  for (int r = 0; r < n && p2p; ++r)
    for (int q = 0; q < n && p2p; ++q) {
      const int dr = shards[r]->device, dq = shards[q]->device;
      if (dr == dq) continue;
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, dr, dq) != hipSuccess || !can) {
        p2p = false;
        break;
      }
      (void)hipSetDevice(dr);
      const hipError_t e = hipDeviceEnablePeerAccess(dq, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) p2p = false;
      (void)hipGetLastError();  // an "already enabled" status is not an error here
    }
  if (exchange == CLV_EXCHANGE_P2P && !p2p)
    return cleanup(fail(CLV_ESTATE, "peer exchange not possible (a shard's grid does not fit at once, or no peer access)"));
  if (p2p) {
    std::vector<uint64_t> ptrs(n);
    for (int r = 0; r < n; ++r) ptrs[r] = (uint64_t)(uintptr_t)shards[r]->d_mail;
    for (int r = 0; r < n; ++r) {
      int rc = clv_p2p_connect(shards[r], nullptr, ptrs.data());
      if (rc) return cleanup(rc);  // (destroy disconnects the shards connected so far)
      G->connected.push_back(shards[r]);
    }
    G->exchange = CLV_EXCHANGE_P2P;
  } else {
    G->exchange = CLV_EXCHANGE_COPY;
  }
  *out = G;
  return CLV_OK;
}

int clv_group_run(clv_group* G, int64_t n_sweeps) {
  if (!G) return fail(CLV_EINVAL, "null group");
  if (n_sweeps < 0) return fail(CLV_EINVAL, "n_sweeps < 0");
  for (clv_sampler* s : G->shards)
    if (s->sweeps_done != G->shards[0]->sweeps_done) return fail(CLV_ESTATE, "shards at different sweeps");
  // bivariate: the level-2 draw of sweep 1 from the initial state (bi:393) — one exchange first
  if (G->shards[0]->pending_init_hyper) {
    int rc = exchange_and_hyper(G);
    if (rc) return rc;
  }
  int rc = G->exchange == CLV_EXCHANGE_P2P ? run_p2p(G, n_sweeps) : run_copy(G, n_sweeps);
  if (rc) return rc;
  for (clv_sampler* s : G->shards) {
    CLV_HIP(hipSetDevice(s->device));
    CLV_HIP(hipStreamSynchronize(s->stream));
  }
  return CLV_OK;
}

int32_t clv_group_exchange(const clv_group* G) { return G ? G->exchange : -1; }

void clv_group_destroy(clv_group* G) {
  if (!G) return;
  // shards outlive the group: none may keep pointers into another shard's mail (a later clv_run
  // would fail with CLV_ESTATE instead of storing into memory that may be freed)
  for (clv_sampler* s : G->connected) (void)clv_p2p_disconnect(s);
  for (size_t q = 0; q < G->shards.size(); ++q) {
    (void)hipSetDevice(G->shards[q]->device);
    (void)hipStreamSynchronize(G->shards[q]->stream);
    for (int p = 0; p < 2; ++p)
      if (2 * q + p < G->gathered.size() && G->gathered[2 * q + p]) (void)hipFree(G->gathered[2 * q + p]);
    if (q < G->ev.size() && G->ev[q]) (void)hipEventDestroy(G->ev[q]);
  }
  delete G;
}

}  // extern "C"
