// Internal declarations shared by the C ABI translation units (capi.hip, analysis.hip):
// the sampler handle's layout and the error/allocation helpers.  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <mutex>
#include <string>
#include <vector>

#include "kernels.h"

namespace clv {

// Records msg as the calling thread's clv_last_error() and returns code.
int fail(int code, const std::string& msg);

// Persistent path in two halves (capi.hip): enqueue one launch of n sweeps; wait for it and adopt
// its carried state (or restore the state it started from, if a wait in it timed out).
int persist_launch(clv_sampler* s, int64_t n_sweeps);
int persist_wait(clv_sampler* s);
int persist_flush(clv_sampler* s);  // the deferred level-2 draw, if one is pending (synchronous)
// A persistent grid of grid_wgs workgroups fits at once (with a residency margin) on n_cu CUs
// admitting blocks_per_cu of its workgroups each (capi.hip).
bool persist_grid_fits(int64_t grid_wgs, int blocks_per_cu, int n_cu);
bool persist_worth(int D, int K, int n_chains, int64_t grid_wgs, int n_cu);

// Level-1 draws streamed to a host buffer during the run (drawstream.hip): the pieces a sampler has
// in flight in the process-wide copy pool, and whether any failed.
struct DrawStreamState {
  std::mutex m;
  std::condition_variable cv;
  int64_t pending = 0;
  std::atomic<int> failed{0};
};
void stream_prefault(DrawStreamState* st, int device, void* dst, size_t bytes);  // touch dst's pages
void stream_copy(DrawStreamState* st, int device, const void* src, void* dst, size_t bytes);
bool stream_wait(DrawStreamState* st);  // every piece done; false if one failed since the last clear
void stream_clear_failed(DrawStreamState* st);  // after a full copy has repaired the destination

template <class T>
hipError_t dalloc(T** p, size_t count) {
  *p = nullptr;
  if (count == 0) return hipSuccess;
  return hipMalloc((void**)p, count * sizeof(T));
}

// Owning device allocation (freed on scope exit) and a scoped device switch, for the host-side
// orchestration of the analysis / data-preparation entry points.
struct DevBuf {
  void* p = nullptr;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  template <class T>
  T* as() const {
    return (T*)p;
  }
};

struct DeviceScope {
  int prev = -1;
  explicit DeviceScope(int dev) {
    (void)hipGetDevice(&prev);
    if (dev >= 0) (void)hipSetDevice(dev);
  }
  ~DeviceScope() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

}  // namespace clv

#define CLV_HIP(expr)                                                                           \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess)                                                                       \
      return ::clv::fail(CLV_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_));          \
  } while (0)

struct clv_sampler {
  clv_config cfg{};
  clv_prior prior{};
  clv::Geometry g{};
  bool replay = false;
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t own = nullptr;  // stream created by the sampler (destroyed with it)
  bool own_stream = false;

  int32_t* d_x = nullptr;
  double *d_tx = nullptr, *d_T = nullptr, *d_cov = nullptr, *d_logs = nullptr;
  double *d_lam = nullptr, *d_mu = nullptr, *d_hyper = nullptr;
  double *d_block = nullptr, *d_unit = nullptr;
  double* d_prior = nullptr;
  clv::Ctrl* d_ctrl = nullptr;
  uint32_t* d_arrive = nullptr;     // fused-tail arrival counters: [chain], then [chain][units_per_rank]
  double* d_hyp2 = nullptr;         // persistent kernel: [2][chain][HS] hand-off slots
  double* d_pblock = nullptr;       // persistent kernel: [chain][nb_local][stride] block-partial slots
  // persistent kernel: the launch writes its carried state into the *_alt buffers; clv_run swaps
  // them in only when no wave aborted (an aborted launch leaves the state untouched), and
  // clv_rollback swaps them back (a sharded step that failed on another rank)
  double *d_lam_alt = nullptr, *d_mu_alt = nullptr, *d_hyper_alt = nullptr;
  double* d_sums_prev = nullptr;    // summary sink: the running sums before the last persistent launch
  uint32_t* h_abort = nullptr;      // host-mapped copy of ctrl->abort (the kernel stores it on a timeout)
  uint32_t* d_h_abort = nullptr;    // its device address
  unsigned long long* d_diag = nullptr;  // wait-timeout record (kernels.hip report_wait), DIAG_WORDS
  unsigned long long* d_clk = nullptr;   // shader-clock record [CLK_RING][2] (SweepArgs::clk)
  int64_t clk_first = 0;            // first sweep of the last clv_run (clv_clock_ghz)
  uint64_t wait_ticks = 0;          // bound on every persistent-kernel wait (s_memrealtime ticks)
  bool slots_dirty = true;          // persistent hand-off slots need the sentinel fill (a completed
                                    // launch leaves them empty; only an aborted one does not)
  int64_t last_persist_n = 0;       // sweeps of the last persistent launch (rollback), 0 = none
  // Deferred level-2 draw (world size 1, persistent, CLV_DEFER != "0"): a launch leaves the draw
  // that follows its last sweep to the next launch, which draws it first while its customer
  // workgroups load (kernels.hip persist_level2, iteration -1), or to persist_flush before anything
  // reads the hyper state or the level-2 records.  The pending statistics live in d_pend[pend_buf]
  // ([2][chain][stride]: a launch reads one buffer and writes the other, so an aborted launch or a
  // rollback finds the state it started from intact).
  bool defer = false;
  bool pend = false;                // the hyper state is the draw of d_pend[pend_buf], not d_hyper
  int pend_buf = 0;
  double* d_pend = nullptr;
  bool rb_pend = false;             // rollback: the pending state before the last persistent launch
  int rb_pend_buf = 0;
  int rb_hyper_swaps = 0;           // hyper / hyper_alt swaps since it (its hyper is in hyper_alt if odd)
  bool persistent = false;          // clv_run uses persist_kernel (all workgroups resident)
  int persist_bpc = 0, n_cu = 0;    // persist_kernel occupancy (workgroups per CU), CUs
  // world size > 1: persistent kernel with the peer (xGMI) exchange
  bool p2p_capable = false;         // the grid fits at once and the unit partials fit UMAIL
  bool p2p_persist_fits = false;    // (p2p_capable as chosen at create; clv_p2p_set_persistent may clear p2p_capable)
  bool fx_capable = false;          // fused peer exchange (launch-per-sweep, any shard size)
  bool p2p_ready = false;           // clv_p2p_connect done: clv_run runs persist_kernel
  double* d_mail = nullptr;         // [2][world][chain][units_per_rank][stride]
  int mail_kind = -1;               // the mail's memory: 0 uncached, 1 fine-grained, 2 plain device memory
  double** d_peers = nullptr;       // [world] mail pointers (peers' opened IPC mappings, own d_mail)
  int32_t* d_wgmap = nullptr;       // persistent grid: linear workgroup -> (chain << 16 | block)
  std::vector<void*> ipc_opened;    // hipIpcOpenMemHandle mappings to close
  double* d_hvar = nullptr;         // [chain][HV] precomputed hyper variates
  unsigned long long* d_stamps = nullptr;  // CLV_STAMPS diagnostic build only
  double *d_level1 = nullptr, *d_level2 = nullptr, *d_loglik = nullptr, *d_sums = nullptr;
  float2* d_qstore = nullptr;       // CLV_SINK_SUMMARY_PCT: [chain][draw][n] (lambda, mu) float32
  double* d_tape = nullptr;
  double* d_bs = nullptr;  // staging for set_hyper
  int64_t tape_sweeps = 0;

  bool pending_init_hyper = false;  // bivariate: the draw for sweep 1 is still due
  int64_t sweeps_done = 0;

  hipGraphExec_t graph_exec = nullptr;
  int graph_sweeps = 0;

  // clv_run waits for a persistent launch by polling its end event
  hipEvent_t done_ev = nullptr;     // recorded after each untimed persistent launch (timing: e1)
  int64_t inflight_n = 0;           // sweeps of the persistent launch in flight (persist_launch)
  hipEvent_t inflight_done = nullptr;  // its end event (null: wait with hipStreamSynchronize)

  // host clock (steady_clock, ns) at the steps of the last persistent clv_run: entry, after
  // hipSetDevice, before the launch call, after it, after the end-event record, wait done, return
  int64_t host_ns[8] = {0, 0, 0, 0, 0, 0, 0, 0};

  // clv_stream_draws: the caller's level-1 buffer and the draws (per chain) handed to the copy pool
  clv::DrawStreamState* ds = nullptr;
  double* ds_dest = nullptr;
  int64_t ds_next = 0;

  bool timing = false;
  std::vector<hipEvent_t> ev;  // 4 per slot: sweep start/end, hyper start/end
  std::vector<int64_t> ev_sweeps;  // sweeps per timed launch (persistent launches time many)
  int ev_used = 0;
  double t_sweep_ms = 0.0, t_hyper_ms = 0.0;
  int64_t n_sweep_timed = 0, n_hyper_timed = 0;
};

