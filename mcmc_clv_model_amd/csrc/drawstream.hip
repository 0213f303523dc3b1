// Streaming of the level-1 draws to the caller's host buffer while the sampler runs (host code).
//
// The drop-in's whole BASELINE run (run_mcmc_abe.py:60-77 times mcmc_draw_parameters end to end;
// bi:402-412 stores every thin-th sweep) returns ~3 GB of float64 draws at c2.  One pageable
// hipMemcpy after the run (~10 GB/s, the destination's pages faulted in by the copying thread)
// cost more than all 20,000 sweeps.  Here the copy is spread over the run and off its path:
//   * a process-wide pool of host worker threads per device, each with its own pinned staging
//     buffer, copying on the device's null stream (no stream of the pool's own: a stream holds one
//     of the process's few HIP hardware queues for good, and persistent grids of one process that
//     share a queue serialise — tests/test_gpu_p2p.py); the samplers launch on non-blocking
//     streams, which the null stream does not wait for.  Each worker waits for its own copy by an
//     event, and the DMA of one worker overlaps the memcpy of the others;
//   * when a destination is registered (clv_stream_draws) the workers first fault its pages in
//     (madvise MADV_POPULATE_WRITE: the page faults and zeroing happen during the burn-in, in
//     parallel);
//   * every clv_run hands the draws its sweeps completed to the pool (capi.hip stream_enqueue) and
//     returns; the copies run while the next sweeps do.  clv_read_draws waits for what is in
//     flight and copies the rest.
// The source ranges are draws of completed launches: later launches write other draw indices only.
#include <hip/hip_runtime.h>

#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "internal.h"

namespace clv {

namespace {

constexpr size_t STAGE_BYTES = 8u << 20;   // pinned staging per worker
constexpr size_t PIECE_BYTES = 32u << 20;  // one queue entry (4 DMA rounds)
constexpr size_t PAGE = 4096;

struct Piece {
  const char* src;  // device memory, or null: touch the destination's pages
  char* dst;
  size_t bytes;
  DrawStreamState* owner;
};

struct Pool {
  int device = 0;
  hipStream_t st = nullptr;  // the null stream (see the file comment)
  std::mutex m;
  std::condition_variable cv;
  std::deque<Piece> q;
  std::vector<std::thread> workers;

  void work() {
    (void)hipSetDevice(device);
    hipEvent_t ev = nullptr;
    char* stage = nullptr;
    const bool ok = hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess &&
                    hipHostMalloc((void**)&stage, STAGE_BYTES, hipHostMallocDefault) == hipSuccess;
    for (;;) {
      Piece p;
      {
        std::unique_lock<std::mutex> lk(m);
        cv.wait(lk, [&] { return !q.empty(); });
        p = q.front();
        q.pop_front();
      }
      bool good = ok;
      if (!p.src) {
        // fault every page in, writable, without touching its bytes (the kernel zero-fills only
        // pages not yet present, so a copy into the same range by another worker is never undone);
        // where MADV_POPULATE_WRITE is refused, a first touch by an atomic OR of zero instead
        const uintptr_t b0 = (uintptr_t)p.dst & ~(uintptr_t)(PAGE - 1);
        if (madvise((void*)b0, (uintptr_t)p.dst + p.bytes - b0, MADV_POPULATE_WRITE) != 0)
          for (size_t off = 0; off < p.bytes; off += PAGE) __atomic_fetch_or(p.dst + off, (char)0, __ATOMIC_RELAXED);
      } else {
        for (size_t off = 0; good && off < p.bytes; off += STAGE_BYTES) {
          const size_t len = std::min(STAGE_BYTES, p.bytes - off);
          good = hipMemcpyAsync(stage, p.src + off, len, hipMemcpyDeviceToHost, st) == hipSuccess &&
                 hipEventRecord(ev, st) == hipSuccess && hipEventSynchronize(ev) == hipSuccess;
          if (good) std::memcpy(p.dst + off, stage, len);
        }
      }
      if (!good) p.owner->failed.store(1);
      {
        std::lock_guard<std::mutex> lk(p.owner->m);
        p.owner->pending -= 1;
      }
      p.owner->cv.notify_all();
    }
  }
};

// One pool per device, created on first use and kept for the process (its threads sleep when idle;
// never joined: a pool outliving static destruction must not take the process down at exit).
Pool* pool_for(int device) {
  static std::mutex mu;
  static std::vector<Pool*> pools;
  std::lock_guard<std::mutex> lk(mu);
  for (Pool* p : pools)
    if (p->device == device) return p;
  auto* p = new Pool();
  p->device = device;
  const unsigned hc = std::max(2u, std::thread::hardware_concurrency());
  const int n = (int)std::min(8u, hc / 2);
  for (int k = 0; k < n; ++k) {
    p->workers.emplace_back([p] { p->work(); });
    p->workers.back().detach();
  }
  pools.push_back(p);
  return p;
}

void submit(DrawStreamState* st, int device, const char* src, char* dst, size_t bytes) {
  Pool* p = pool_for(device);
  std::vector<Piece> pieces;
  for (size_t off = 0; off < bytes; off += PIECE_BYTES)
    pieces.push_back(Piece{src ? src + off : nullptr, dst + off, std::min(PIECE_BYTES, bytes - off), st});
  {
    std::lock_guard<std::mutex> lk(st->m);
    st->pending += (int64_t)pieces.size();
  }
  {
    std::lock_guard<std::mutex> lk(p->m);
    for (auto& pc : pieces) p->q.push_back(pc);
  }
  p->cv.notify_all();
}

}  // namespace

void stream_prefault(DrawStreamState* st, int device, void* dst, size_t bytes) {
  if (bytes) submit(st, device, nullptr, (char*)dst, bytes);
}

void stream_copy(DrawStreamState* st, int device, const void* src, void* dst, size_t bytes) {
  if (bytes) submit(st, device, (const char*)src, (char*)dst, bytes);
}

// A failed piece stays recorded (sticky) until stream_clear_failed: whichever later call waits first
// (a rewind, a re-registration, the read) must not consume it, or clv_read_draws would take the
// destination for complete and skip the full copy that repairs it.
bool stream_wait(DrawStreamState* st) {
  std::unique_lock<std::mutex> lk(st->m);
  st->cv.wait(lk, [&] { return st->pending == 0; });
  return st->failed.load() == 0;
}

void stream_clear_failed(DrawStreamState* st) { st->failed.store(0); }

}  // namespace clv
