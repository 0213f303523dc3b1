// Shader-clock probe (measurement only; the reference has no counterpart).
//
// MI355X boxes of one pool run the same kernels' cycles at shader clocks ~13% apart (DESIGN.md §8
// round 5), so every timed bench line carries the clock it ran at.  The persistent kernel records
// its own (clv_clock_ghz); the launch-per-sweep kernel cannot without slowing down (a mark in one
// workgroup per launch measured c4 +1.5%, c5 +1%).  clv_clock_probe instead runs a short busy kernel
// on the sampler's stream right after the caller's timed launches — the clock governor changes
// state on a millisecond scale, so a ~50 us probe enqueued behind them reads the clock they ran at:
// one 64-lane workgroup per CU spins on dependent fp64 FMAs until `us` microseconds of
// s_memrealtime (100 MHz) have passed and records (delta s_memtime, delta s_memrealtime) of its own
// CU (s_memtime counts per XCD, so each interval starts and ends on the same CU).  GHz = 0.1 x the
// sum of s_memtime deltas / the sum of s_memrealtime deltas.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "internal.h"

namespace clv {
namespace {

__global__ __launch_bounds__(64) void clock_probe_kernel(unsigned long long ticks, unsigned long long* out,
                                                         double seed) {
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long m0 = __builtin_amdgcn_s_memtime();
  double x = seed + threadIdx.x;
  unsigned long long r1 = r0;
  while (r1 - r0 < ticks) {
#pragma unroll
    for (int k = 0; k < 32; ++k) x = __builtin_fma(x, 0.999999, 1e-9);
    r1 = __builtin_amdgcn_s_memrealtime();
  }
  const unsigned long long m1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    out[3 * blockIdx.x] = m1 - m0;
    out[3 * blockIdx.x + 1] = r1 - r0;
    out[3 * blockIdx.x + 2] = x == 12345.678 ? 1ull : 0ull;  // keeps the FMAs live
  }
}

}  // namespace
}  // namespace clv

using namespace clv;

extern "C" int clv_clock_probe(clv_sampler* s, double us, double* ghz) {
  if (!s || !ghz) return fail(CLV_EINVAL, "null argument");
  *ghz = 0.0;
  if (!(us >= 1.0 && us <= 1e5)) return fail(CLV_EINVAL, "clv_clock_probe: us must be in [1, 1e5]");
  CLV_HIP(hipSetDevice(s->device));
  int n_cu = 0;
  CLV_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, s->device));
  n_cu = std::max(1, n_cu);
  DevBuf buf;
  CLV_HIP(hipMalloc(&buf.p, sizeof(unsigned long long) * 3 * n_cu));
  hipLaunchKernelGGL(clock_probe_kernel, dim3(n_cu), dim3(64), 0, s->stream, (unsigned long long)(us * 100.0),
                     buf.as<unsigned long long>(), 1.0);
  CLV_HIP(hipGetLastError());
  std::vector<unsigned long long> h(3 * (size_t)n_cu);
  CLV_HIP(hipMemcpyAsync(h.data(), buf.p, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost, s->stream));
  CLV_HIP(hipStreamSynchronize(s->stream));
  double dm = 0.0, dr = 0.0;
  for (int b = 0; b < n_cu; ++b) {
    dm += (double)h[3 * b];
    dr += (double)h[3 * b + 1];
  }
  if (dr > 0.0) *ghz = 0.1 * dm / dr;
  return CLV_OK;
}
