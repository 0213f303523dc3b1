// Calibrates the in-kernel clocks against HIP events: one workgroup spins for a fixed number of
// s_memrealtime ticks and records both counters; the host compares with the event-timed duration.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void spin(unsigned long long ticks, unsigned long long* out) {
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long m0 = __builtin_amdgcn_s_memtime();
  unsigned long long r = r0;
  while (r - r0 < ticks) {
    __builtin_amdgcn_s_sleep(10);
    r = __builtin_amdgcn_s_memrealtime();
  }
  const unsigned long long m1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    out[0] = r - r0;
    out[1] = m1 - m0;
  }
}

int main() {
  unsigned long long* d;
  unsigned long long h[2];
  hipMalloc(&d, 16);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (unsigned long long ticks : {100000ull, 1000000ull, 5000000ull}) {
    hipEventRecord(e0);
    spin<<<1, 64>>>(ticks, d);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    printf("realtime ticks %llu memtime %llu event %.3f ms -> realtime %.2f MHz, memtime %.1f MHz\n", h[0], h[1], ms,
           h[0] / (ms * 1e3), h[1] / (ms * 1e3));
  }
  return 0;
}
