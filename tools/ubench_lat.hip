// Microbenchmark (tools only): dependent-issue latency and throughput of the MH step's instruction
// classes on gfx950 — one wave per SIMD, C independent chains per lane (C = 1: pure latency).
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_lat.hip -o tools/ubench_lat
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int N = 2048;

template <int OP, int C>
__global__ void kern(uint64_t* out, double* dout, uint32_t seed, const double* tab_g) {
  __shared__ double tab[256];
  tab[threadIdx.x & 255] = tab_g[threadIdx.x & 255];
  __syncthreads();
  uint32_t a[C];
  float f[C];
  double d[C];
  for (int i = 0; i < C; ++i) {
    a[i] = seed * (threadIdx.x + 7 * i + 1);
    f[i] = 0.5f + 1e-3f * (threadIdx.x + i);
    d[i] = 0.5 + 1e-3 * (threadIdx.x + i);
  }
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int n = 0; n < N; ++n) {
#pragma unroll
    for (int i = 0; i < C; ++i) {
      if constexpr (OP == 0) d[i] = __builtin_fma(d[i], 0.999999, 1e-7);          // v_fma_f64
      else if constexpr (OP == 1) f[i] = __builtin_fmaf(f[i], 0.999f, 1e-4f);     // v_fma_f32
      else if constexpr (OP == 2) a[i] = (a[i] ^ 0x9E3779B9u) + (a[i] >> 3);      // int (2 ops)
      else if constexpr (OP == 3) {                                                // v_mad_u64_u32 (+xor)
        const uint64_t p = (uint64_t)0xD2511F53u * a[i];
        a[i] = (uint32_t)(p >> 32) ^ (uint32_t)p;
      } else if constexpr (OP == 4) f[i] = __builtin_amdgcn_logf(f[i]) + 2.0f;    // v_log_f32 (+add)
      else if constexpr (OP == 5) d[i] = tab[__double2int_rz(d[i]) & 255] + d[i];  // ds_read_b64 chain (cvt, and, shl, ds, add)
      else if constexpr (OP == 6) d[i] = d[i] > 0.5 ? d[i] * 0.999999 : d[i] + 1e-3;  // cmp + mul/add + cndmask
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  double z = 0;
  for (int i = 0; i < C; ++i) z += d[i] + f[i] + a[i];
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  dout[blockIdx.x * blockDim.x + threadIdx.x] = z;
}

template <int OP, int C>
void run(const char* name, double ops) {
  uint64_t* out;
  double *dd, *tab;
  const int blocks = 256;
  hipMalloc(&out, blocks * 8);
  hipMalloc(&dd, blocks * 256 * 8);
  hipMalloc(&tab, 256 * 8);
  hipMemset(tab, 0, 256 * 8);
  hipLaunchKernelGGL((kern<OP, C>), dim3(blocks), dim3(256), 0, 0, out, dd, 12345u, tab);
  hipDeviceSynchronize();
  uint64_t h[256];
  hipMemcpy(h, out, blocks * 8, hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < blocks; ++i) m += h[i];
  m /= blocks;
  printf("%-26s chains=%d  cycles per chain-step: %7.2f   per instruction (%.0f/step): %6.2f\n", name, C,
         m / (double(N) * C) * C, ops, m / (double(N) * C * ops));
  hipFree(out);
  hipFree(dd);
  hipFree(tab);
}

#define ALLC(OP, NAME, OPS) run<OP, 1>(NAME, OPS); run<OP, 2>(NAME, OPS); run<OP, 4>(NAME, OPS); run<OP, 8>(NAME, OPS);
int main() {
  ALLC(0, "v_fma_f64", 1)
  ALLC(1, "v_fma_f32", 1)
  ALLC(2, "xor+shr+add", 3)
  ALLC(3, "mad_u64_u32+xor", 2)
  ALLC(4, "v_log_f32+add", 2)
  ALLC(5, "lds table chain", 5)
  ALLC(6, "cmp+mul/add+cndmask", 4)
  return 0;
}
