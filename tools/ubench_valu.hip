// Microbenchmark (tools only): cycles per wave-instruction of the instruction classes in the MH
// step on gfx950, with 1 and 2 waves per SIMD.  Each lane runs 8 independent chains of N ops.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_valu.hip -o /tmp/ubench && /tmp/ubench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int N = 4096;

template <int OP>
__global__ void kern(uint64_t* out, float* fo, double* dout, uint32_t seed) {
  uint32_t a[8];
  float f[8];
  double d[8];
  for (int i = 0; i < 8; ++i) {
    a[i] = seed * (threadIdx.x + 7 * i + 1);
    f[i] = 0.5f + 1e-3f * (threadIdx.x + i);
    d[i] = 0.5 + 1e-3 * (threadIdx.x + i);
  }
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int n = 0; n < N; ++n) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (OP == 0) {  // v_mad_u64_u32 (32x32 -> 64)
        const uint64_t p = (uint64_t)0xD2511F53u * a[i];
        a[i] = (uint32_t)(p >> 32) ^ (uint32_t)p;
      } else if constexpr (OP == 1) {  // v_xor_b32
        a[i] = a[i] ^ (a[i] >> 1);
      } else if constexpr (OP == 2) {  // v_fma_f64
        d[i] = __builtin_fma(d[i], 0.999999, 1e-7);
      } else if constexpr (OP == 3) {  // v_log_f32
        f[i] = __builtin_amdgcn_logf(f[i] + 2.0f);
      } else if constexpr (OP == 4) {  // fp64 exp (ocml)
        d[i] = exp(d[i] * 0.5);
      } else if constexpr (OP == 5) {  // v_fma_f32
        f[i] = __builtin_fmaf(f[i], 0.999f, 1e-4f);
      } else if constexpr (OP == 6) {  // v_mul_hi_u32 only
        a[i] = __umulhi(a[i], 0xD2511F53u) ^ a[i];
      } else if constexpr (OP == 7) {  // v_mul_u32_u24 + xor
        a[i] = __umul24(a[i], 0x9F53u) ^ (a[i] >> 3);
      } else if constexpr (OP == 8) {  // v_mul_lo_u32 + xor
        a[i] = (a[i] * 0xD2511F53u) ^ (a[i] >> 3);
      } else if constexpr (OP == 9) {  // v_add_f64
        d[i] = d[i] + 1e-7;
      } else if constexpr (OP == 10) {  // v_mul_f64
        d[i] = d[i] * 0.9999999;
      } else if constexpr (OP == 11) {  // v_exp_f32
        f[i] = __builtin_amdgcn_exp2f(f[i] - 0.5f);
      } else if constexpr (OP == 12) {  // v_sqrt_f32
        f[i] = __builtin_amdgcn_sqrtf(f[i] + 0.25f);
      } else if constexpr (OP == 13) {  // v_cos_f32 (revolutions)
        f[i] = __builtin_amdgcn_cosf(f[i] * 0.5f);
      } else if constexpr (OP == 14) {  // v_add_f32 chain
        f[i] = f[i] + 1e-4f;
      }
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t x = 0;
  float y = 0;
  double z = 0;
  for (int i = 0; i < 8; ++i) {
    x ^= a[i];
    y += f[i];
    z += d[i];
  }
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  fo[blockIdx.x * blockDim.x + threadIdx.x] = y + x;
  dout[blockIdx.x * blockDim.x + threadIdx.x] = z;
}

template <int OP>
void run(const char* name, int ops_per_iter) {
  uint64_t* out;
  float* fo;
  double* dd;
  const int blocks = 1024;
  hipMalloc(&out, blocks * 8);
  hipMalloc(&fo, blocks * 256 * 4);
  hipMalloc(&dd, blocks * 256 * 8);
  for (int wps : {1, 2}) {  // waves per SIMD: blocks of 256 (4 waves = 1 per SIMD) x blocks per CU
    const int nb = 256 * wps;
    hipLaunchKernelGGL(kern<OP>, dim3(nb), dim3(256), 0, 0, out, fo, dd, 12345u);
    hipDeviceSynchronize();
    uint64_t h[2048];
    hipMemcpy(h, out, nb * 8, hipMemcpyDeviceToHost);
    double m = 0;
    for (int i = 0; i < nb; ++i) m += h[i];
    m /= nb;
    // s_memtime = shader clock; per wave-instruction cost = cycles / (N * 8 * ops)
    printf("%-22s waves/SIMD=%d  cycles per wave-instruction: %6.2f\n", name, wps, m / (double(N) * 8 * ops_per_iter));
  }
  hipFree(out);
  hipFree(fo);
  hipFree(dd);
}

int main() {
  run<0>("mad_u64_u32 + xor", 2);
  run<6>("mul_hi_u32 + xor", 2);
  run<1>("xor + shift", 2);
  run<5>("v_fma_f32", 1);
  run<2>("v_fma_f64", 1);
  run<3>("v_log_f32 + add", 2);
  run<4>("exp(double) ocml", 1);
  run<7>("mul_u32_u24 + xor + shr", 3);
  run<8>("mul_lo_u32 + xor + shr", 3);
  run<9>("v_add_f64", 1);
  run<10>("v_mul_f64", 1);
  run<11>("v_exp_f32 + add", 2);
  run<12>("v_sqrt_f32 + add", 2);
  run<13>("v_cos_f32 + mul", 2);
  run<14>("v_add_f32", 1);
  return 0;
}
