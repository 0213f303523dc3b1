// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE for the sweep kernel's access widths on gfx950
// (MI355X_MICROARCH.md "HBM": other widths than 16 B/lane are uncalibrated).  Each kernel moves a
// known byte count through HBM (512 MiB arrays, beyond the 256 MiB Infinity Cache):
//   read4 / read8 / read16: coalesced loads of 4 / 8 / 16 B per lane;  write8: 8 B per lane stores.
// Build: hipcc --offload-arch=gfx950 -O3 tools/calib_fetch.hip -o tools/calib_fetch
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr size_t BYTES = 512ull << 20;

__global__ void read4(const unsigned* a, size_t n, unsigned* out) {
  unsigned s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s ^= a[i];
  if (s == 0x12345678u) out[0] = s;
}
__global__ void read8(const double* a, size_t n, double* out) {
  double s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
  if (s == 1.2345) out[0] = s;
}
__global__ void read16(const double2* a, size_t n, double* out) {
  double s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i].x + a[i].y;
  if (s == 1.2345) out[0] = s;
}
__global__ void write8(double* a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = (double)i;
}

int main() {
  void *a, *o;
  if (hipMalloc(&a, BYTES) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) return 1;
  if (hipMemset(a, 0, BYTES) != hipSuccess) return 1;
  const dim3 g(4096), b(256);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(read4, g, b, 0, 0, (const unsigned*)a, BYTES / 4, (unsigned*)o);
    hipLaunchKernelGGL(read8, g, b, 0, 0, (const double*)a, BYTES / 8, (double*)o);
    hipLaunchKernelGGL(read16, g, b, 0, 0, (const double2*)a, BYTES / 16, (double*)o);
    hipLaunchKernelGGL(write8, g, b, 0, 0, (double*)a, BYTES / 8);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  printf("calib: %zu bytes per kernel\n", BYTES);
  return 0;
}
