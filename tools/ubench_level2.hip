// Microbenchmark (tools only): latency of the Philox-mode level-2 draw on gfx950 — the serial link
// of every sweep's hand-off in the persistent kernel — with the IEEE sqrt /
// division sequences (NR = 0) against the rsq / rcp estimate + Newton forms (NR = 1), and the
// dependent latency of the operations themselves.  One workgroup per launch, lane 0 of wavefront 0
// times each phase with s_memtime (shader clock) over many iterations.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/ubench_level2.hip -o tools/ubench_level2
#include "../mcmc_clv_model_amd/csrc/kernels.hip"

#include <cmath>
#include <cstdio>
#include <vector>

using namespace clv;

constexpr int IN_PRIOR = 0, IN_TOT = 198, IN_IW = 240, IN_CHI = 244, IN_NOISE = 248, IN_N = 280;
constexpr int OUT_N = HS + 9;

template <int D, int K, int LANE0, bool NR>
__global__ __launch_bounds__(256) void ub_draw(const double* in, double* out, unsigned long long* cyc, int iters) {
  constexpr int NS = K * D + D * (D + 1) / 2 + 1;
  __shared__ double tot[NS];
  __shared__ double var_iw[4], var_chi[4], var_noise[32];
  __shared__ L2Scratch l2;
  __shared__ double Hs[HS];
  const int tid = threadIdx.x;
  stage_prior(in + IN_PRIOR, &l2);
  if (tid < NS) tot[tid] = in[IN_TOT + tid];
  if (tid < 4) {
    var_iw[tid] = in[IN_IW + tid];
    var_chi[tid] = in[IN_CHI + tid];
  }
  if (tid < 32) var_noise[tid] = in[IN_NOISE + tid];
  if (tid < HS) Hs[tid] = 0.0;
  __syncthreads();
  if (tid == 0) bartlett_inverse<D>(var_iw, var_chi, l2.Ai);
  __syncthreads();
  unsigned long long c_draw = 0, c_fin = 0;
  for (int it = 0; it < iters; ++it) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    level2_draw_fast<D, K, LANE0, NR>(tot, var_iw, var_chi, var_noise, l2.Ai, &l2);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) {
      double Sig[D][D];
#pragma unroll
      for (int p = 0; p < D; ++p)
#pragma unroll
        for (int q = 0; q < D; ++q) Sig[p][q] = l2.Sig[p * D + q];
      finalize_hyper<D, K, true, NR>(l2.beta, Sig, 2.0, Hs);
    }
    __syncthreads();
    const unsigned long long t2 = __builtin_amdgcn_s_memtime();
    if (it > 0) {
      c_draw += t1 - t0;
      c_fin += t2 - t1;
    }
    __syncthreads();
  }
  if (tid == 0) {
    cyc[0] = c_draw;
    cyc[1] = c_fin;
  }
  if (tid < HS) out[tid] = Hs[tid];
  if (tid < D * D) out[HS + tid] = l2.Sig[tid];
}

// dependent chains of one operation (every lane the same work)
template <int OP>
__global__ void ub_op(const double* in, double* out, unsigned long long* cyc, int iters) {
  double x = in[threadIdx.x & 7] + 2.0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    if constexpr (OP == 0) x = __builtin_fma(x, 0.999999, 1e-3);
    else if constexpr (OP == 1) x = sqrt(x) + 1.5;
    else if constexpr (OP == 2) x = 3.0 / x + 1.5;
    else if constexpr (OP == 3) x = x * rsq_nr(x) + 1.5;
    else if constexpr (OP == 4) x = 3.0 * rcp_nr(x) + 1.5;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
  out[threadIdx.x] = x;
}

static unsigned long long* g_cyc;
static double *g_in, *g_out;

template <int D, int K>
static void make_input(std::vector<double>& h) {
  // V = I / n, chol V = I / sqrt(n), A0 B0 = 0, S0 + B0'A0B0 = nu0 I, X'Y ~ 0.1 n, Y'Y ~ n (PD S_n)
  const double n = 23570.0;
  h.assign(IN_N, 0.0);
  for (int k = 0; k < K; ++k) {
    h[IN_PRIOR + k * K + k] = 1.0 / n;
    h[IN_PRIOR + 81 + k * K + k] = 1.0 / std::sqrt(n);
  }
  for (int d = 0; d < D; ++d) h[IN_PRIOR + 189 + d * D + d] = D + 2.0;
  for (int q = 0; q < K * D; ++q) h[IN_TOT + q] = 0.1 * n * (1.0 + 0.37 * q) * (q % 2 ? -1 : 1);
  int t = K * D;
  for (int p = 0; p < D; ++p)
    for (int q = p; q < D; ++q) h[IN_TOT + t++] = p == q ? n * (1.0 + 0.5 * p) : 0.2 * n;
  h[IN_TOT + t] = -3.0 * n;
  for (int q = 0; q < 3; ++q) h[IN_IW + q] = 0.3 - 0.2 * q;
  for (int q = 0; q < D; ++q) h[IN_CHI + q] = n - q + 0.5;
  for (int q = 0; q < 32; ++q) h[IN_NOISE + q] = std::sin(1.0 + q);
}

template <int D, int K, int LANE0, bool NR>
static void run_draw(int iters, std::vector<double>& res, double* c_draw, double* c_fin) {
  std::vector<double> h;
  make_input<D, K>(h);
  hipMemcpy(g_in, h.data(), IN_N * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL((ub_draw<D, K, LANE0, NR>), dim3(1), dim3(256), 0, 0, g_in, g_out, g_cyc, iters);
  hipDeviceSynchronize();
  unsigned long long c[2];
  hipMemcpy(c, g_cyc, 16, hipMemcpyDeviceToHost);
  res.resize(OUT_N);
  hipMemcpy(res.data(), g_out, OUT_N * 8, hipMemcpyDeviceToHost);
  *c_draw = double(c[0]) / (iters - 1);
  *c_fin = double(c[1]) / (iters - 1);
}

template <int D, int K, int LANE0>
static void compare(const char* name) {
  const int iters = 2001;
  std::vector<double> r0, r1;
  double d0, f0, d1, f1;
  run_draw<D, K, LANE0, false>(iters, r0, &d0, &f0);
  run_draw<D, K, LANE0, true>(iters, r1, &d1, &f1);
  double worst = 0.0;
  for (int i = 0; i < OUT_N; ++i) {
    if (r0[i] == 0.0 && r1[i] == 0.0) continue;
    const double rel = std::fabs(r1[i] - r0[i]) / std::fabs(r0[i]);
    worst = std::fmax(worst, rel);
  }
  printf("%-24s IEEE: draw %7.0f + finalize %6.0f cycles   NR: draw %7.0f + finalize %6.0f cycles   "
         "(saved %5.0f, %.3f us at 2.4 GHz)  max rel diff of (beta, Sigma, hyper) %.2e\n",
         name, d0, f0, d1, f1, (d0 + f0) - (d1 + f1), ((d0 + f0) - (d1 + f1)) / 2400.0, worst);
}

template <int OP>
static void op_lat(const char* name) {
  const int iters = 4096;
  std::vector<double> h(8, 1.0);
  hipMemcpy(g_in, h.data(), 64, hipMemcpyHostToDevice);
  hipLaunchKernelGGL((ub_op<OP>), dim3(1), dim3(64), 0, 0, g_in, g_out, g_cyc, iters);
  hipDeviceSynchronize();
  unsigned long long c;
  hipMemcpy(&c, g_cyc, 8, hipMemcpyDeviceToHost);
  printf("%-34s %6.1f cycles per dependent step\n", name, double(c) / iters);
}

int main() {
  hipMalloc(&g_cyc, 64);
  hipMalloc(&g_in, IN_N * 8);
  hipMalloc(&g_out, 4096 * 8);
  op_lat<0>("v_fma_f64");
  op_lat<1>("sqrt(double) + add (IEEE)");
  op_lat<2>("3 / x + add (IEEE)");
  op_lat<3>("x * rsq_nr(x) + add");
  op_lat<4>("3 * rcp_nr(x) + add");
  compare<2, 2, 6>("c2  D=2 K=2 (one lane)");
  compare<3, 3, 6>("c3  D=3 K=3 (element)");
  compare<3, 3, 12>("c3  D=3 K=3 (one lane)");
  compare<2, 5, 6>("c4  D=2 K=5 (element)");
  compare<2, 5, 12>("c4  D=2 K=5 (one lane)");
  compare<3, 9, 6>("c5  D=3 K=9 (element)");
  return 0;
}
