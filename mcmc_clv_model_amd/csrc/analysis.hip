// Posterior analysis on device: computed from level-1 draws that are already
// in HBM (a full-sink sampler) or uploaded from the caller's numpy arrays.
//
//   clv_predict*        posterior-predictive future transactions (bivariate/mcmc.py:506-546) and
//                       lognormal spend totals (trivariate/mcmc.py:660-749)
//   clv_track*          weekly cumulative-repeat-transactions tracking curve
//                       (bivariate/analysis_abe.py:444-464)
//   clv_level1_summary* per-customer posterior statistics of Table 4 (utils/analysis_bi_helpers.py:
//                       post_mean_lambdas :15-20, post_mean_mus :22-27, compute_table4 :75-107)
//   clv_chain_total_loglik*  analysis_bi_helpers.py:52-72
//
// Random numbers: Philox4x32-10 keyed by the caller's seed, counter (customer or week, flat draw
// index, slot, stream); the reference draws from one numpy Generator, so parity is distributional
// (tests/test_gpu_analysis.py).  Statistics are exact: the means sum the draws in the reference's
// order (numpy's axis-0 reduction is sequential over draws) and the percentiles apply numpy's
// 'linear' rule to exactly sorted draws.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_segmented_radix_sort.hpp>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "internal.h"
#include "philox.h"

using namespace clv;

namespace {

enum : uint32_t { STREAM_PREDICT = 2u, STREAM_TRACK = 3u };
constexpr uint32_t SLOT_SPEND0 = 1u << 20;  // spend normals of a customer-draw: slots SLOT_SPEND0 + j/2
constexpr int POISSON_MAX_ITER = 1 << 16;   // bound for the inversion / rejection loops

__device__ __forceinline__ u32x4 pblock(uint32_t k0, uint32_t k1, uint32_t a, uint32_t d, uint32_t slot,
                                        uint32_t stream) {
  return philox4x32_10(u32x4{a, d, slot, stream}, k0, k1);
}

// Exact Poisson(m) sample.  m < 10: inversion by sequential search (one uniform); m >= 10: the
// transformed rejection PTRS of Hoermann (1993), as numpy's random_poisson_ptrs.  Each attempt
// uses Philox block (a, d, slot0 + attempt, stream).
__device__ int64_t poisson_draw(double m, uint32_t k0, uint32_t k1, uint32_t a, uint32_t d, uint32_t slot0,
                                uint32_t stream) {
  if (!(m > 0.0)) return 0;
  if (m < 10.0) {
    const u32x4 r = pblock(k0, k1, a, d, slot0, stream);
    const double u = u53(r.x, r.y);
    double p = exp(-m), F = p;
    int64_t k = 0;
    while (u > F && k < POISSON_MAX_ITER) {
      ++k;
      p *= m / (double)k;
      F += p;
    }
    return k;
  }
  const double slam = sqrt(m);
  const double loglam = log(m);
  const double b = 0.931 + 2.53 * slam;
  const double aa = -0.059 + 0.02483 * b;
  const double invalpha = 1.1239 + 1.1328 / (b - 3.4);
  const double vr = 0.9277 - 3.6224 / (b - 2.0);
  for (int it = 0; it < POISSON_MAX_ITER; ++it) {
    const u32x4 r = pblock(k0, k1, a, d, slot0 + (uint32_t)it, stream);
    const double U = u53(r.x, r.y) - 0.5;
    const double V = u53(r.z, r.w);
    const double us = 0.5 - fabs(U);
    const int64_t k = (int64_t)floor((2.0 * aa / us + b) * U + m + 0.43);
    if (us >= 0.07 && V <= vr) return k;
    if (k < 0 || (us < 0.013 && V > us)) continue;
    if (log(V) + log(invalpha) - log(aa / (us * us) + b) <= -m + (double)k * loglam - lgamma((double)k + 1.0)) return k;
  }
  return (int64_t)floor(m);  // unreachable in practice (acceptance > 0.85 per attempt)
}

// ---------------------------------------------------------------------------------------------
// Posterior predictive (bi:533-544, tri:711-741): one lane per (draw, customer).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void predict_kernel(const double* level1, int64_t n_draws, int64_t n, int width,
                                                      const double* T_cal, double T_star, uint32_t k0, uint32_t k1,
                                                      int simulate_spend, double sigma_s, int64_t* x_out,
                                                      double* spend_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double Tc = T_cal[i];
  for (int64_t d = blockIdx.y; d < n_draws; d += gridDim.y) {
    const double* row = level1 + (d * n + i) * width;
    const double lam = row[0];
    const double tau = row[2];
    const bool alive = row[3] > 0.5;
    // tau_star = T_star if alive else clip(tau - T_cal, 0, T_star)   (bi:538-540, tri:717-722)
    double ts = T_star;
    if (!alive) ts = fmin(fmax(tau - Tc, 0.0), T_star);
    const int64_t x = poisson_draw(lam * ts, k0, k1, (uint32_t)i, (uint32_t)d, 0u, STREAM_PREDICT);
    x_out[d * n + i] = x;
    if (simulate_spend) {
      // spend = sum over the x transactions of lognormal(mean=eta, sigma=sigma_s) (tri:730-738;
      // the reference passes the natural-scale eta column as the log-mean — reproduced)
      const double eta = row[4];
      double tot = 0.0;
      for (int64_t j = 0; j < x; j += 2) {
        const u32x4 r = pblock(k0, k1, (uint32_t)i, (uint32_t)d, SLOT_SPEND0 + (uint32_t)(j >> 1), STREAM_PREDICT);
        const double rad = sqrt(-2.0 * log(u53_open0(r.x, r.y)));
        const double ang = 2.0 * u53(r.z, r.w);
        tot += exp(eta + sigma_s * (rad * cospi(ang)));
        if (j + 1 < x) tot += exp(eta + sigma_s * (rad * sinpi(ang)));
      }
      spend_out[d * n + i] = tot;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Weekly tracking (analysis_abe.py:444-464): per draw and week, the reference sums independent
// Poisson(lambda_i * 1[b_i < t <= b_i + tau_i]) over customers; the sum is Poisson(Lambda(t)) with
// Lambda(t) the sum of the active rates, so one exact Poisson draw per (draw, week) has the same
// distribution.  One 64-lane workgroup per draw; each lane owns a difference array over the
// weeks in LDS (deterministic, no atomics), rates are prefix-summed in fixed order.
// ---------------------------------------------------------------------------------------------
constexpr int TRACK_LANES = 64;
constexpr int TRACK_WEEKS = 112;  // weeks per pass (LDS: 64 x 113 doubles)

__global__ __launch_bounds__(TRACK_LANES) void track_kernel(const double* level1, int64_t n_draws, int64_t n,
                                                            int width, const double* birth, const double* times,
                                                            int n_times, uint32_t k0, uint32_t k1, int64_t* inc_out) {
  __shared__ double diff[TRACK_LANES][TRACK_WEEKS + 1];
  __shared__ double tw[TRACK_WEEKS];
  __shared__ double rate[TRACK_WEEKS];
  const int t = threadIdx.x;
  for (int64_t d = blockIdx.x; d < n_draws; d += gridDim.x) {
    for (int w0 = 0; w0 < n_times; w0 += TRACK_WEEKS) {
      const int nw = min(TRACK_WEEKS, n_times - w0);
      for (int j = t; j < nw; j += TRACK_LANES) tw[j] = times[w0 + j];
      for (int j = 0; j <= TRACK_WEEKS; ++j) diff[t][j] = 0.0;
      __syncthreads();
      for (int64_t i = t; i < n; i += TRACK_LANES) {
        const double* row = level1 + (d * n + i) * width;
        const double lam = row[0], tau = row[2], b = birth[i];
        // first week with t > b, first week with t > b + tau (times ascending)
        int lo = 0, hi = nw;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (tw[mid] > b) hi = mid; else lo = mid + 1;
        }
        const int jl = lo;
        const double e = b + tau;
        lo = jl;
        hi = nw;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (tw[mid] > e) hi = mid; else lo = mid + 1;
        }
        const int jh = lo;
        if (jl < jh) {
          diff[t][jl] += lam;
          diff[t][jh] -= lam;
        }
      }
      __syncthreads();
      if (t == 0) {
        double run = 0.0;
        for (int j = 0; j < nw; ++j) {
          double col = 0.0;
          for (int q = 0; q < TRACK_LANES; ++q) col += diff[q][j];
          run += col;
          rate[j] = run > 0.0 ? run : 0.0;
        }
      }
      __syncthreads();
      for (int j = t; j < nw; j += TRACK_LANES)
        inc_out[d * n_times + w0 + j] = poisson_draw(rate[j], k0, k1, (uint32_t)(w0 + j), (uint32_t)d, 0u, STREAM_TRACK);
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Level-1 summaries
// ---------------------------------------------------------------------------------------------
enum : int { SUM_MEAN_LAMBDA = 0, SUM_MEAN_MU, SUM_MEAN_MU_CAP, SUM_MEAN_Z, SUM_MEAN_TAU, SUM_MEAN_ETA, SUM_N_MEANS };

// Sequential sums over draws, in draw order (numpy's axis-0 reduction), divided by n_draws.
__global__ __launch_bounds__(256) void mean_kernel(const double* level1, int64_t n_draws, int64_t n, int width,
                                                   double mu_cap, double* out /*[n][CLV_N_L1_STATS]*/) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double s[SUM_N_MEANS] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  for (int64_t d = 0; d < n_draws; ++d) {
    const double* row = level1 + (d * n + i) * width;
    s[SUM_MEAN_LAMBDA] += row[0];
    s[SUM_MEAN_MU] += row[1];
    s[SUM_MEAN_MU_CAP] += fmin(row[1], mu_cap);  // np.clip(mu, None, cap)
    s[SUM_MEAN_TAU] += row[2];
    s[SUM_MEAN_Z] += row[3];
    if (width > 4) s[SUM_MEAN_ETA] += row[4];
  }
  double* o = out + i * CLV_N_L1_STATS;
  o[CLV_L1_MEAN_LAMBDA] = s[SUM_MEAN_LAMBDA] / (double)n_draws;
  o[CLV_L1_MEAN_MU] = s[SUM_MEAN_MU] / (double)n_draws;
  o[CLV_L1_MEAN_MU_CAPPED] = s[SUM_MEAN_MU_CAP] / (double)n_draws;
  o[CLV_L1_MEAN_Z] = s[SUM_MEAN_Z] / (double)n_draws;
  o[CLV_L1_MEAN_TAU] = s[SUM_MEAN_TAU] / (double)n_draws;
  o[CLV_L1_MEAN_ETA] = width > 4 ? s[SUM_MEAN_ETA] / (double)n_draws : 0.0;
}

// Column `col` of customers [i0, i0 + nc) transposed to [customer][draw] (the sort's segments).
__global__ __launch_bounds__(256) void gather_kernel(const double* level1, int64_t n_draws, int64_t n, int width,
                                                     int col, int64_t i0, int64_t nc, double* seg) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nc * n_draws) return;
  const int64_t d = e / nc, c = e - d * nc;  // consecutive lanes: consecutive customers (coalesced-ish reads)
  seg[c * n_draws + d] = level1[(d * n + i0 + c) * width + col];
}

__global__ void offsets_kernel(int64_t nc, int64_t n_draws, uint32_t* off) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c <= nc) off[c] = (uint32_t)(c * n_draws);
}

// CLV_SINK_SUMMARY_PCT: column col (0 lambda, 1 mu) of customers [i0, i0 + nc) from the sampler's
// float32 store [chain * draw][n] to [customer][chain * draw] (the sort's segments).
__global__ __launch_bounds__(256) void gather_q_kernel(const float2* q, int64_t n_draws, int64_t n, int col,
                                                       int64_t i0, int64_t nc, float* seg) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nc * n_draws) return;
  const int64_t d = e / nc, c = e - d * nc;  // consecutive lanes: consecutive customers (coalesced reads)
  const float2 v = q[d * n + i0 + c];
  seg[c * n_draws + d] = col ? v.y : v.x;
}

// CLV_SINK_SUMMARY_PCT: per-customer means from the running sums, pooled over chains (chain order).
__global__ __launch_bounds__(256) void sums_mean_kernel(const double* sums, int n_chains, int64_t n, int64_t n_stored,
                                                        int D, double* out /*[n][CLV_N_L1_STATS]*/) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int stat[6] = {CLV_SUM_LAMBDA, CLV_SUM_MU, CLV_SUM_MU_CAPPED, CLV_SUM_Z, CLV_SUM_TAU, CLV_SUM_ETA};
  const int dst[6] = {CLV_L1_MEAN_LAMBDA, CLV_L1_MEAN_MU, CLV_L1_MEAN_MU_CAPPED, CLV_L1_MEAN_Z, CLV_L1_MEAN_TAU,
                      CLV_L1_MEAN_ETA};
  const double tot = (double)n_chains * (double)n_stored;
  for (int k = 0; k < 6; ++k) {
    double acc = 0.0;
    for (int c = 0; c < n_chains; ++c) acc += sums[((int64_t)c * CLV_N_SUM_STATS + stat[k]) * n + i];
    out[i * CLV_N_L1_STATS + dst[k]] = (k == 5 && D != 3) ? 0.0 : acc / tot;
  }
}

// numpy.percentile(a, q, method='linear') of a sorted segment (numpy/lib/_function_base_impl.py:
// virtual index (n-1) q, floor/next neighbours, _lerp with the t >= 0.5 branch); float32 segments
// (the percentile store) are widened to double before the interpolation, as numpy would on them.
template <class T>
__device__ double np_percentile_sorted(const T* a, int64_t n, double q_percent) {
  const double q = q_percent / 100.0;
  const double v = (double)(n - 1) * q;
  int64_t prev, next;
  if (v >= (double)(n - 1)) {
    prev = next = n - 1;
  } else if (v < 0.0) {
    prev = next = 0;
  } else {
    prev = (int64_t)floor(v);
    next = prev + 1;
  }
  const double gamma = v - floor(v);
  const double lo = (double)a[prev], hi = (double)a[next];
  const double diff = hi - lo;
  return gamma >= 0.5 ? hi - diff * (1.0 - gamma) : lo + diff * gamma;
}

template <class T>
__global__ __launch_bounds__(256) void percentile_kernel(const T* sorted, int64_t nc, int64_t n_draws,
                                                         int64_t i0, int col_lo, int col_hi, double* out) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nc) return;
  const T* a = sorted + c * n_draws;
  double* o = out + (i0 + c) * CLV_N_L1_STATS;
  o[col_lo] = np_percentile_sorted(a, n_draws, 2.5);
  o[col_hi] = np_percentile_sorted(a, n_draws, 97.5);
}

// chain_total_loglik: per draw, sum over customers of x log(lam) + (1-z) log(mu)
// - (lam+mu)(z T + (1-z) tau) - lgamma(x+1); fixed-order block reduction per draw.
__global__ __launch_bounds__(256) void loglik_kernel(const double* level1, int64_t n_draws, int64_t n, int width,
                                                     const int32_t* x, const double* T_cal, double* per_draw) {
  __shared__ double red[256];
  for (int64_t d = blockIdx.x; d < n_draws; d += gridDim.x) {
    double acc = 0.0;
    for (int64_t i = threadIdx.x; i < n; i += 256) {
      const double* row = level1 + (d * n + i) * width;
      const double lam = row[0], mu = row[1], tau = row[2];
      const double z = row[3] > 0.5 ? 1.0 : 0.0;
      const double xi = (double)x[i];
      acc += x[i] * log(lam) + (1.0 - z) * log(mu) - (lam + mu) * (z * T_cal[i] + (1.0 - z) * tau) - lgamma(xi + 1.0);
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
      if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
      __syncthreads();
    }
    if (threadIdx.x == 0) per_draw[d] = red[0];
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// Host helpers
// ---------------------------------------------------------------------------------------------
int check_l1(int64_t n_draws, int64_t n, int32_t width) {
  if (n_draws < 1 || n < 1 || (width != 4 && width != 5)) return fail(CLV_EINVAL, "bad level-1 shape");
  if (n > 0xffffffffLL || n_draws > 0xffffffffLL) return fail(CLV_EINVAL, "level-1 shape exceeds the 32-bit Philox counter words");
  return CLV_OK;
}

void seed_key(uint64_t seed, uint32_t* k0, uint32_t* k1) {
  *k0 = (uint32_t)seed;
  *k1 = (uint32_t)(seed >> 32);
}

// Uploads a host level-1 array [n_draws][n][width] (or uses the device pointer as is).
int stage_level1(const double* host, int64_t n_draws, int64_t n, int32_t width, DevBuf& buf, const double** dev,
                 hipStream_t st) {
  const size_t bytes = sizeof(double) * (size_t)n_draws * n * width;
  CLV_HIP(hipMalloc(&buf.p, bytes));
  CLV_HIP(hipMemcpyAsync(buf.p, host, bytes, hipMemcpyHostToDevice, st));
  *dev = (const double*)buf.p;
  return CLV_OK;
}

int predict_dev(const double* l1, int64_t n_draws, int64_t n, int32_t width, const double* dT, double T_star,
                uint64_t seed, int32_t spend, double sigma_s, int64_t* x_future, double* spend_future, hipStream_t st) {
  DevBuf bx, bs;
  CLV_HIP(hipMalloc(&bx.p, sizeof(int64_t) * n_draws * n));
  if (spend) CLV_HIP(hipMalloc(&bs.p, sizeof(double) * n_draws * n));
  uint32_t k0, k1;
  seed_key(seed, &k0, &k1);
  const dim3 grid((unsigned)((n + 255) / 256), (unsigned)std::min<int64_t>(n_draws, 65535));
  hipLaunchKernelGGL(predict_kernel, grid, dim3(256), 0, st, l1, n_draws, n, width, dT, T_star, k0, k1, spend,
                     sigma_s, (int64_t*)bx.p, (double*)bs.p);
  CLV_HIP(hipGetLastError());
  CLV_HIP(hipMemcpyAsync(x_future, bx.p, sizeof(int64_t) * n_draws * n, hipMemcpyDeviceToHost, st));
  if (spend) CLV_HIP(hipMemcpyAsync(spend_future, bs.p, sizeof(double) * n_draws * n, hipMemcpyDeviceToHost, st));
  CLV_HIP(hipStreamSynchronize(st));
  return CLV_OK;
}

int track_dev(const double* l1, int64_t n_draws, int64_t n, int32_t width, const double* birth, const double* times,
              int32_t n_times, uint64_t seed, double* inc_mean, hipStream_t st) {
  if (n_times < 1) return fail(CLV_EINVAL, "n_times must be >= 1");
  for (int j = 1; j < n_times; ++j)
    if (!(times[j] >= times[j - 1])) return fail(CLV_EINVAL, "times must be ascending");
  DevBuf bb, bt, bi;
  CLV_HIP(hipMalloc(&bb.p, sizeof(double) * n));
  CLV_HIP(hipMalloc(&bt.p, sizeof(double) * n_times));
  CLV_HIP(hipMalloc(&bi.p, sizeof(int64_t) * n_draws * n_times));
  CLV_HIP(hipMemcpyAsync(bb.p, birth, sizeof(double) * n, hipMemcpyHostToDevice, st));
  CLV_HIP(hipMemcpyAsync(bt.p, times, sizeof(double) * n_times, hipMemcpyHostToDevice, st));
  uint32_t k0, k1;
  seed_key(seed, &k0, &k1);
  hipLaunchKernelGGL(track_kernel, dim3((unsigned)std::min<int64_t>(n_draws, 1 << 20)), dim3(TRACK_LANES), 0, st,
                     l1, n_draws, n, width, (const double*)bb.p, (const double*)bt.p, n_times, k0, k1,
                     (int64_t*)bi.p);
  CLV_HIP(hipGetLastError());
  std::vector<int64_t> inc((size_t)n_draws * n_times);
  CLV_HIP(hipMemcpyAsync(inc.data(), bi.p, sizeof(int64_t) * inc.size(), hipMemcpyDeviceToHost, st));
  CLV_HIP(hipStreamSynchronize(st));
  // inc_hb_weekly[t] += inc.sum() over draws, then /= n_draws (analysis_abe.py:461-464)
  for (int j = 0; j < n_times; ++j) {
    double acc = 0.0;
    for (int64_t d = 0; d < n_draws; ++d) acc += (double)inc[(size_t)d * n_times + j];
    inc_mean[j] = acc / (double)n_draws;
  }
  return CLV_OK;
}

int summary_dev(const double* l1, int64_t n_draws, int64_t n, int32_t width, double mu_cap, double* out,
                hipStream_t st) {
  DevBuf bo;
  CLV_HIP(hipMalloc(&bo.p, sizeof(double) * n * CLV_N_L1_STATS));
  double* dout = (double*)bo.p;
  hipLaunchKernelGGL(mean_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, l1, n_draws, n, width, mu_cap,
                     dout);
  CLV_HIP(hipGetLastError());
  // percentiles: customers in batches of <= 2^27 keys, exact segmented radix sort per customer
  const int64_t per_batch = std::max<int64_t>(1, std::min<int64_t>(n, (int64_t(1) << 27) / n_draws));
  DevBuf bin, bsorted, boff, btmp;
  const size_t keys = (size_t)per_batch * n_draws;
  CLV_HIP(hipMalloc(&bin.p, sizeof(double) * keys));
  CLV_HIP(hipMalloc(&bsorted.p, sizeof(double) * keys));
  CLV_HIP(hipMalloc(&boff.p, sizeof(uint32_t) * (per_batch + 1)));
  size_t tmp_bytes = 0;
  CLV_HIP(rocprim::segmented_radix_sort_keys((void*)nullptr, tmp_bytes, (const double*)bin.p, (double*)bsorted.p,
                                             (unsigned)keys, (unsigned)per_batch, (const uint32_t*)boff.p,
                                             (const uint32_t*)boff.p + 1, 0, 64, st));
  CLV_HIP(hipMalloc(&btmp.p, std::max<size_t>(tmp_bytes, 16)));
  const int cols[2] = {0, 1};
  const int lo_idx[2] = {CLV_L1_LAMBDA_P025, CLV_L1_MU_P025};
  const int hi_idx[2] = {CLV_L1_LAMBDA_P975, CLV_L1_MU_P975};
  for (int64_t i0 = 0; i0 < n; i0 += per_batch) {
    const int64_t nc = std::min<int64_t>(per_batch, n - i0);
    hipLaunchKernelGGL(offsets_kernel, dim3((unsigned)((nc + 256) / 256)), dim3(256), 0, st, nc, n_draws,
                       (uint32_t*)boff.p);
    for (int q = 0; q < 2; ++q) {
      const int64_t ne = nc * n_draws;
      hipLaunchKernelGGL(gather_kernel, dim3((unsigned)((ne + 255) / 256)), dim3(256), 0, st, l1, n_draws, n, width,
                         cols[q], i0, nc, (double*)bin.p);
      CLV_HIP(hipGetLastError());
      size_t tb = tmp_bytes;
      CLV_HIP(rocprim::segmented_radix_sort_keys(btmp.p, tb, (const double*)bin.p, (double*)bsorted.p, (unsigned)ne,
                                                 (unsigned)nc, (const uint32_t*)boff.p, (const uint32_t*)boff.p + 1,
                                                 0, 64, st));
      hipLaunchKernelGGL(percentile_kernel<double>, dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, st,
                         (const double*)bsorted.p, nc, n_draws, i0, lo_idx[q], hi_idx[q], dout);
      CLV_HIP(hipGetLastError());
    }
  }
  CLV_HIP(hipMemcpyAsync(out, dout, sizeof(double) * n * CLV_N_L1_STATS, hipMemcpyDeviceToHost, st));
  CLV_HIP(hipStreamSynchronize(st));
  return CLV_OK;
}

// CLV_SINK_SUMMARY_PCT sampler: means from the running sums, exact order statistics of the float32
// (lambda, mu) store (segmented radix sort on 32-bit keys, customers in batches of <= 2^27 keys).
int summary_pct_dev(clv_sampler* s, double* out) {
  const Geometry& g = s->g;
  const int64_t n = g.n, n_draws = (int64_t)g.n_chains * g.n_draws;
  hipStream_t st = s->stream;
  DevBuf bo;
  CLV_HIP(hipMalloc(&bo.p, sizeof(double) * n * CLV_N_L1_STATS));
  double* dout = (double*)bo.p;
  hipLaunchKernelGGL(sums_mean_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, (const double*)s->d_sums,
                     g.n_chains, n, (int64_t)g.n_draws, g.D, dout);
  CLV_HIP(hipGetLastError());
  const int64_t per_batch = std::max<int64_t>(1, std::min<int64_t>(n, (int64_t(1) << 27) / n_draws));
  DevBuf bin, bsorted, boff, btmp;
  const size_t keys = (size_t)per_batch * n_draws;
  CLV_HIP(hipMalloc(&bin.p, sizeof(float) * keys));
  CLV_HIP(hipMalloc(&bsorted.p, sizeof(float) * keys));
  CLV_HIP(hipMalloc(&boff.p, sizeof(uint32_t) * (per_batch + 1)));
  size_t tmp_bytes = 0;
  CLV_HIP(rocprim::segmented_radix_sort_keys((void*)nullptr, tmp_bytes, (const float*)bin.p, (float*)bsorted.p,
                                             (unsigned)keys, (unsigned)per_batch, (const uint32_t*)boff.p,
                                             (const uint32_t*)boff.p + 1, 0, 32, st));
  CLV_HIP(hipMalloc(&btmp.p, std::max<size_t>(tmp_bytes, 16)));
  const int lo_idx[2] = {CLV_L1_LAMBDA_P025, CLV_L1_MU_P025};
  const int hi_idx[2] = {CLV_L1_LAMBDA_P975, CLV_L1_MU_P975};
  for (int64_t i0 = 0; i0 < n; i0 += per_batch) {
    const int64_t nc = std::min<int64_t>(per_batch, n - i0);
    hipLaunchKernelGGL(offsets_kernel, dim3((unsigned)((nc + 256) / 256)), dim3(256), 0, st, nc, n_draws,
                       (uint32_t*)boff.p);
    for (int q = 0; q < 2; ++q) {
      const int64_t ne = nc * n_draws;
      hipLaunchKernelGGL(gather_q_kernel, dim3((unsigned)((ne + 255) / 256)), dim3(256), 0, st,
                         (const float2*)s->d_qstore, n_draws, n, q, i0, nc, (float*)bin.p);
      CLV_HIP(hipGetLastError());
      size_t tb = tmp_bytes;
      CLV_HIP(rocprim::segmented_radix_sort_keys(btmp.p, tb, (const float*)bin.p, (float*)bsorted.p, (unsigned)ne,
                                                 (unsigned)nc, (const uint32_t*)boff.p, (const uint32_t*)boff.p + 1,
                                                 0, 32, st));
      hipLaunchKernelGGL(percentile_kernel<float>, dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, st,
                         (const float*)bsorted.p, nc, n_draws, i0, lo_idx[q], hi_idx[q], dout);
      CLV_HIP(hipGetLastError());
    }
  }
  CLV_HIP(hipMemcpyAsync(out, dout, sizeof(double) * n * CLV_N_L1_STATS, hipMemcpyDeviceToHost, st));
  CLV_HIP(hipStreamSynchronize(st));
  return CLV_OK;
}

int loglik_dev(const double* l1, int64_t n_draws, int64_t n, int32_t width, const int32_t* dx, const double* dT,
               double* mean_out, hipStream_t st) {
  DevBuf bp;
  CLV_HIP(hipMalloc(&bp.p, sizeof(double) * n_draws));
  hipLaunchKernelGGL(loglik_kernel, dim3((unsigned)std::min<int64_t>(n_draws, 1 << 20)), dim3(256), 0, st, l1,
                     n_draws, n, width, dx, dT, (double*)bp.p);
  CLV_HIP(hipGetLastError());
  std::vector<double> per(n_draws);
  CLV_HIP(hipMemcpyAsync(per.data(), bp.p, sizeof(double) * n_draws, hipMemcpyDeviceToHost, st));
  CLV_HIP(hipStreamSynchronize(st));
  double acc = 0.0;  // np.mean(totals)
  for (double v : per) acc += v;
  *mean_out = acc / (double)n_draws;
  return CLV_OK;
}

int sampler_l1(clv_sampler* s, const double** l1, int64_t* n_draws, int32_t* width) {
  if (!s) return fail(CLV_EINVAL, "null sampler");
  if (!s->d_level1) return fail(CLV_ESTATE, "level-1 draws are on the device only with draw_sink == CLV_SINK_FULL");
  int64_t stored = 0;
  if (s->sweeps_done > s->g.burnin) stored = (s->sweeps_done - 1 - s->g.burnin) / s->g.thin + 1;
  stored = std::min<int64_t>(stored, s->g.n_draws);
  if (stored < (int64_t)s->g.n_draws) return fail(CLV_ESTATE, "the run has not stored all of its draws yet");
  CLV_HIP(hipSetDevice(s->device));
  CLV_HIP(hipStreamSynchronize(s->stream));
  *l1 = s->d_level1;
  *n_draws = (int64_t)s->g.n_chains * s->g.n_draws;  // [chain][draw] flattened = np.vstack order
  *width = s->g.D + 2;
  return check_l1(*n_draws, s->g.n, *width);
}

}  // namespace

extern "C" {

int clv_predict(int32_t device, const double* level1, int64_t n_draws, int64_t n, int32_t width, const double* T_cal,
                double T_star, uint64_t seed, int32_t simulate_spend, double sigma_s, int64_t* x_future,
                double* spend_future) {
  int rc = check_l1(n_draws, n, width);
  if (rc) return rc;
  if (!level1 || !T_cal || !x_future || (simulate_spend && (!spend_future || width < 5)))
    return fail(CLV_EINVAL, "bad arguments (spend needs width 5 and an output buffer)");
  DeviceScope ds(device);
  DevBuf b1, bT;
  const double* l1;
  rc = stage_level1(level1, n_draws, n, width, b1, &l1, nullptr);
  if (rc) return rc;
  CLV_HIP(hipMalloc(&bT.p, sizeof(double) * n));
  CLV_HIP(hipMemcpy(bT.p, T_cal, sizeof(double) * n, hipMemcpyHostToDevice));
  return predict_dev(l1, n_draws, n, width, (const double*)bT.p, T_star, seed, simulate_spend, sigma_s, x_future,
                     spend_future, nullptr);
}

int clv_predict_sampler(clv_sampler* s, double T_star, uint64_t seed, int32_t simulate_spend, double sigma_s,
                        int64_t* x_future, double* spend_future) {
  const double* l1;
  int64_t nd;
  int32_t w;
  int rc = sampler_l1(s, &l1, &nd, &w);
  if (rc) return rc;
  if (!x_future || (simulate_spend && (!spend_future || w < 5))) return fail(CLV_EINVAL, "bad arguments");
  return predict_dev(l1, nd, s->g.n, w, s->d_T, T_star, seed, simulate_spend, sigma_s, x_future, spend_future,
                     s->stream);
}

int clv_track(int32_t device, const double* level1, int64_t n_draws, int64_t n, int32_t width,
              const double* birth_week, const double* times, int32_t n_times, uint64_t seed, double* inc_weekly) {
  int rc = check_l1(n_draws, n, width);
  if (rc) return rc;
  if (!level1 || !birth_week || !times || !inc_weekly) return fail(CLV_EINVAL, "null argument");
  DeviceScope ds(device);
  DevBuf b1;
  const double* l1;
  rc = stage_level1(level1, n_draws, n, width, b1, &l1, nullptr);
  if (rc) return rc;
  return track_dev(l1, n_draws, n, width, birth_week, times, n_times, seed, inc_weekly, nullptr);
}

int clv_track_sampler(clv_sampler* s, const double* birth_week, const double* times, int32_t n_times, uint64_t seed,
                      double* inc_weekly) {
  const double* l1;
  int64_t nd;
  int32_t w;
  int rc = sampler_l1(s, &l1, &nd, &w);
  if (rc) return rc;
  if (!birth_week || !times || !inc_weekly) return fail(CLV_EINVAL, "null argument");
  return track_dev(l1, nd, s->g.n, w, birth_week, times, n_times, seed, inc_weekly, s->stream);
}

int clv_level1_summary(int32_t device, const double* level1, int64_t n_draws, int64_t n, int32_t width,
                       double mu_cap, double* out) {
  int rc = check_l1(n_draws, n, width);
  if (rc) return rc;
  if (!level1 || !out) return fail(CLV_EINVAL, "null argument");
  DeviceScope ds(device);
  DevBuf b1;
  const double* l1;
  rc = stage_level1(level1, n_draws, n, width, b1, &l1, nullptr);
  if (rc) return rc;
  return summary_dev(l1, n_draws, n, width, mu_cap, out, nullptr);
}

int clv_level1_summary_sampler(clv_sampler* s, double mu_cap, double* out) {
  if (s && !s->d_level1 && s->d_qstore) {  // CLV_SINK_SUMMARY_PCT
    if (!out) return fail(CLV_EINVAL, "null argument");
    if (mu_cap != CLV_SUMMARY_MU_CAP) return fail(CLV_EINVAL, "a summary sampler's capped mean uses mu_cap = CLV_SUMMARY_MU_CAP");
    int64_t stored = 0;
    if (s->sweeps_done > s->g.burnin) stored = (s->sweeps_done - 1 - s->g.burnin) / s->g.thin + 1;
    if (std::min<int64_t>(stored, s->g.n_draws) < (int64_t)s->g.n_draws)
      return fail(CLV_ESTATE, "the run has not stored all of its draws yet");
    CLV_HIP(hipSetDevice(s->device));
    CLV_HIP(hipStreamSynchronize(s->stream));
    return summary_pct_dev(s, out);
  }
  const double* l1;
  int64_t nd;
  int32_t w;
  int rc = sampler_l1(s, &l1, &nd, &w);
  if (rc) return rc;
  if (!out) return fail(CLV_EINVAL, "null argument");
  return summary_dev(l1, nd, s->g.n, w, mu_cap, out, s->stream);
}

int clv_chain_total_loglik(int32_t device, const double* level1, int64_t n_draws, int64_t n, int32_t width,
                           const int32_t* x, const double* T_cal, double* mean_total) {
  int rc = check_l1(n_draws, n, width);
  if (rc) return rc;
  if (!level1 || !x || !T_cal || !mean_total) return fail(CLV_EINVAL, "null argument");
  DeviceScope ds(device);
  DevBuf b1, bx, bT;
  const double* l1;
  rc = stage_level1(level1, n_draws, n, width, b1, &l1, nullptr);
  if (rc) return rc;
  CLV_HIP(hipMalloc(&bx.p, sizeof(int32_t) * n));
  CLV_HIP(hipMalloc(&bT.p, sizeof(double) * n));
  CLV_HIP(hipMemcpy(bx.p, x, sizeof(int32_t) * n, hipMemcpyHostToDevice));
  CLV_HIP(hipMemcpy(bT.p, T_cal, sizeof(double) * n, hipMemcpyHostToDevice));
  return loglik_dev(l1, n_draws, n, width, (const int32_t*)bx.p, (const double*)bT.p, mean_total, nullptr);
}

int clv_chain_total_loglik_sampler(clv_sampler* s, double* mean_total) {
  const double* l1;
  int64_t nd;
  int32_t w;
  int rc = sampler_l1(s, &l1, &nd, &w);
  if (rc) return rc;
  if (!mean_total) return fail(CLV_EINVAL, "null argument");
  return loglik_dev(l1, nd, s->g.n, w, s->d_x, s->d_T, mean_total, s->stream);
}

}  // extern "C"
