// Data preparation on device: the event log -> CBS conversion and the
// synthetic Pareto/NBD generator that feed the sampler at 1M-10M customers.
//
//   clv_elog2cbs            utils/elog2cbs2param.py:33-94 (date-based event log, calibration and
//                           hold-out statistics): stable radix sorts by (customer, date), same-day
//                           merge, one lane per customer over its date-ordered events.
//   clv_generate_pareto_abe bivariate/mcmc.py:95-187 (Abe 2009 simulation: covariates, log-normal
//                           heterogeneity, exponential lifetimes, Poisson purchase process) with
//                           the CBS of bi:75-89 formed in the same pass, one lane per customer.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "internal.h"
#include "philox.h"

using namespace clv;

namespace {

template <class T>
int alloc(DevBuf& b, size_t count) {
  CLV_HIP(hipMalloc(&b.p, sizeof(T) * std::max<size_t>(count, 1)));
  return CLV_OK;
}

// ---------------------------------------------------------------------------------------------
// elog2cbs
// ---------------------------------------------------------------------------------------------
__global__ void gather_events(int64_t n, const int64_t* perm, const int64_t* cust, const int64_t* date,
                              const double* sales, int64_t* cust_s, int64_t* date_s, double* sales_s) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t j = perm[i];
  cust_s[i] = cust[j];
  date_s[i] = date[j];
  sales_s[i] = sales ? sales[j] : 1.0;  // 'sales' absent -> 1 per event (elog2cbs2param.py:46-47)
}

// flags of the first event of each (customer, date) run, and of each customer
__global__ void run_flags(int64_t n, const int64_t* cust_s, const int64_t* date_s, uint8_t* run_flag,
                          uint8_t* cust_flag) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bool newc = i == 0 || cust_s[i] != cust_s[i - 1];
  run_flag[i] = (newc || date_s[i] != date_s[i - 1]) ? 1 : 0;
  cust_flag[i] = newc ? 1 : 0;
}

// Per customer (its runs are the same-day-merged transactions in date order): the statistics of
// elog2cbs2param.py:70-93.
__global__ void customer_stats(int64_t n_cust, const int64_t* cust_start_ev, const int64_t* run_start,
                               int64_t n_runs, int64_t n_events, const int64_t* cust_s, const int64_t* date_s,
                               const double* sales_s, const int64_t* cust_first_run, double unit_ns,
                               int64_t T_cal_ns, int64_t T_tot_ns, int holdout, int64_t* o_cust, int64_t* o_x,
                               double* o_tx, double* o_litt, double* o_sales, double* o_sales_x, int64_t* o_first,
                               double* o_Tcal, double* o_Tstar, int64_t* o_xstar, double* o_sales_star,
                               uint8_t* o_keep) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n_cust) return;
  const int64_t r0 = cust_first_run[c];
  const int64_t r1 = c + 1 < n_cust ? cust_first_run[c + 1] : n_runs;
  const int64_t first = date_s[run_start[r0]];
  int64_t count = 0, xstar = 0;
  double tmax = -INFINITY, litt = 0.0, sales = 0.0, sales_x = 0.0, sales_star = 0.0, t_prev = 0.0;
  for (int64_t r = r0; r < r1; ++r) {
    const int64_t e0 = run_start[r];
    const int64_t e1 = r + 1 < n_runs ? run_start[r + 1] : n_events;
    const int64_t date = date_s[e0];
    double s = 0.0;  // groupby(['cust', 'date']).agg(sales='sum'), original order within the day
    for (int64_t e = e0; e < e1; ++e) s += sales_s[e];
    const double t = (double)(date - first) / unit_ns;  // (date - first) / np.timedelta64(1, units)
    const double itt = r == r0 ? 0.0 : t - t_prev;     // groupby('cust')['t'].diff().fillna(0)
    t_prev = t;
    if (date <= T_cal_ns) {
      ++count;
      tmax = fmax(tmax, t);
      if (itt > 0.0) litt += log(itt);
      sales += s;
      if (r > r0) sales_x += s;  // s.iloc[1:].sum()
    } else if (holdout && date <= T_tot_ns) {
      ++xstar;
      sales_star += s;
    }
  }
  o_keep[c] = count > 0 ? 1 : 0;  // customers without calibration events have no CBS row
  o_cust[c] = cust_s[cust_start_ev[c]];
  o_x[c] = count - 1;
  o_tx[c] = tmax;
  o_litt[c] = litt;
  o_sales[c] = sales;
  o_sales_x[c] = sales_x;
  o_first[c] = first;
  const double Tc = (double)(T_cal_ns - first) / unit_ns;
  o_Tcal[c] = Tc;
  o_Tstar[c] = holdout ? (double)(T_tot_ns - first) / unit_ns - Tc : 0.0;
  o_xstar[c] = xstar;
  o_sales_star[c] = sales_star;
}

// customer-start flags over runs: run r starts a customer iff its first event starts one
__global__ void cust_flag_of_runs(int64_t n_runs, const int64_t* run_start, const uint8_t* cust_flag_ev,
                                  uint8_t* cust_flag_run) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < n_runs) cust_flag_run[r] = cust_flag_ev[run_start[r]];
}

template <class T>
__global__ void compact(int64_t n, const int64_t* idx, const T* in, T* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = in[idx[i]];
}

template <class KeyT, class ValT>
int sort_pairs(const KeyT* kin, KeyT* kout, const ValT* vin, ValT* vout, int64_t n, hipStream_t st) {
  size_t bytes = 0;
  CLV_HIP(rocprim::radix_sort_pairs((void*)nullptr, bytes, kin, kout, vin, vout, (size_t)n, 0, 8 * sizeof(KeyT), st));
  DevBuf tmp;
  CLV_HIP(hipMalloc(&tmp.p, std::max<size_t>(bytes, 16)));
  CLV_HIP(rocprim::radix_sort_pairs(tmp.p, bytes, kin, kout, vin, vout, (size_t)n, 0, 8 * sizeof(KeyT), st));
  return CLV_OK;
}

// indices i in [0, n) with flag[i] != 0, in order; count -> *n_sel (host)
int select_flagged(const uint8_t* flags, int64_t n, int64_t* out, int64_t* n_sel, hipStream_t st) {
  rocprim::counting_iterator<int64_t> it(0);
  DevBuf cnt;
  int rc = alloc<int64_t>(cnt, 1);
  if (rc) return rc;
  size_t bytes = 0;
  CLV_HIP(rocprim::select((void*)nullptr, bytes, it, flags, out, cnt.as<int64_t>(), (size_t)n, st));
  DevBuf tmp;
  CLV_HIP(hipMalloc(&tmp.p, std::max<size_t>(bytes, 16)));
  CLV_HIP(rocprim::select(tmp.p, bytes, it, flags, out, cnt.as<int64_t>(), (size_t)n, st));
  CLV_HIP(hipMemcpyAsync(n_sel, cnt.p, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  CLV_HIP(hipStreamSynchronize(st));
  return CLV_OK;
}

inline dim3 grid1(int64_t n) { return dim3((unsigned)((n + 255) / 256)); }

// ---------------------------------------------------------------------------------------------
// Synthetic generator (bi:95-187): one lane per customer, Philox stream 4 keyed by the seed,
// counter (customer, 0, slot, 4).  Slots: 0-4 covariate uniforms, 8 heterogeneity normals,
// 9 lifetime uniform, 16+ inter-purchase gaps (two per block).
// ---------------------------------------------------------------------------------------------
constexpr uint32_t STREAM_GEN = 4u;
constexpr int GEN_MAX_STAR = 8;

struct GenArgs {
  int64_t n;
  int K;
  const double* covars;  // [n][K] incl. the intercept column, or null (generate U(-1,1))
  double beta[CLV_MAX_K * 2];
  double chol_gamma[4];  // lower Cholesky factor of gamma (2 x 2)
  const double* T_cal;   // [n] (per customer) — scalar callers broadcast
  double T_cal_fix;      // max(T_cal)
  int n_star;
  double T_star[GEN_MAX_STAR];
  double T_star_max;
  uint32_t k0, k1;
  int64_t* x;
  double* t_x;
  double* lambda_true;
  double* mu_true;
  double* tau_true;
  uint8_t* alive_true;
  int64_t* x_star;       // [n_star][n]
  double* covars_out;    // [n][K]
  int64_t* n_events;     // kept events per customer (elog rows)
  const int64_t* ev_offset;  // second pass: first elog row of each customer, or null
  int64_t* ev_cust;          //   elog cust column (1-based, bi:163)
  double* ev_t;              //   elog t column
};

__global__ __launch_bounds__(256) void generate_kernel(GenArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  const uint32_t ci = (uint32_t)i;
  auto blk = [&](uint32_t slot) { return philox4x32_10(u32x4{ci, 0u, slot, STREAM_GEN}, a.k0, a.k1); };
  double xr[CLV_MAX_K];
  xr[0] = 1.0;
  for (int k = 1; k < a.K; ++k) {
    if (a.covars) {
      xr[k] = a.covars[i * a.K + k];
    } else {  // rng.uniform(-1, 1, size=(n, K-1)) (bi:122-125)
      const u32x4 r = blk((uint32_t)((k - 1) >> 1));
      const double u = ((k - 1) & 1) ? u53(r.z, r.w) : u53(r.x, r.y);
      xr[k] = -1.0 + 2.0 * u;
    }
  }
  // theta = exp(X beta + MVN(0, gamma))  (bi:137-140)
  const u32x4 rn = blk(8u);
  const double rad = sqrt(-2.0 * log(u53_open0(rn.x, rn.y)));
  const double ang = 2.0 * u53(rn.z, rn.w);
  const double z0 = rad * cospi(ang), z1 = rad * sinpi(ang);
  const double e0 = a.chol_gamma[0] * z0;
  const double e1 = a.chol_gamma[2] * z0 + a.chol_gamma[3] * z1;
  double m0 = 0.0, m1 = 0.0;
  for (int k = 0; k < a.K; ++k) {
    m0 += xr[k] * a.beta[k * 2 + 0];
    m1 += xr[k] * a.beta[k * 2 + 1];
  }
  const double lam = exp(m0 + e0), mu = exp(m1 + e1);
  // tau ~ Exp(mu)  (bi:142)
  const u32x4 rt = blk(9u);
  const double tau = -log(u53_open0(rt.x, rt.y)) / mu;
  // purchase times: t = 0, then exponential gaps of mean 1/lambda until the running time reaches
  // min(T_cal_i + max T_star, tau) (bi:154-160); keep t <= tau, shift by the birth offset, keep
  // t <= T_cal_fix + max T_star (bi:161-162); CBS of bi:75-89 and hold-out counts (bi:170-179)
  const double Tc = a.T_cal[i];
  const double T_zero = a.T_cal_fix - Tc;
  const double min_T = fmin(Tc + a.T_star_max, tau);
  const double t_end = a.T_cal_fix + a.T_star_max;
  int64_t cnt_cal = 0, kept = 0;
  double tmax = -INFINITY;
  int64_t xs[GEN_MAX_STAR] = {0, 0, 0, 0, 0, 0, 0, 0};
  double t_acc = 0.0;
  uint32_t slot = 16u;
  int half = 0;
  u32x4 rg{0, 0, 0, 0};
  bool more = true;
  while (more) {
    // the event at t_acc
    if (t_acc <= tau) {
      const double ta = t_acc + T_zero;
      if (ta <= t_end) {
        if (a.ev_offset) {
          a.ev_cust[a.ev_offset[i] + kept] = i + 1;
          a.ev_t[a.ev_offset[i] + kept] = ta;
        }
        ++kept;
        if (ta <= a.T_cal_fix) {
          ++cnt_cal;
          tmax = fmax(tmax, ta);
        } else {
          for (int k = 0; k < a.n_star; ++k)
            if (ta <= a.T_cal_fix + a.T_star[k]) ++xs[k];
        }
      }
    }
    if (!(t_acc < min_T)) {
      more = false;
    } else {
      if (half == 0) rg = blk(slot++);
      const double u = half == 0 ? u53_open0(rg.x, rg.y) : u53_open0(rg.z, rg.w);
      half ^= 1;
      t_acc += -log(u) / lam;  // rng.exponential(scale=1/lam)
    }
  }
  a.x[i] = cnt_cal > 0 ? cnt_cal - 1 : 0;  // np.clip(count - 1, 0, None)
  a.t_x[i] = tmax;
  a.lambda_true[i] = lam;
  a.mu_true[i] = mu;
  a.tau_true[i] = tau;
  a.alive_true[i] = (T_zero + tau) > a.T_cal_fix ? 1 : 0;
  for (int k = 0; k < a.n_star; ++k) a.x_star[(int64_t)k * a.n + i] = xs[k];
  if (a.covars_out)
    for (int k = 0; k < a.K; ++k) a.covars_out[i * a.K + k] = xr[k];
  a.n_events[i] = kept;
}

}  // namespace

extern "C" {

int clv_elog2cbs(int32_t device, int64_t n_events, const int64_t* cust, const int64_t* date_ns, const double* sales,
                 int64_t unit_ns, int64_t T_cal_ns, int64_t T_tot_ns, int64_t* n_customers, int64_t* o_cust,
                 int64_t* o_x, double* o_t_x, double* o_litt, double* o_sales, double* o_sales_x, int64_t* o_first,
                 double* o_T_cal, double* o_T_star, int64_t* o_x_star, double* o_sales_star) {
  if (n_events < 0 || !cust || !date_ns || unit_ns <= 0 || !n_customers) return fail(CLV_EINVAL, "bad arguments");
  *n_customers = 0;
  if (n_events == 0) return CLV_OK;
  if (!o_cust || !o_x || !o_t_x || !o_litt || !o_sales || !o_sales_x || !o_first || !o_T_cal || !o_T_star ||
      !o_x_star || !o_sales_star)
    return fail(CLV_EINVAL, "null output buffer");
  DeviceScope ds(device);
  hipStream_t st = nullptr;
  const int64_t n = n_events;
  DevBuf dc, dd, dsl, idx0, k1, i1, k2, i2, cs, dts, sls, rflag, cflag, rstart, crflag, crun, cev;
  int rc;
  if ((rc = alloc<int64_t>(dc, n)) || (rc = alloc<int64_t>(dd, n)) || (rc = alloc<int64_t>(idx0, n)) ||
      (rc = alloc<int64_t>(k1, n)) || (rc = alloc<int64_t>(i1, n)) || (rc = alloc<int64_t>(k2, n)) ||
      (rc = alloc<int64_t>(i2, n)) || (rc = alloc<int64_t>(cs, n)) || (rc = alloc<int64_t>(dts, n)) ||
      (rc = alloc<double>(sls, n)) || (rc = alloc<uint8_t>(rflag, n)) || (rc = alloc<uint8_t>(cflag, n)) ||
      (rc = alloc<int64_t>(rstart, n)))
    return rc;
  CLV_HIP(hipMemcpy(dc.p, cust, sizeof(int64_t) * n, hipMemcpyHostToDevice));
  CLV_HIP(hipMemcpy(dd.p, date_ns, sizeof(int64_t) * n, hipMemcpyHostToDevice));
  if (sales) {
    if ((rc = alloc<double>(dsl, n))) return rc;
    CLV_HIP(hipMemcpy(dsl.p, sales, sizeof(double) * n, hipMemcpyHostToDevice));
  }
  {
    std::vector<int64_t> iota(n);
    for (int64_t i = 0; i < n; ++i) iota[i] = i;
    CLV_HIP(hipMemcpy(idx0.p, iota.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice));
  }
  // stable sorts: by date, then by customer -> (customer, date) order, ties in input order
  if ((rc = sort_pairs(dd.as<int64_t>(), k1.as<int64_t>(), idx0.as<int64_t>(), i1.as<int64_t>(), n, st))) return rc;
  hipLaunchKernelGGL(compact<int64_t>, grid1(n), dim3(256), 0, st, n, i1.as<int64_t>(), dc.as<int64_t>(),
                     k2.as<int64_t>());  // customers in date order
  CLV_HIP(hipGetLastError());
  if ((rc = sort_pairs(k2.as<int64_t>(), cs.as<int64_t>(), i1.as<int64_t>(), i2.as<int64_t>(), n, st))) return rc;
  hipLaunchKernelGGL(gather_events, grid1(n), dim3(256), 0, st, n, i2.as<int64_t>(), dc.as<int64_t>(),
                     dd.as<int64_t>(), dsl.as<double>(), cs.as<int64_t>(), dts.as<int64_t>(), sls.as<double>());
  hipLaunchKernelGGL(run_flags, grid1(n), dim3(256), 0, st, n, cs.as<int64_t>(), dts.as<int64_t>(),
                     rflag.as<uint8_t>(), cflag.as<uint8_t>());
  CLV_HIP(hipGetLastError());
  int64_t n_runs = 0, n_cust = 0;
  if ((rc = select_flagged(rflag.as<uint8_t>(), n, rstart.as<int64_t>(), &n_runs, st))) return rc;
  if ((rc = alloc<uint8_t>(crflag, n_runs)) || (rc = alloc<int64_t>(crun, n_runs)) || (rc = alloc<int64_t>(cev, n)))
    return rc;
  hipLaunchKernelGGL(cust_flag_of_runs, grid1(n_runs), dim3(256), 0, st, n_runs, rstart.as<int64_t>(),
                     cflag.as<uint8_t>(), crflag.as<uint8_t>());
  CLV_HIP(hipGetLastError());
  if ((rc = select_flagged(crflag.as<uint8_t>(), n_runs, crun.as<int64_t>(), &n_cust, st))) return rc;  // first run
  int64_t n_cust_ev = 0;
  if ((rc = select_flagged(cflag.as<uint8_t>(), n, cev.as<int64_t>(), &n_cust_ev, st))) return rc;      // first event
  if (n_cust_ev != n_cust) return fail(CLV_EINVAL, "internal: customer segmentation mismatch");
  DevBuf oc, ox, otx, olitt, os, osx, of, oT, oTs, oxs, oss, keep, sel;
  if ((rc = alloc<int64_t>(oc, n_cust)) || (rc = alloc<int64_t>(ox, n_cust)) || (rc = alloc<double>(otx, n_cust)) ||
      (rc = alloc<double>(olitt, n_cust)) || (rc = alloc<double>(os, n_cust)) || (rc = alloc<double>(osx, n_cust)) ||
      (rc = alloc<int64_t>(of, n_cust)) || (rc = alloc<double>(oT, n_cust)) || (rc = alloc<double>(oTs, n_cust)) ||
      (rc = alloc<int64_t>(oxs, n_cust)) || (rc = alloc<double>(oss, n_cust)) || (rc = alloc<uint8_t>(keep, n_cust)) ||
      (rc = alloc<int64_t>(sel, n_cust)))
    return rc;
  const int holdout = T_cal_ns < T_tot_ns ? 1 : 0;
  hipLaunchKernelGGL(customer_stats, grid1(n_cust), dim3(256), 0, st, n_cust, cev.as<int64_t>(),
                     rstart.as<int64_t>(), n_runs, n, cs.as<int64_t>(), dts.as<int64_t>(), sls.as<double>(),
                     crun.as<int64_t>(), (double)unit_ns, T_cal_ns, T_tot_ns, holdout, oc.as<int64_t>(),
                     ox.as<int64_t>(), otx.as<double>(), olitt.as<double>(), os.as<double>(), osx.as<double>(),
                     of.as<int64_t>(), oT.as<double>(), oTs.as<double>(), oxs.as<int64_t>(), oss.as<double>(),
                     keep.as<uint8_t>());
  CLV_HIP(hipGetLastError());
  int64_t n_keep = 0;
  if ((rc = select_flagged(keep.as<uint8_t>(), n_cust, sel.as<int64_t>(), &n_keep, st))) return rc;
  // compact into the first n_keep rows and copy out
  DevBuf tmp_i, tmp_d;
  if ((rc = alloc<int64_t>(tmp_i, n_keep)) || (rc = alloc<double>(tmp_d, n_keep))) return rc;
  auto out_i = [&](const DevBuf& src, int64_t* host) -> int {
    hipLaunchKernelGGL(compact<int64_t>, grid1(n_keep), dim3(256), 0, st, n_keep, sel.as<int64_t>(),
                       src.as<int64_t>(), tmp_i.as<int64_t>());
    CLV_HIP(hipGetLastError());
    CLV_HIP(hipMemcpy(host, tmp_i.p, sizeof(int64_t) * n_keep, hipMemcpyDeviceToHost));
    return CLV_OK;
  };
  auto out_d = [&](const DevBuf& src, double* host) -> int {
    hipLaunchKernelGGL(compact<double>, grid1(n_keep), dim3(256), 0, st, n_keep, sel.as<int64_t>(),
                       src.as<double>(), tmp_d.as<double>());
    CLV_HIP(hipGetLastError());
    CLV_HIP(hipMemcpy(host, tmp_d.p, sizeof(double) * n_keep, hipMemcpyDeviceToHost));
    return CLV_OK;
  };
  if ((rc = out_i(oc, o_cust)) || (rc = out_i(ox, o_x)) || (rc = out_d(otx, o_t_x)) || (rc = out_d(olitt, o_litt)) ||
      (rc = out_d(os, o_sales)) || (rc = out_d(osx, o_sales_x)) || (rc = out_i(of, o_first)) ||
      (rc = out_d(oT, o_T_cal)) || (rc = out_d(oTs, o_T_star)) || (rc = out_i(oxs, o_x_star)) ||
      (rc = out_d(oss, o_sales_star)))
    return rc;
  *n_customers = n_keep;
  return CLV_OK;
}

int clv_generate_pareto_abe(int32_t device, int64_t n, int32_t K, const double* beta, const double* gamma,
                            const double* covars, const double* T_cal, int32_t n_star, const double* T_star,
                            uint64_t seed, int64_t* x, double* t_x, double* lambda_true, double* mu_true,
                            double* tau_true, uint8_t* alive_true, int64_t* x_star, double* covars_out,
                            int64_t* n_events, const int64_t* elog_offsets, int64_t elog_rows, int64_t* elog_cust,
                            double* elog_t) {
  if (n < 1 || K < 1 || K > CLV_MAX_K || !beta || !gamma || !T_cal || n_star < 1 || n_star > GEN_MAX_STAR ||
      !T_star || !x || !t_x || !lambda_true || !mu_true || !tau_true || !alive_true || !x_star || !n_events)
    return fail(CLV_EINVAL, "bad arguments");
  if (n > 0xffffffffLL) return fail(CLV_EINVAL, "n exceeds the 32-bit Philox customer counter");
  GenArgs a{};
  a.n = n;
  a.K = K;
  for (int i = 0; i < 2 * K; ++i) a.beta[i] = beta[i];
  // a factor F with F F' = gamma (the reference draws MVN(0, gamma) via SVD, which also accepts
  // singular PSD gamma — its own smoke test uses one, bi:555): pivot-free Cholesky with the
  // residual clamped at 0, l00 = 0 handled
  const double g00 = gamma[0], g01 = gamma[1], g11 = gamma[3];
  const double scale = std::max(std::fabs(g00), std::fabs(g11));
  if (g00 < 0.0 || g11 < 0.0 || std::fabs(gamma[1] - gamma[2]) > 1e-12 * std::max(scale, 1.0))
    return fail(CLV_EINVAL, "gamma must be symmetric positive semi-definite");
  const double l00 = std::sqrt(g00);
  const double l10 = l00 > 0.0 ? g01 / l00 : 0.0;
  double d = g11 - l10 * l10;
  if (d < -1e-10 * std::max(scale, 1e-300) || (l00 == 0.0 && g01 != 0.0))
    return fail(CLV_EINVAL, "gamma must be symmetric positive semi-definite");
  d = std::max(d, 0.0);
  a.chol_gamma[0] = l00;
  a.chol_gamma[1] = 0.0;
  a.chol_gamma[2] = l10;
  a.chol_gamma[3] = std::sqrt(d);
  a.n_star = n_star;
  a.T_star_max = -INFINITY;
  for (int k = 0; k < n_star; ++k) {
    a.T_star[k] = T_star[k];
    a.T_star_max = std::max(a.T_star_max, T_star[k]);
  }
  a.T_cal_fix = -INFINITY;
  for (int64_t i = 0; i < n; ++i) a.T_cal_fix = std::max(a.T_cal_fix, T_cal[i]);
  a.k0 = (uint32_t)seed;
  a.k1 = (uint32_t)(seed >> 32);
  DeviceScope ds(device);
  DevBuf dcov, dT, dx, dtx, dl, dm, dtau, dal, dxs, dco, dne;
  int rc;
  if ((rc = alloc<double>(dT, n)) || (rc = alloc<int64_t>(dx, n)) || (rc = alloc<double>(dtx, n)) ||
      (rc = alloc<double>(dl, n)) || (rc = alloc<double>(dm, n)) || (rc = alloc<double>(dtau, n)) ||
      (rc = alloc<uint8_t>(dal, n)) || (rc = alloc<int64_t>(dxs, (size_t)n * n_star)) || (rc = alloc<int64_t>(dne, n)))
    return rc;
  if (covars) {
    if ((rc = alloc<double>(dcov, (size_t)n * K))) return rc;
    CLV_HIP(hipMemcpy(dcov.p, covars, sizeof(double) * n * K, hipMemcpyHostToDevice));
  }
  if (covars_out && (rc = alloc<double>(dco, (size_t)n * K))) return rc;
  CLV_HIP(hipMemcpy(dT.p, T_cal, sizeof(double) * n, hipMemcpyHostToDevice));
  a.covars = dcov.as<double>();
  a.T_cal = dT.as<double>();
  a.x = dx.as<int64_t>();
  a.t_x = dtx.as<double>();
  a.lambda_true = dl.as<double>();
  a.mu_true = dm.as<double>();
  a.tau_true = dtau.as<double>();
  a.alive_true = dal.as<uint8_t>();
  a.x_star = dxs.as<int64_t>();
  a.covars_out = dco.as<double>();
  a.n_events = dne.as<int64_t>();
  hipLaunchKernelGGL(generate_kernel, grid1(n), dim3(256), 0, nullptr, a);
  CLV_HIP(hipGetLastError());
  CLV_HIP(hipMemcpy(x, dx.p, sizeof(int64_t) * n, hipMemcpyDeviceToHost));
  CLV_HIP(hipMemcpy(t_x, dtx.p, sizeof(double) * n, hipMemcpyDeviceToHost));
  CLV_HIP(hipMemcpy(lambda_true, dl.p, sizeof(double) * n, hipMemcpyDeviceToHost));
  CLV_HIP(hipMemcpy(mu_true, dm.p, sizeof(double) * n, hipMemcpyDeviceToHost));
  CLV_HIP(hipMemcpy(tau_true, dtau.p, sizeof(double) * n, hipMemcpyDeviceToHost));
  CLV_HIP(hipMemcpy(alive_true, dal.p, n, hipMemcpyDeviceToHost));
  CLV_HIP(hipMemcpy(x_star, dxs.p, sizeof(int64_t) * n * n_star, hipMemcpyDeviceToHost));
  CLV_HIP(hipMemcpy(n_events, dne.p, sizeof(int64_t) * n, hipMemcpyDeviceToHost));
  if (covars_out) CLV_HIP(hipMemcpy(covars_out, dco.p, sizeof(double) * n * K, hipMemcpyDeviceToHost));
  if (elog_offsets) {  // second pass: the same counters replay the same events into the elog
    if (!elog_cust || !elog_t || elog_rows < 0) return fail(CLV_EINVAL, "elog buffers missing");
    DevBuf doff, dec, det;
    if ((rc = alloc<int64_t>(doff, n)) || (rc = alloc<int64_t>(dec, elog_rows)) || (rc = alloc<double>(det, elog_rows)))
      return rc;
    CLV_HIP(hipMemcpy(doff.p, elog_offsets, sizeof(int64_t) * n, hipMemcpyHostToDevice));
    a.ev_offset = doff.as<int64_t>();
    a.ev_cust = dec.as<int64_t>();
    a.ev_t = det.as<double>();
    hipLaunchKernelGGL(generate_kernel, grid1(n), dim3(256), 0, nullptr, a);
    CLV_HIP(hipGetLastError());
    CLV_HIP(hipMemcpy(elog_cust, dec.p, sizeof(int64_t) * elog_rows, hipMemcpyDeviceToHost));
    CLV_HIP(hipMemcpy(elog_t, det.p, sizeof(double) * elog_rows, hipMemcpyDeviceToHost));
  }
  return CLV_OK;
}

}  // extern "C"
