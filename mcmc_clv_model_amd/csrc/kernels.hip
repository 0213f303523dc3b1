// HIP kernels of the MI355X-native Abe (2009/2015) HB Pareto/NBD sampler (gfx950).
//
//   sweep_kernel  one lane per (chain, customer): draw_z, draw_tau, the n_mh_steps MH updates of
//                 (log lambda, log mu), draw_eta (D == 3), draw storage, and the customer's
//                 contribution to the level-2 sufficient statistics X'Y, Y'Y (+ log-lik term),
//                 reduced to one partial per workgroup of CLV_BLOCK customers.
//   group_kernel  sums blocks_per_unit consecutive block partials (large N: fewer exchanged units).
//   hyper_kernel  one workgroup per chain: fixed-order sum of all unit partials, then the
//                 conjugate multivariate-regression / inverse-Wishart draw (bi:233-262).
//
// Reference: src/models/bivariate/mcmc.py (bi), src/models/trivariate/mcmc.py (tri).
// All model arithmetic is float64 and follows the reference's operation order, so that with
// replayed variates (CLV_RNG_REPLAY) trajectories agree with the reference to rounding.
#include <hip/hip_ext.h>

#include "fastmath.h"
#include "kernels.h"
#include "philox.h"

#ifndef SWEEP_MH_PIPELINE
#define SWEEP_MH_PIPELINE 1  // 1: next MH chunk's variates drawn during the current chunk's steps
#endif
// register-pressure knobs of the persistent kernel (A/B builds override them):
#ifndef CLV_OPAQUE_GI
#define CLV_OPAQUE_GI(D) ((D) == 3)   // customer Philox products recomputed per sweep (not hoisted)
#endif
#ifndef CLV_L2_OPAQUE
#define CLV_L2_OPAQUE(P) (P)          // level-2 lane bookkeeping recomputed per sweep (not hoisted)
#endif
#ifndef CLV_L2_LANE0_MAX
#define CLV_L2_LANE0_MAX 6  // every level-2 draw (persistent kernel, fused tail, hyper kernel): one-lane algebra up to K*D (c3, K*D = 9: the element-parallel form 15.31 -> 15.11 us)
#endif
#ifndef PERSIST_REDUCE_GEN
#define PERSIST_REDUCE_GEN 1  // persistent kernel: statistics formed chunk-wise in the reduction
#endif
#ifndef SWEEP_REDUCE_CHUNK
#define SWEEP_REDUCE_CHUNK 8  // statistics formed and reduced per chunk in the customer workgroups
#endif
// sweep_kernel __launch_bounds__ minimum workgroups per CU: 4 (<= 128 VGPRs, 4 waves per SIMD)
// for the bivariate instances (but K = 6, whose 128-register cap spills): c4 104.4 -> 101.0 us
// per sweep (round 1), and 101.5 -> 100.3 against the compiler's choice now.  The trivariate
// ones keep the compiler's choice: with the covariates in LDS (CovLds, K >= 6) c5 needs 127 VGPRs
// and runs 4 waves per SIMD either way, but the cap's scheduling cost it 146.2 -> 160.5 us
// (measured).  SWEEP_MIN_BLOCKS overrides (A/B builds).
template <int D, int K>
struct SweepOcc;

// Launch-per-sweep instances whose covariate rows live in LDS (Cust CL) — K >= 6, where the
// covariates' registers decided the occupancy.  SWEEP_COV_LDS_MIN_K overrides (A/B builds).
#ifndef SWEEP_COV_LDS_MIN_K
#define SWEEP_COV_LDS_MIN_K 6
#endif
template <int D, int K>
struct CovLds {
  static constexpr bool value = K >= SWEEP_COV_LDS_MIN_K;
};

template <int D, int K>
struct SweepOcc {  // waves per SIMD the launched instance is compiled for (sweep_kernel_occ4 if 4)
#ifdef SWEEP_MIN_BLOCKS
  static constexpr int value = SWEEP_MIN_BLOCKS;  // 4: every instance occ4, else none
#else
  static constexpr int value = (D == 2 && K != 6) ? 4 : 1;
#endif
};

namespace clv {


__device__ __forceinline__ double clip70(double v) {  // np.clip(v, -70, 70) for non-NaN v (bi:323)
  return __builtin_fmin(__builtin_fmax(v, -70.0), 70.0);   // v_max_f64 + v_min_f64
}
__device__ __forceinline__ double min700(double v) {  // np.minimum(700, v) (bi:223)
  return v > 700.0 ? 700.0 : v;
}

// Per-customer constants of log_posterior (bi:291-310).
struct LPConst {
  double xm, omz, w, m0, m1, p00, p01, p11;
};

__device__ __forceinline__ double log_post(const LPConst& c, double ll, double lm) {
  const double dl = ll - c.m0;
  const double dm = lm - c.m1;
  const double lik = (c.xm * ll + c.omz * lm) - (exp(ll) + exp(lm)) * c.w;
  const double prior = -0.5 * ((dl * dl * c.p00 + 2.0 * dl * dm * c.p01) + dm * dm * c.p11);
  const double res = lik + prior;
  return lm > 5.0 ? -__builtin_inf() : res;  // cap (quirk Q3)
}

// Philox-mode log posterior up to a per-customer constant (only differences enter the MH test):
// the quadratic prior of bi:303-306 expanded in (ll, lm) with per-customer linear coefficients,
// the likelihood of bi:299-301, and ocml exp replaced by exp_fast (|ll|, |lm| <= 70 by the clip).
//   lp = ll (A ll + B lm + Dl) + lm (C lm + El) - w (e^ll + e^lm)
//   A = -p00/2, B = -p01, C = -p11/2, Dl = xm + p00 m0 + p01 m1, El = (1-z) + p01 m0 + p11 m1.
// The lm > 5 cap (quirk Q3) is applied by the caller.
struct LPFast {
  double A, B, C, Dl, El, w;
};
__device__ __forceinline__ double log_post_fast(const LPFast& c, double ll, double lm, const double* tab) {
  const double t1 = __builtin_fma(c.A, ll, __builtin_fma(c.B, lm, c.Dl));
  const double t2 = __builtin_fma(c.C, lm, c.El);
  const double q = __builtin_fma(ll, t1, lm * t2);
  double el, em;
  exp_fast2(ll, lm, tab, el, em);  // = exp_fast(ll), exp_fast(lm), both table reads in flight
  return __builtin_fma(-c.w, el + em, q);
}

// ---- wave-level reduce-scatter on CDNA4 cross-lane instructions ----
__device__ __forceinline__ uint64_t dbits(double x) { return __builtin_bit_cast(uint64_t, x); }
__device__ __forceinline__ double bitsd(uint64_t x) { return __builtin_bit_cast(double, x); }

// v_permlane32_swap: lanes 32-63 of a <-> lanes 0-31 of b (both dwords of each double).
__device__ __forceinline__ void swap_halves(double& a, double& b) {
  const uint64_t ua = dbits(a), ub = dbits(b);
  const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)ua, (uint32_t)ub, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(ua >> 32), (uint32_t)(ub >> 32), false, false);
  a = bitsd(((uint64_t)hi[0] << 32) | lo[0]);
  b = bitsd(((uint64_t)hi[1] << 32) | lo[1]);
}
// v_permlane16_swap: odd rows (16 lanes) of a <-> even rows of b.
__device__ __forceinline__ void swap_rows(double& a, double& b) {
  const uint64_t ua = dbits(a), ub = dbits(b);
  const auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)ua, (uint32_t)ub, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)(ua >> 32), (uint32_t)(ub >> 32), false, false);
  a = bitsd(((uint64_t)hi[0] << 32) | lo[0]);
  b = bitsd(((uint64_t)hi[1] << 32) | lo[1]);
}
// x + (x of the lane R places further round the 16-lane row), DPP row_ror:R (VALU, no LDS).
template <int R>
__device__ __forceinline__ double add_row_ror(double x) {
  const uint64_t u = dbits(x);
  // row_ror reads a valid lane everywhere: no "old" operand to initialise (v_mov_b32 0 per dword)
  const uint32_t lo = __builtin_amdgcn_mov_dpp((uint32_t)u, 0x120 + R, 0xf, 0xf, true);
  const uint32_t hi = __builtin_amdgcn_mov_dpp((uint32_t)(u >> 32), 0x120 + R, 0xf, 0xf, true);
  return x + bitsd(((uint64_t)hi << 32) | lo);
}

// Deterministic workgroup reduction of NS doubles.  Per wave: reduce-scatter across the halves
// (v_permlane32_swap: element j stays in lanes 0-31, element j+H1 in lanes 32-63), then across
// row pairs (v_permlane16_swap), then a 16-lane DPP rotate-allreduce of the remaining
// ceil(NS/4) values — ~3 VALU per element-step, instead of 6 ds_bpermute butterflies of all NS
// values.  Lane 0 of each row writes its row's values; waves are summed in fixed order.
// Result valid in `out` (LDS) for all threads after the call.
// Workgroup barrier ordering LDS accesses only: unlike __syncthreads it does not wait for the
// wave's outstanding global loads/stores (vmcnt), so write-through or remote stores issued before
// it stay in flight.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// LDS_ONLY: its barriers are lds_barrier() (callers with stores in flight that need no ordering).
template <int NS, int NT = BLOCK, bool LDS_ONLY = false>
__device__ __forceinline__ void block_reduce(double (&v)[NS], double (*red)[NS], double* out) {
  constexpr int H1 = (NS + 1) / 2;
  constexpr int H2 = (H1 + 1) / 2;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  constexpr int NW = NT / 64;
  double w1[H1];
#pragma unroll
  for (int j = 0; j < H1; ++j) {
    double a = v[j];
    double b = (j + H1 < NS) ? v[j + H1] : 0.0;
    swap_halves(a, b);
    w1[j] = a + b;  // lanes 0-31: element j;  lanes 32-63: element j + H1
  }
  double w2[H2];
#pragma unroll
  for (int j = 0; j < H2; ++j) {
    double a = w1[j];
    double b = (j + H2 < H1) ? w1[j + H2] : 0.0;
    swap_rows(a, b);
    w2[j] = a + b;  // even rows: w1 index j;  odd rows: w1 index j + H2
  }
#pragma unroll
  for (int j = 0; j < H2; ++j) {
    double x = w2[j];
    x = add_row_ror<8>(x);
    x = add_row_ror<4>(x);
    x = add_row_ror<2>(x);
    x = add_row_ror<1>(x);
    w2[j] = x;
  }
  if ((lane & 15) == 0) {
    const int row = lane >> 4;
#pragma unroll
    for (int j = 0; j < H2; ++j) {
      const int i1 = j + ((row & 1) ? H2 : 0);
      const int idx = i1 + ((row >> 1) ? H1 : 0);
      if (i1 < H1 && idx < NS) red[wave][idx] = w2[j];
    }
  }
  if constexpr (LDS_ONLY) lds_barrier(); else __syncthreads();
  if (threadIdx.x < NS) {
    double t = red[0][threadIdx.x];
#pragma unroll
    for (int w = 1; w < NW; ++w) t += red[w][threadIdx.x];
    out[threadIdx.x] = t;
  }
  if constexpr (LDS_ONLY) lds_barrier(); else __syncthreads();
}

// The same reduction with the NS values produced on demand, G at a time (gen(j) = element j), so
// at most G of them are live in registers: every element is summed over the lanes in exactly the
// order of block_reduce (lane l + lane l+32, then row pairs, then the DPP rotate), whatever its
// partner in the swaps — results are bitwise those of block_reduce on the materialised array.
template <int NS, int G, int NT = BLOCK, class Gen>
__device__ __forceinline__ void block_reduce_gen(const Gen& gen, double (*red)[NS], double* out) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  constexpr int NW = NT / 64;
#pragma unroll
  for (int base = 0; base < NS; base += G) {
    constexpr int GG = G;
    const int n = NS - base < GG ? NS - base : GG;  // compile-time after unrolling
    const int h1 = (n + 1) / 2;
    const int h2 = (h1 + 1) / 2;
    double w1[(G + 1) / 2];
#pragma unroll
    for (int j = 0; j < (G + 1) / 2; ++j) {
      if (j < h1) {
        double a = gen(base + j);
        double b = (j + h1 < n) ? gen(base + j + h1) : 0.0;
        swap_halves(a, b);
        w1[j] = a + b;
      }
    }
    double w2[(G + 3) / 4];
#pragma unroll
    for (int j = 0; j < (G + 3) / 4; ++j) {
      if (j < h2) {
        double a = w1[j];
        double b = (j + h2 < h1) ? w1[j + h2] : 0.0;
        swap_rows(a, b);
        double x = a + b;
        x = add_row_ror<8>(x);
        x = add_row_ror<4>(x);
        x = add_row_ror<2>(x);
        x = add_row_ror<1>(x);
        w2[j] = x;
      }
    }
    if ((lane & 15) == 0) {
      const int row = lane >> 4;
#pragma unroll
      for (int j = 0; j < (G + 3) / 4; ++j) {
        const int i1 = j + ((row & 1) ? h2 : 0);
        const int idx = i1 + ((row >> 1) ? h1 : 0);
        if (j < h2 && i1 < h1 && idx < n) red[wave][base + idx] = w2[j];
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < NS) {
    double t = red[0][threadIdx.x];
#pragma unroll
    for (int w = 1; w < NW; ++w) t += red[w][threadIdx.x];
    out[threadIdx.x] = t;
  }
  __syncthreads();
}

// One customer's level-2 sufficient statistics as a generator (element j of X'Y (K x D), the
// upper triangle of Y'Y, the likelihood term), each 0.0 + value as the accumulation from zero
// gave it, and 0.0 for an inactive lane.
template <int D, int K>
struct StatGen {
  double xr[K];  // by value (constant indices after unrolling: registers, no private-memory array)
  double Y[D];
  double lik;
  bool on;
  __device__ __forceinline__ double operator()(int j) const {
    double v;
    if (j < K * D) {
      v = xr[j / D] * Y[j % D];
    } else if (j < K * D + D * (D + 1) / 2) {
      v = 0.0;
      int t = K * D;
#pragma unroll
      for (int p = 0; p < D; ++p)
#pragma unroll
        for (int q = p; q < D; ++q, ++t)
          if (t == j) v = Y[p] * Y[q];
    } else {
      v = lik;
    }
    // no select on `on`: an inactive lane's StatGen is value-initialised (all inputs 0), so its
    // products are exact zeros already
    return v;
  }
};

// bi:402 (the reference's loop ends at burnin + mcmc, bi:383, so nothing beyond is stored)
#ifdef CLV_STAMPS
// Diagnostic build only: s_memrealtime (100 MHz) stamps per launch, slot = sweep % 1024:
// [0] first block start (min) [1] last block end of customer work (max) [2] tail start (max)
// [3] tail end (max) [4] first block end (min) [5] last block start (max)
__device__ __forceinline__ void stamp(unsigned long long* st, int64_t s, int k, bool is_min) {
  if (!st) return;
  const unsigned long long t = __builtin_amdgcn_s_memrealtime();
  unsigned long long* p = st + (s & 1023) * 8 + k;
  if (is_min) __hip_atomic_fetch_min(p, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else __hip_atomic_fetch_max(p, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
#define CLV_STAMP(st, s, k, is_min) stamp(st, s, k, is_min)
// per-workgroup record of the latest launch after the 1024 x 8 sweep stamps (wave 0, lane 0):
// [0] s_memrealtime start [1] s_memrealtime end of customer work [2] HW_ID [3] XCC_ID
// [4] s_memtime start [5] s_memtime MH start [6] s_memtime MH end [7] s_memtime end of customer work
// [8] s_memtime after the workgroup barrier [9] s_memtime after draw_z / draw_tau
__device__ __forceinline__ void wg_stamp(unsigned long long* st, int64_t wg, int k) {
  if (!st) return;
  unsigned long long v;
  if (k < 2) v = __builtin_amdgcn_s_memrealtime();
  else if (k == 2) v = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID
  else if (k == 3) v = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));  // HW_REG_XCC_ID
  else v = __builtin_amdgcn_s_memtime();
  st[1024 * 8 + wg * 12 + k] = v;
}
#define CLV_WG_STAMP(st, wg, k) wg_stamp(st, wg, k)
// persistent kernel: the same per-workgroup record, s_memrealtime only, for one chosen sweep
#define CLV_P_STAMP(st, wg, k, on) \
  do {                             \
    if ((on) && (st)) (st)[1024 * 8 + (wg) * 12 + (k)] = (k) == 8 ? __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)) : (k) == 9 ? __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11)) : __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define CLV_P_STAMP(st, wg, k, on) ((void)0)
#define CLV_WG_STAMP(st, wg, k) ((void)0)
#define CLV_STAMP(st, s, k, is_min) ((void)0)
#endif

__device__ __forceinline__ int64_t uniform_i64(int64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// s is wave-uniform at every call site and sweep counts are 32-bit (clv_config): the offset is
// made explicitly uniform so the modulo / division run on the scalar unit (the persistent kernel
// holds its loop counter in vector registers, where they were ~60 VALU of 64-bit division emulation
// per sweep and lane).
__device__ __forceinline__ int64_t uniform64(int64_t x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)x >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ uint32_t stored_offset(int64_t s, const Geometry& g) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(s - 1 - g.burnin));
}
__device__ __forceinline__ bool is_stored(int64_t s, const Geometry& g) {
  return s > g.burnin && s <= (int64_t)g.burnin + g.mcmc && stored_offset(s, g) % (uint32_t)g.thin == 0u;
}
__device__ __forceinline__ int64_t draw_index(int64_t s, const Geometry& g) {
  return (int64_t)(stored_offset(s, g) / (uint32_t)g.thin);  // (only called for stored sweeps: s > burnin)
}

// ---------------------------------------------------------------------------------------------
// Group kernel: unit partial = sequential sum of blocks_per_unit block partials.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void group_kernel(GroupArgs a) {
  const Geometry& g = a.g;
  const int u = blockIdx.x;
  const int c = blockIdx.y;
  const int j = threadIdx.x;
  if (j >= g.stride) return;
  const double* p = a.blockpart + ((int64_t)c * g.stride + j) * g.blocks_per_rank + (int64_t)u * g.blocks_per_unit;
  double t = 0.0;
  for (int bb = 0; bb < g.blocks_per_unit; ++bb) t += p[bb];
  a.unitpart[((int64_t)c * g.stride + j) * g.units_per_rank + u] = t;
}

// ---------------------------------------------------------------------------------------------
// Level-2 algebra (bi:243-261) on reduced statistics.
// ---------------------------------------------------------------------------------------------
// Philox mode: the level-2 draw's one-lane chain (Cholesky pivots, the inverse's determinant, the
// trivariate posterior variance) takes 1/sqrt and 1/x as the hardware estimate (v_rsq_f64 /
// v_rcp_f64, relative error ~2^-23) refined by two Newton steps (~1 ulp): 7 / 5 dependent VALU
// instead of the IEEE sqrt / division sequences with their range scaling.  The draw is the serial
// link of every sweep's hand-off (persistent kernel: publish -> customers -> partials -> draw).
// Their arguments there are positive normal numbers (S_n's pivots, Sigma's diagonal and
// determinant).  Replay mode keeps sqrt and '/' (the reference's operations).
#ifndef CLV_L2_NR
#define CLV_L2_NR 1
#endif
__device__ __forceinline__ double rsq_nr(double x) {
  double y = __builtin_amdgcn_rsq(x);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const double h = x * y;
    const double e = __builtin_fma(-h, y, 1.0);  // 1 - x y^2
    y = __builtin_fma(0.5 * y, e, y);
  }
  return y;
}
__device__ __forceinline__ double rcp_nr(double x) {
  double y = __builtin_amdgcn_rcp(x);
#pragma unroll
  for (int i = 0; i < 2; ++i) y = __builtin_fma(y, __builtin_fma(-x, y, 1.0), y);
  return y;
}

template <int D, bool NR = false>
__device__ void cholesky(const double (&A)[D][D], double (&L)[D][D]) {
#pragma unroll
  for (int r = 0; r < D; ++r)
#pragma unroll
    for (int q = 0; q < D; ++q) L[r][q] = 0.0;
#pragma unroll
  for (int j = 0; j < D; ++j) {
    double sdiag = A[j][j];
#pragma unroll
    for (int k = 0; k < j; ++k) sdiag -= L[j][k] * L[j][k];
    const double rj = NR ? rsq_nr(sdiag) : 0.0;  // NR: sqrt(d) = d / sqrt(d), x / L[j][j] = x rsq(d)
    L[j][j] = NR ? sdiag * rj : sqrt(sdiag);
#pragma unroll
    for (int r = j + 1; r < D; ++r) {
      double sv = A[r][j];
#pragma unroll
      for (int k = 0; k < j; ++k) sv -= L[r][k] * L[j][k];
      L[r][j] = NR ? sv * rj : sv / L[j][j];
    }
  }
}

// Hyper-state writes are write-through (sc1): a persistent sweep kernel reads them on other CUs in
// the same launch, after the chain's release flag.
__device__ __forceinline__ void hstore(double* H, int idx, double v) {
  __hip_atomic_store(H + idx, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// TO_LDS: plain stores into a workgroup-local block (the persistent kernel's tail publishes it
// with one coalesced store per lane)
template <bool TO_LDS>
__device__ __forceinline__ void hput(double* H, int idx, double v) {
  if constexpr (TO_LDS) H[idx] = v;
  else hstore(H, idx, v);
}

// hyper-state finalisation from (beta, Sigma): inverse block, proposal scales, eta constants.
// NR (Philox mode): the divisions as products with rcp_nr, sqrt(post_var) as rsq_nr of its
// reciprocal (the level-2 chain's tail; see rsq_nr).
template <int D, int K, bool TO_LDS = false, bool NR = false>
__device__ void finalize_hyper(const double* beta_flat, const double (&Sig)[D][D], double omega2, double* H) {
#pragma unroll
  for (int q = 0; q < K * D; ++q) hput<TO_LDS>(H, H_BETA + q, beta_flat[q]);
  for (int q = 0; q < 9; ++q) hput<TO_LDS>(H, H_SIGMA + q, 0.0);
#pragma unroll
  for (int p = 0; p < D; ++p)
#pragma unroll
    for (int q = 0; q < D; ++q) hput<TO_LDS>(H, H_SIGMA + p * 3 + q, Sig[p][q]);
  if constexpr (D == 2) {
    const double det = Sig[0][0] * Sig[1][1] - Sig[0][1] * Sig[1][0];
    if constexpr (NR) {
      const double id = rcp_nr(det);
      hput<TO_LDS>(H, H_P00, Sig[1][1] * id);
      hput<TO_LDS>(H, H_P01, -Sig[0][1] * id);
      hput<TO_LDS>(H, H_P11, Sig[0][0] * id);
    } else {
      hput<TO_LDS>(H, H_P00, Sig[1][1] / det);
      hput<TO_LDS>(H, H_P01, -Sig[0][1] / det);
      hput<TO_LDS>(H, H_P11, Sig[0][0] / det);
    }
  } else {
    // top-left 2x2 block of the full 3x3 inverse (tri:402 with tri:422-424; quirk Q4)
    const double c00 = Sig[1][1] * Sig[2][2] - Sig[1][2] * Sig[2][1];
    const double c01 = Sig[1][0] * Sig[2][2] - Sig[1][2] * Sig[2][0];
    const double c02 = Sig[1][0] * Sig[2][1] - Sig[1][1] * Sig[2][0];
    const double det = Sig[0][0] * c00 - Sig[0][1] * c01 + Sig[0][2] * c02;
    const double n01 = -(Sig[0][1] * Sig[2][2] - Sig[0][2] * Sig[2][1]);
    const double n11 = Sig[0][0] * Sig[2][2] - Sig[0][2] * Sig[2][0];
    hput<TO_LDS>(H, H_S22, Sig[2][2]);
    hput<TO_LDS>(H, H_OMEGA2, omega2);
    if constexpr (NR) {
      const double id = rcp_nr(det);
      hput<TO_LDS>(H, H_P00, c00 * id);
      hput<TO_LDS>(H, H_P01, n01 * id);
      hput<TO_LDS>(H, H_P11, n11 * id);
      const double inv_om = 1.0 / omega2;  // (the run's constant: off the chain)
      const double inv_s22 = rcp_nr(Sig[2][2]);
      const double prec = inv_om + inv_s22;  // tri:325-326: post_var = 1 / prec
      hput<TO_LDS>(H, H_POSTVAR, rcp_nr(prec));
      hput<TO_LDS>(H, H_SQRT_POSTVAR, rsq_nr(prec));
      hput<TO_LDS>(H, H_INV_OMEGA2, inv_om);
      hput<TO_LDS>(H, H_INV_S22, inv_s22);
    } else {
      hput<TO_LDS>(H, H_P00, c00 / det);
      hput<TO_LDS>(H, H_P01, n01 / det);
      hput<TO_LDS>(H, H_P11, n11 / det);
      const double post_var = 1.0 / (1.0 / omega2 + 1.0 / Sig[2][2]);  // tri:325-326
      hput<TO_LDS>(H, H_POSTVAR, post_var);
      hput<TO_LDS>(H, H_SQRT_POSTVAR, sqrt(post_var));
      hput<TO_LDS>(H, H_INV_OMEGA2, 1.0 / omega2);
      hput<TO_LDS>(H, H_INV_S22, 1.0 / Sig[2][2]);
    }
  }
  hput<TO_LDS>(H, H_S00, Sig[0][0]);
  hput<TO_LDS>(H, H_S11, Sig[1][1]);
}

// LDS scratch of the level-2 draw.
struct L2Scratch {
  double prior[81 + 81 + 27 + 9];  // V, chol(V), A0 B0, S0 + B0'A0B0 (staged at the tail's start)
  double R[CLV_MAX_K * 3];   // X'Y + A0 B0            [k*D + d]
  double Bh[CLV_MAX_K * 3];  // B_hat = V R            [k*D + d]
  double Sn[6];              // S_n upper triangle     (p, q >= p) order
  double Sig[9];             // Sigma                  [p*D + q]
  double Ls[9];              // chol(Sigma)            [p*D + q]
  double beta[CLV_MAX_K * 3];// beta = B_hat + w       [k*D + d] (= beta.ravel() row-major)
  double Ai[9];              // Philox mode: inverse Bartlett factor (persistent kernel: formed early)
};

// Orders LDS accesses between the lanes of one wavefront (LDS operations of a wave complete in
// order; the fences keep the compiler from moving accesses across).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Stage the prior block (V, chol V, A0 B0, S0B: 198 doubles) into the scratch; a later barrier
// publishes it.
__device__ __forceinline__ void stage_prior(const double* prior, L2Scratch* sc) {
  for (int t = threadIdx.x; t < 198; t += blockDim.x) sc->prior[t] = prior[t];
}

// Given the reduced statistics `tot` (LDS), the variates (LDS) and the staged prior, draw
// (beta, Sigma) with wavefront 0 (lanes >= 64 return at once; no workgroup barriers).  Element-parallel phases
// (one lane per element of B_hat, S_n, w) around a one-lane D x D core; each element's sum runs in
// the sequential order of bi:243-261, so the result does not depend on the lane mapping.
// iwn: n_tril normals, chi2: D chi-square draws, noise: either the replayed mvn noise (w, D*K)
// or standard normals z (D*K) mapped through kron(chol(Sigma), chol(V)).
template <int D, int K>
__device__ void level2_draw_exact(const double* tot, const double* iwn, const double* chi2, const double* noise,
                            bool noise_is_w, L2Scratch* sc) {
  constexpr int NXY = K * D;
  const int t = threadIdx.x;
  if (t >= 64) return;
  const double* V = sc->prior;
  const double* cholV = sc->prior + 81;
  const double* A0B0 = sc->prior + 162;
  const double* S0B = sc->prior + 189;
  if (t < NXY) sc->R[t] = tot[t] + A0B0[t];
  wave_sync();
  if (t < NXY) {  // B_hat[k][d] = sum_j V[k][j] R[j][d]
    const int k = t / D, d = t % D;
    double sv = 0.0;
#pragma unroll
    for (int j = 0; j < K; ++j) sv += V[k * K + j] * sc->R[j * D + d];
    sc->Bh[t] = sv;
  }
  wave_sync();
  if (t < D * (D + 1) / 2) {  // S_n = S0 + Y'Y + B0'A0B0 - R'B_hat   (== S0 + E'E + C'A0C, bi:253-255)
    int p = 0, q = t;
    while (q >= D - p) {
      q -= D - p;
      ++p;
    }
    q += p;
    double rb = 0.0;
#pragma unroll
    for (int k = 0; k < K; ++k) rb += sc->R[k * D + p] * sc->Bh[k * D + q];
    sc->Sn[t] = (S0B[p * D + q] + tot[NXY + t]) - rb;
  }
  wave_sync();
  if (t == 0) {
    double Sn[D][D];
    int n = 0;
#pragma unroll
    for (int p = 0; p < D; ++p)
#pragma unroll
      for (int q = p; q < D; ++q) {
        Sn[p][q] = sc->Sn[n];
        Sn[q][p] = sc->Sn[n++];
      }
    // Sigma ~ IW(nu_n, S_n): scipy invwishart Bartlett form, Sigma = (L A^-1)(L A^-1)'
    double L[D][D], A[D][D], M[D][D], Sig[D][D];
    cholesky<D>(Sn, L);
#pragma unroll
    for (int p = 0; p < D; ++p)
#pragma unroll
      for (int q = 0; q < D; ++q) A[p][q] = 0.0;
    {
      int m = 0;
#pragma unroll
      for (int p = 1; p < D; ++p)
#pragma unroll
        for (int q = 0; q < p; ++q) A[p][q] = iwn[m++];  // np.tril_indices(D, -1) order
#pragma unroll
      for (int p = 0; p < D; ++p) A[p][p] = sqrt(chi2[p]);
    }
#pragma unroll
    for (int r = 0; r < D; ++r)
#pragma unroll
      for (int j = D - 1; j >= 0; --j) {
        double sv = L[r][j];
#pragma unroll
        for (int k = j + 1; k < D; ++k) sv -= M[r][k] * A[k][j];
        M[r][j] = sv / A[j][j];
      }
#pragma unroll
    for (int p = 0; p < D; ++p)
#pragma unroll
      for (int q = 0; q < D; ++q) {
        double sv = 0.0;
#pragma unroll
        for (int k = 0; k < D; ++k) sv += M[p][k] * M[q][k];
        Sig[p][q] = sv;
      }
#pragma unroll
    for (int p = 0; p < D; ++p)
#pragma unroll
      for (int q = p + 1; q < D; ++q) Sig[q][p] = Sig[p][q];
    double Ls[D][D];
    if (!noise_is_w) cholesky<D>(Sig, Ls);
#pragma unroll
    for (int p = 0; p < D; ++p)
#pragma unroll
      for (int q = 0; q < D; ++q) {
        sc->Sig[p * D + q] = Sig[p][q];
        sc->Ls[p * D + q] = noise_is_w ? 0.0 : Ls[p][q];
      }
  }
  wave_sync();
  // beta | Sigma: MVN(B_hat.ravel(), kron(Sigma, V)) with the reference's row-major ravel (quirk
  // Q1): flat element q = p*K + bq of the noise pairs with beta.ravel()[q] = beta[q / D][q % D]
  if (t < NXY) {
    double w;
    if (noise_is_w) {
      w = noise[t];
    } else {
      const int p = t / K, bq = t % K;
      double sv = 0.0;
      for (int cc = 0; cc <= p; ++cc)
        for (int e = 0; e <= bq; ++e) sv += sc->Ls[p * D + cc] * cholV[bq * K + e] * noise[cc * K + e];
      w = sv;
    }
    sc->beta[t] = sc->Bh[t] + w;
  }
  wave_sync();
}

// Inverse of the Bartlett factor A (lower triangular: A[p][p] = sqrt(chi2[p]), strict lower part
// the iw normals in np.tril_indices(D, -1) order).  Depends on the variates only, so the
// persistent kernel's level-2 workgroup forms it while the sweep runs.
template <int D>
__device__ __forceinline__ void bartlett_inverse(const double* iwn, const double* chi2, double* Ai /* [D*D] */) {
  double A[D][D], I[D][D];
  {
    int m = 0;
#pragma unroll
    for (int p = 0; p < D; ++p)
#pragma unroll
      for (int q = 0; q < D; ++q) A[p][q] = 0.0;
#pragma unroll
    for (int p = 1; p < D; ++p)
#pragma unroll
      for (int q = 0; q < p; ++q) A[p][q] = iwn[m++];
#pragma unroll
    for (int p = 0; p < D; ++p) A[p][p] = sqrt(chi2[p]);
  }
#pragma unroll
  for (int j = 0; j < D; ++j) {
#pragma unroll
    for (int q = 0; q < D; ++q) I[j][q] = 0.0;
    I[j][j] = 1.0 / A[j][j];
  }
#pragma unroll
  for (int i = 1; i < D; ++i)
#pragma unroll
    for (int j = 0; j < i; ++j) {
      double sv = 0.0;
#pragma unroll
      for (int k = j; k < i; ++k) sv += A[i][k] * I[k][j];
      I[i][j] = -(sv * I[i][i]);
    }
#pragma unroll
  for (int p = 0; p < D; ++p)
#pragma unroll
    for (int q = 0; q < D; ++q) Ai[p * D + q] = I[p][q];
}

// Philox-mode core (one lane): Sigma = (L A^-1)(L A^-1)' with L = chol(S_n) — the Bartlett form of
// level2_draw_exact with A^-1 applied by multiplication instead of a triangular solve.  M = L A^-1
// is lower triangular with a positive diagonal, so it IS chol(Sigma): no second factorisation.
template <int D, bool NR = CLV_L2_NR != 0>
__device__ __forceinline__ void iw_core_fast(const double (&Sn)[D][D], const double* Ai, double (&Sig)[D][D],
                                             double (&M)[D][D]) {
  double L[D][D];
  cholesky<D, NR>(Sn, L);
#pragma unroll
  for (int r = 0; r < D; ++r)
#pragma unroll
    for (int j = 0; j < D; ++j) {
      double sv = 0.0;
#pragma unroll
      for (int k = j; k <= r; ++k) sv += L[r][k] * Ai[k * D + j];
      M[r][j] = j <= r ? sv : 0.0;
    }
#pragma unroll
  for (int p = 0; p < D; ++p)
#pragma unroll
    for (int q = 0; q <= p; ++q) {
      double sv = 0.0;
#pragma unroll
      for (int k = 0; k <= q; ++k) sv += M[p][k] * M[q][k];
      Sig[p][q] = sv;
      Sig[q][p] = sv;
    }
}

// Philox-mode level-2 draw.  Small K*D (the persistent kernel's sizes): lane 0 alone, all in
// registers — no LDS round trips between phases, which dominate at these sizes; larger K: the
// element-parallel phases of level2_draw_exact around the fast core.  `Ai`: the Bartlett inverse
// if already formed (LDS), else null.  Every path (fused, sharded, persistent) calls this same
// function in Philox mode, so they stay bitwise identical.
template <int D, int K, int LANE0_MAX = 12, bool NR = CLV_L2_NR != 0>
__device__ void level2_draw_fast(const double* tot, const double* iwn, const double* chi2, const double* noise,
                                 const double* Ai_pre, L2Scratch* sc) {
  constexpr int NXY = K * D;
  const int t = threadIdx.x;
  if (t >= 64) return;
  const double* V = sc->prior;
  const double* cholV = sc->prior + 81;
  const double* A0B0 = sc->prior + 162;
  const double* S0B = sc->prior + 189;
  if constexpr (NXY <= LANE0_MAX) {  // (both forms form the same sums in the same order)
    if (t == 0) {
      double Ai[D * D];
      if (Ai_pre) {
#pragma unroll
        for (int q = 0; q < D * D; ++q) Ai[q] = Ai_pre[q];
      } else {
        bartlett_inverse<D>(iwn, chi2, Ai);
      }
      // One lane issues in order, so every sum below runs its terms in the reference order per
      // element but with the independent elements' chains interleaved (term-major loops): the
      // dependent fp64 latency is paid once per term, not once per term and element.
      double R[NXY], Bh[NXY];
#pragma unroll
      for (int q = 0; q < NXY; ++q) R[q] = tot[q] + A0B0[q];
#pragma unroll
      for (int q = 0; q < NXY; ++q) Bh[q] = 0.0;
#pragma unroll
      for (int j = 0; j < K; ++j)  // B_hat[k][d] = sum_j V[k][j] R[j][d]
#pragma unroll
        for (int q = 0; q < NXY; ++q) Bh[q] += V[(q / D) * K + j] * R[j * D + q % D];
      double Sn[D][D], rb[D][D];
#pragma unroll
      for (int p = 0; p < D; ++p)
#pragma unroll
        for (int q = p; q < D; ++q) rb[p][q] = 0.0;
#pragma unroll
      for (int k = 0; k < K; ++k)
#pragma unroll
        for (int p = 0; p < D; ++p)
#pragma unroll
          for (int q = p; q < D; ++q) rb[p][q] += R[k * D + p] * Bh[k * D + q];
      int n = NXY;
#pragma unroll
      for (int p = 0; p < D; ++p)
#pragma unroll
        for (int q = p; q < D; ++q) {
          Sn[p][q] = (S0B[p * D + q] + tot[n++]) - rb[p][q];
          Sn[q][p] = Sn[p][q];
        }
      double Sig[D][D], M[D][D];
      iw_core_fast<D, NR>(Sn, Ai, Sig, M);
      asm volatile("" ::: "memory");  // chol(V) and the noise are read here, not hoisted above (registers)
      double sv[NXY];
#pragma unroll
      for (int q = 0; q < NXY; ++q) sv[q] = 0.0;
#pragma unroll
      for (int cc = 0; cc < D; ++cc)  // beta = B_hat + kron(chol Sigma, chol V) z, row-major ravel (Q1);
#pragma unroll                      // per element the terms (cc <= p, e <= bq) in cc-major order
        for (int e = 0; e < K; ++e)
#pragma unroll
          for (int q = 0; q < NXY; ++q)
            if (cc <= q / K && e <= q % K) sv[q] += M[q / K][cc] * cholV[(q % K) * K + e] * noise[cc * K + e];
#pragma unroll
      for (int q = 0; q < NXY; ++q) sc->beta[q] = Bh[q] + sv[q];
#pragma unroll
      for (int p = 0; p < D; ++p)
#pragma unroll
        for (int q = 0; q < D; ++q) sc->Sig[p * D + q] = Sig[p][q];
    }
    wave_sync();
  } else {
    if (t < NXY) sc->R[t] = tot[t] + A0B0[t];
    wave_sync();
    if (t < NXY) {
      const int k = t / D, d = t % D;
      double sv = 0.0;
#pragma unroll
      for (int j = 0; j < K; ++j) sv += V[k * K + j] * sc->R[j * D + d];
      sc->Bh[t] = sv;
    }
    wave_sync();
    if (t < D * (D + 1) / 2) {
      int p = 0, q = t;
      while (q >= D - p) {
        q -= D - p;
        ++p;
      }
      q += p;
      double rb = 0.0;
#pragma unroll
      for (int k = 0; k < K; ++k) rb += sc->R[k * D + p] * sc->Bh[k * D + q];
      sc->Sn[t] = (S0B[p * D + q] + tot[NXY + t]) - rb;
    }
    wave_sync();
    if (t == 0) {
      double Ai[D * D];
      if (Ai_pre) {
#pragma unroll
        for (int q = 0; q < D * D; ++q) Ai[q] = Ai_pre[q];
      } else {
        bartlett_inverse<D>(iwn, chi2, Ai);
      }
      double Sn[D][D];
      int n = 0;
#pragma unroll
      for (int p = 0; p < D; ++p)
#pragma unroll
        for (int q = p; q < D; ++q) {
          Sn[p][q] = sc->Sn[n];
          Sn[q][p] = sc->Sn[n++];
        }
      double Sig[D][D], M[D][D];
      iw_core_fast<D, NR>(Sn, Ai, Sig, M);
#pragma unroll
      for (int p = 0; p < D; ++p)
#pragma unroll
        for (int q = 0; q < D; ++q) {
          sc->Sig[p * D + q] = Sig[p][q];
          sc->Ls[p * D + q] = M[p][q];
        }
    }
    wave_sync();
    if (t < NXY) {
      const int p = t / K, bq = t % K;
      double sv = 0.0;
#pragma unroll
      for (int cc = 0; cc < D; ++cc)  // fully unrolled: the LDS reads go out together; the terms
#pragma unroll                      // (cc <= p, e <= bq) are added in the same order as before
        for (int e = 0; e < K; ++e) {
          const double term = sc->Ls[p * D + cc] * cholV[bq * K + e] * noise[cc * K + e];
          sv = (cc <= p && e <= bq) ? sv + term : sv;
        }
      sc->beta[t] = sc->Bh[t] + sv;
    }
    wave_sync();
  }
}

// Level-2 draw: replay mode follows the reference's operation order (level2_draw_exact, bitwise
// trajectories); Philox mode takes the latency-optimised form.
template <int D, int K, int LANE0_MAX = 12>
__device__ __forceinline__ void level2_draw(const double* tot, const double* iwn, const double* chi2,
                                            const double* noise, bool noise_is_w, L2Scratch* sc,
                                            const double* Ai_pre = nullptr) {
  if (noise_is_w) level2_draw_exact<D, K>(tot, iwn, chi2, noise, true, sc);
  else level2_draw_fast<D, K, LANE0_MAX>(tot, iwn, chi2, noise, Ai_pre, sc);
}

// Philox-mode hyper variates (fp64).
__device__ double hyper_normal(uint32_t k0, uint32_t k1, uint32_t slot, uint32_t sweep) {
  const u32x4 r = hyper_block(k0, k1, slot, sweep);
  return sqrt(-2.0 * log(u53_open0(r.x, r.y))) * cospi(2.0 * u53(r.z, r.w));
}

// Marsaglia–Tsang Gamma(alpha, 1), alpha >= 1; chi2(df) = 2 Gamma(df / 2).
__device__ double chi2_draw(uint32_t k0, uint32_t k1, uint32_t sweep, int idx, double df) {
  const double alpha = 0.5 * df;
  const double dd = alpha - 1.0 / 3.0;
  const double cc = 1.0 / sqrt(9.0 * dd);
  for (int at = 0; at < GAMMA_MAX_ATTEMPTS; ++at) {
    const uint32_t slot = HSLOT_GAMMA0 + (uint32_t)idx * HSLOT_GAMMA_STRIDE + 2u * at;
    const double x = hyper_normal(k0, k1, slot, sweep);
    const double t = cc * x;
    if (t <= -1.0) continue;
    const double v1 = t * (3.0 + t * (3.0 + t));  // (1 + t)^3 - 1
    const u32x4 r2 = hyper_block(k0, k1, slot + 1u, sweep);
    const double lu = log(u53_open0(r2.x, r2.y));
    if (lu < 0.5 * x * x + dd * (3.0 * log1p(t) - v1)) return 2.0 * dd * (1.0 + v1);
  }
  return df;  // unreachable in practice (acceptance > 0.95 per attempt)
}

// Level-2 draw of chain c after sweep s (mode 0), or the bivariate initial draw (mode 1):
// fixed-order sum of all unit partials, variates, algebra, hyper state, level-2 record and
// log-likelihood, then the sweep-counter arrival.  Executed by one 256-thread workgroup: the
// standalone hyper_kernel (sharded path) or the last-arriving sweep workgroup of the chain
// (fused path).  `units`: [world][chain][stride][units_per_rank] unit partials (the gathered
// buffer; at world size 1 this rank's unit partials, or its block partials when a unit is one
// block), summed in global unit order — so every path and GPU count is bitwise identical.
// Level-2 draw, part 1: stage the prior and this draw's variates (independent of the statistics,
// so their loads overlap the reduction's).
template <int D, int K, bool REPLAY>
__device__ __forceinline__ void hyper_variates(const HyperArgs& a, int c, int64_t s, double* var_iw, double* var_chi,
                                               double* var_noise, L2Scratch* l2) {
  constexpr int NTRIL = D * (D - 1) / 2;
  const int tid = threadIdx.x;
  const int64_t hs = (D == 2) ? s + 1 : s;  // sweep the drawn (beta, Sigma) belongs to
  stage_prior(a.V, l2);  // published by block_reduce's barriers
  if constexpr (REPLAY) {
    const double* tv = a.r.tape + ((int64_t)c * a.r.tape_sweeps + (hs - 1)) * a.r.tape_sweep_stride +
                       (a.r.tape_sweep_stride - TAPE_HYPER);
    if (tid < 3) var_iw[tid] = tv[tid];
    if (tid < 3) var_chi[tid] = tv[3 + tid];
    if (tid < D * K) var_noise[tid] = tv[6 + tid];
  } else if (a.hvar) {  // precomputed by this sweep's kernel (sc1 stores: read with sc1 loads)
    const double* hv = a.hvar + (int64_t)c * HV;
    if (tid < 3) var_iw[tid] = __hip_atomic_load(hv + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid < 3) var_chi[tid] = __hip_atomic_load(hv + 3 + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid < D * K) var_noise[tid] = __hip_atomic_load(hv + 8 + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    uint32_t k0, k1;
    chain_key(a.r.seed, (int64_t)a.r.chain_first + c, &k0, &k1);
    if (tid < NTRIL) var_iw[tid] = hyper_normal(k0, k1, HSLOT_NORMAL0 + tid, (uint32_t)hs);
    if (tid >= 32 && tid < 32 + D * K)
      var_noise[tid - 32] = hyper_normal(k0, k1, HSLOT_BETA_NORMAL0 + (tid - 32), (uint32_t)hs);
    if (tid >= 64 && tid < 64 + D) {  // second wavefront: the gamma rejection loops
      const int q = tid - 64;
      var_chi[q] = chi2_draw(k0, k1, (uint32_t)hs, q, a.nu_n - D + 1 + q);
    }
  }
}

// Part 2: this lane's share of the fixed-order sum over all units of all shards (independent of
// world size): lane u sums units u, u + NT, ... in order.  Unit partials are read with sc1 loads:
// in the fused path other CUs wrote them during this launch.
template <int NS, int NT>
__device__ __forceinline__ void hyper_sum_units(const HyperArgs& a, int c, const double* units, double (&acc)[NS]) {
  const Geometry& g = a.g;
  // (every default plan: <= 512 units) both units' loads issued together, then added in the loop's
  // order: one memory round trip instead of one per unit.  Small NS only: the 2 NS values in
  // flight must not raise the sweep kernel's registers (trivariate K = 9: NS = 34, 125 -> 161 VGPRs)
  if (NS <= 16 && g.n_units_global <= 2 * NT) {
    const int u0 = threadIdx.x, u1 = threadIdx.x + NT, upr = g.units_per_rank;
    const bool h0 = u0 < g.n_units_global, h1 = u1 < g.n_units_global;
    const int64_t cs = (int64_t)g.stride * upr;
    const double* p0 = units + ((int64_t)(u0 / upr) * g.n_chains + c) * cs + (u0 % upr);
    const double* p1 = units + ((int64_t)(u1 / upr) * g.n_chains + c) * cs + (u1 % upr);
    const double* q0 = h0 ? p0 : units;  // lanes without a unit read unit 0 and discard it
    const double* q1 = h1 ? p1 : units;
    double v0[NS], v1[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      v0[j] = __hip_atomic_load(q0 + (int64_t)j * upr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      v1[j] = __hip_atomic_load(q1 + (int64_t)j * upr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      acc[j] = 0.0;
      if (h0) acc[j] += v0[j];
      if (h1) acc[j] += v1[j];
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < NS; ++j) acc[j] = 0.0;
  for (int64_t u = threadIdx.x; u < g.n_units_global; u += NT) {
    const int64_t r = u / g.units_per_rank;
    const int64_t lu = u - r * g.units_per_rank;
    const double* p = units + (r * g.n_chains + c) * g.stride * (int64_t)g.units_per_rank + lu;
#pragma unroll
    for (int j = 0; j < NS; ++j)  // lanes read consecutive units: coalesced
      acc[j] += __hip_atomic_load(p + (int64_t)j * g.units_per_rank, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Part 3: the workgroup reduction of the lanes' sums, the algebra and the outputs.
struct NoWork {
  __device__ void operator()() const {}
};

// after_reduce: work for the other wavefronts once the sums are formed (the fused exchange empties
// its mail slots there), run while wavefront 0 draws; no barrier follows it here.
template <int D, int K, bool REPLAY, int NS, int NT, class After = NoWork>
__device__ void hyper_finish(const HyperArgs& a, int c, int64_t s, int mode, double (&acc)[NS], double (*red)[NS],
                             double* tot, double* var_iw, double* var_chi, double* var_noise, L2Scratch* l2,
                             After after_reduce = After{}) {
  const Geometry& g = a.g;
  const int tid = threadIdx.x;
  const int64_t hs = (D == 2) ? s + 1 : s;
  block_reduce<NS, NT>(acc, red, tot);  // its barriers also publish the variates written to LDS above
  after_reduce();

  // algebra (element-parallel phases + one-lane core) and outputs
  if (tid == 0) CLV_STAMP(a.stamps, s, 6, false);
  L2Scratch* sc = l2;
  // (one-lane algebra up to K*D = 6 as in the persistent kernel: the element-parallel form at c4,
  // K*D = 10, measured 84.4 -> 83.7 us per sweep against the one-lane one; the same bits)
  level2_draw<D, K, CLV_L2_LANE0_MAX>(tot, var_iw, var_chi, var_noise, REPLAY, sc);
#ifdef CLV_STAMP_L2SPLIT  // diagnostic: slot 5 = the level-2 draw's end (before finalize_hyper)
  if (tid == 0) CLV_STAMP(a.stamps, s, 5, false);
#endif
  const bool store_l2 = hs >= 1 && is_stored(hs, g);
  double* o = store_l2 ? a.level2 + ((int64_t)c * g.n_draws + draw_index(hs, g)) * g.l2w : nullptr;
  if (tid < K * D && store_l2) o[(tid % D) * K + tid / D] = sc->beta[tid];  // beta.T.ravel() (bi:411)
  if (tid == 0) {
    double Sig[D][D];
#pragma unroll
    for (int p = 0; p < D; ++p)
#pragma unroll
      for (int q = 0; q < D; ++q) Sig[p][q] = sc->Sig[p * D + q];
    finalize_hyper<D, K, false, !REPLAY && CLV_L2_NR != 0>(sc->beta, Sig, a.omega2, a.hyper + (int64_t)c * HS);
    CLV_STAMP(a.stamps, s, 7, false);
    if (store_l2) {
      int q = K * D;
#pragma unroll
      for (int p = 0; p < D; ++p)
#pragma unroll
        for (int r = p; r < D; ++r) o[q++] = Sig[p][r];  // bi:412, tri:550-554
    }
    if (mode != 1 && is_stored(s, g))
      a.loglik[(int64_t)c * g.n_draws + draw_index(s, g)] = tot[NS - 1] / (double)g.n_global;  // np.mean
    if (mode == 0) {  // (mode 2, the persistent kernel, keeps the sweep index itself)
      // the last chain to finish advances the sweep counter (every workgroup of this launch has
      // read it before arriving)
      // relaxed: the next launch reads cur and the hyper state after the kernel boundary (whose
      // release/acquire makes them visible); an acq_rel RMW here would write back the whole L2
      const uint32_t old = __hip_atomic_fetch_add(&a.ctrl->arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old == (uint32_t)g.n_chains - 1) {
        __hip_atomic_store(&a.ctrl->arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&a.ctrl->cur, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// Level-2 draw of chain c after sweep s (mode 0), or the bivariate initial draw (mode 1):
// fixed-order sum of all unit partials, variates, algebra, hyper state, level-2 record and
// log-likelihood, then the sweep-counter arrival.  Executed by one 256-thread workgroup: the
// standalone hyper_kernel (sharded path) or the last-arriving sweep workgroup of the chain
// (fused path).  `units`: [world][chain][stride][units_per_rank] unit partials (the gathered
// buffer; at world size 1 this rank's unit partials, or its block partials when a unit is one
// block), summed in global unit order — so every path and GPU count is bitwise identical.
template <int D, int K, bool REPLAY, int NS, int NT>
__device__ void hyper_body(const HyperArgs& a, int c, int64_t s, int mode, const double* units,
                           double (*red)[NS], double* tot, double* var_iw, double* var_chi, double* var_noise,
                           L2Scratch* l2) {
  if constexpr (NS <= 16) {  // (trivariate / large K: the registers of the batch raised the
                             // sweep kernel's allocation, K = 9 125 -> 159 VGPRs; the phases below)
  // every load of the draw issued back to back — the prior block, the precomputed / replayed
  // variates and this lane's unit partials — then the LDS staging: one memory round trip for all
  // of them (hyper_variates' staging waits for its own loads before the units' are issued)
  const int tid = threadIdx.x;
  const int64_t hs = (D == 2) ? s + 1 : s;
  static_assert(NT >= 198, "one prior element per lane");
  const double pr = tid < 198 ? a.V[tid] : 0.0;
  double w_iw = 0.0, w_chi = 0.0, w_noise = 0.0;
  const bool preloaded = REPLAY || a.hvar;
  if constexpr (REPLAY) {
    const double* tv = a.r.tape + ((int64_t)c * a.r.tape_sweeps + (hs - 1)) * a.r.tape_sweep_stride +
                       (a.r.tape_sweep_stride - TAPE_HYPER);
    if (tid < 3) w_iw = tv[tid];
    if (tid < 3) w_chi = tv[3 + tid];
    if (tid < D * K) w_noise = tv[6 + tid];
  } else if (a.hvar) {  // precomputed by this sweep's kernel (sc1 stores: read with sc1 loads)
    const double* hv = a.hvar + (int64_t)c * HV;
    if (tid < 3) w_iw = __hip_atomic_load(hv + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid < 3) w_chi = __hip_atomic_load(hv + 3 + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid < D * K) w_noise = __hip_atomic_load(hv + 8 + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  double acc[NS];
  hyper_sum_units<NS, NT>(a, c, units, acc);
  if (tid < 198) l2->prior[tid] = pr;  // published by block_reduce's barriers
  if (preloaded) {
    if (tid < 3) var_iw[tid] = w_iw;
    if (tid < 3) var_chi[tid] = w_chi;
    if (tid < D * K) var_noise[tid] = w_noise;
  } else {
    uint32_t k0, k1;
    chain_key(a.r.seed, (int64_t)a.r.chain_first + c, &k0, &k1);
    constexpr int NTRIL = D * (D - 1) / 2;
    if (tid < NTRIL) var_iw[tid] = hyper_normal(k0, k1, HSLOT_NORMAL0 + tid, (uint32_t)hs);
    if (tid >= 32 && tid < 32 + D * K)
      var_noise[tid - 32] = hyper_normal(k0, k1, HSLOT_BETA_NORMAL0 + (tid - 32), (uint32_t)hs);
    if (tid >= 64 && tid < 64 + D) {  // second wavefront: the gamma rejection loops
      const int q = tid - 64;
      var_chi[q] = chi2_draw(k0, k1, (uint32_t)hs, q, a.nu_n - D + 1 + q);
    }
  }
  hyper_finish<D, K, REPLAY, NS, NT>(a, c, s, mode, acc, red, tot, var_iw, var_chi, var_noise, l2);
  return;
  }
  hyper_variates<D, K, REPLAY>(a, c, s, var_iw, var_chi, var_noise, l2);
  double acc[NS];
  hyper_sum_units<NS, NT>(a, c, units, acc);
  hyper_finish<D, K, REPLAY, NS, NT>(a, c, s, mode, acc, red, tot, var_iw, var_chi, var_noise, l2);
}

template <int D, int K, bool REPLAY>
__global__ __launch_bounds__(256) void hyper_kernel(HyperArgs a) {
  constexpr int NS = K * D + D * (D + 1) / 2 + 1;
  __shared__ double red[4][NS];
  __shared__ double tot[NS];
  __shared__ double var_iw[4], var_chi[4], var_noise[32];
  __shared__ L2Scratch l2;
  const int64_t done = __hip_atomic_load(&a.ctrl->cur, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int64_t s = a.mode == 1 ? 0 : done + 1;  // sweep whose statistics are reduced here
  hyper_body<D, K, REPLAY, NS, 256>(a, blockIdx.x, s, a.mode, a.units, red, tot, var_iw, var_chi, var_noise, &l2);
}

// ---------------------------------------------------------------------------------------------
// Hand-off helpers (fused peer exchange, persistent kernel)
// ---------------------------------------------------------------------------------------------
constexpr long long SLOT_EMPTY = -1ll;              // all-ones bit pattern: a NaN no arithmetic yields

__device__ __forceinline__ double ld_wt(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// System scope for the peer exchange: other GPUs write this rank's mail buffer over xGMI.
__device__ __forceinline__ double ld_sys(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ bool slot_full(double v) { return __double_as_longlong(v) != SLOT_EMPTY; }
__device__ __forceinline__ double slot_empty() { return __longlong_as_double(SLOT_EMPTY); }

// Bounded wait bookkeeping (uniform).  WAIT_GOING: keep polling; WAIT_OBSERVED: another wave raised
// the abort flag — leave without a record (the wave that raised it writes it); WAIT_EXPIRED: this
// wave's own bound ran out — write the record (report_wait) and only THEN raise the flag
// (raise_abort), so no wave that merely saw the flag can claim the record first (verdict r5: a
// customer wave that observed the level-2 workgroup's abort claimed it at 299.99 of 300 ms).  The
// abort flag is read every 16th poll only, so a poll iteration costs one memory round trip, not two.
enum : int { WAIT_GOING = 0, WAIT_OBSERVED = 1, WAIT_EXPIRED = 2 };
__device__ __forceinline__ int wait_state(const SweepArgs& a, uint64_t t0, uint32_t poll, uint64_t bound) {
  if ((poll & 15u) == 15u && __hip_atomic_load(&a.ctrl_rw->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    return WAIT_OBSERVED;
  return __builtin_amdgcn_s_memrealtime() - t0 > bound ? WAIT_EXPIRED : WAIT_GOING;
}
__device__ __forceinline__ void raise_abort(const SweepArgs& a) {
  __hip_atomic_store(&a.ctrl_rw->abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (a.abort_host) __hip_atomic_store(a.abort_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// The customers' wait for (beta, Sigma) is downstream of the level-2 side's waits (the draw it waits
// for is what those waits feed), so its bound is 1.5x theirs: a stall upstream expires upstream first
// and the record names the statistic that never came, not the hand-off slot that waited on it.
__device__ __forceinline__ uint64_t hyper_wait_ticks(const SweepArgs& a) { return a.wait_ticks + a.wait_ticks / 2; }

// The wait-timeout record (SweepArgs::diag): the wave whose bounded wait expired names what it was
// waiting for — the lowest lane still missing a slot reports its (unit or block, statistic, the
// bits it read) — and, with peers, the progress words in this rank's mail (the sweep each rank's
// level-2 side last started to poll for).  Word layout: [0] claimed, [1] kind (WAIT_*), [2] sweep,
// [3] chain, [4] rank, [5] unit / block, [6] statistic, [7] bits, [8] polls, [9] waited ticks
// (100 MHz), [10] lanes of the wave still missing, [11..15] progress of ranks 0..4 (-1: none).
// Called by every lane of the wave (one ballot), only by a wave whose own bound expired (WAIT_EXPIRED),
// before it raises the abort flag; the first such wave of the launch writes.  Waves that stop because
// they observed the flag never call it, so the recorded wait is always >= its bound.
__device__ __forceinline__ void report_wait(const SweepArgs& a, int kind, int64_t s, int c, bool lane_ok,
                                            int64_t unit, int stat, uint64_t bits, uint32_t polls, uint64_t t0) {
  if (!a.diag) return;
  const uint64_t miss = __ballot(!lane_ok);
  if (!miss) return;
  const int first = __ffsll((unsigned long long)miss) - 1;
  if ((int)(threadIdx.x & 63) != first) return;
  if (atomicCAS(a.diag, 0ull, 1ull) != 0ull) return;
  a.diag[1] = (unsigned long long)kind;
  a.diag[2] = (unsigned long long)s;
  a.diag[3] = (unsigned long long)c;
  a.diag[4] = (unsigned long long)a.rank;
  a.diag[5] = (unsigned long long)unit;
  a.diag[6] = (unsigned long long)stat;
  a.diag[7] = bits;
  a.diag[8] = polls;
  a.diag[9] = __builtin_amdgcn_s_memrealtime() - t0;
  a.diag[10] = (unsigned long long)__popcll(miss);
  const Geometry& g = a.g;
  for (int q = 0; q < 5; ++q) {
    unsigned long long v = ~0ull;
    if (a.mail && q < g.world_size)
      v = __builtin_bit_cast(unsigned long long,
                             __hip_atomic_load(a.mail + mail_slots(g.world_size, g.n_chains, g.stride, g.units_per_rank) + q,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    a.diag[11 + q] = v;
  }
}

// This rank's level-2 side starts to poll for sweep s: its progress word in every rank's mail.
__device__ __forceinline__ void post_progress(const SweepArgs& a, double* const* peers, int64_t s) {
  const Geometry& g = a.g;
  const int64_t off = mail_slots(g.world_size, g.n_chains, g.stride, g.units_per_rank) + a.rank;
  for (int q = 0; q < g.world_size; ++q)
    __hip_atomic_store(peers[q] + off, __builtin_bit_cast(double, (int64_t)s), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

// The shader clock against the 100 MHz s_memrealtime: (delta s_memtime, delta s_memrealtime) of one
// interval of sweep s on one CU, chain 0 (SweepArgs::clk, clv_clock_ghz).
// s_memtime counts per XCD — differences taken across CUs of different XCDs would be meaningless —
// so each slot holds one workgroup's own interval: the persistent level-2 workgroup's from its
// previous publish.  The launch-per-sweep kernel keeps no record: marks in one workgroup per launch
// (its start to its block partial) measured c4 +1.5%, c5 +1% per sweep (profiles/r05_ab_clock_record.txt).
#ifndef CLV_CLOCK_RECORD
#define CLV_CLOCK_RECORD 1
#endif
struct ClockMark {
  unsigned long long m, r;
  __device__ __forceinline__ static ClockMark now() {
    return ClockMark{__builtin_amdgcn_s_memtime(), __builtin_amdgcn_s_memrealtime()};
  }
};
__device__ __forceinline__ ClockMark clock_mark(unsigned long long* clk, int64_t s, ClockMark from) {
  const ClockMark t = ClockMark::now();
  unsigned long long* p = clk + 2 * (s & (CLK_RING - 1));
  p[0] = t.m - from.m;
  p[1] = t.r - from.r;
  return t;
}

// ---------------------------------------------------------------------------------------------
// Sweep kernel
// ---------------------------------------------------------------------------------------------
// One customer's sweep state (per lane and task).
// CL (covariates in LDS): the launch-per-sweep kernel keeps a lane's covariate row in its
// workgroup's LDS ([k-1][BLOCK], each lane reads back only what it wrote — no barrier) instead of
// K-1 register pairs live across the whole MH phase (c5, K = 9: 16 VGPRs).
template <int D, int K, bool CL = false>
struct Cust {
  int64_t i;          // local customer index (clamped to a valid row for inactive tasks)
  bool active;
  double xr_[CL ? 1 : K];  // [1, covariates] in registers (CL: unused)
  double* cl;         // CL: this lane's covariate column in LDS (element k-1 at cl[(k-1) * BLOCK])
  __device__ __forceinline__ double x(int k) const {
    if constexpr (CL) return k == 0 ? 1.0 : cl[(k - 1) * BLOCK];
    else return xr_[k];
  }
  double tx, T, xm;
  int32_t xi;         // x as loaded (converted in cust_prepare, so the load is not waited for early)
  double lam, mu, eta, tau;
  bool z;
  double ll, lm, cur; // MH state (log scale) and its log posterior
  LPFast fc;          // Philox-mode log-posterior coefficients
  LPConst lc;         // replay-mode log-posterior constants
  uint32_t gi;        // global customer index (Philox counter)
};

// Phase A1: the customer's loads (CBS row, covariates, state), issued before the workgroup's
// exp-table barrier so their latency overlaps it.
template <int D, int K, bool CL>
__device__ __forceinline__ void cust_load(Cust<D, K, CL>& u, const SweepArgs& a, int c) {
  const Geometry& g = a.g;
  const int64_t i = u.i;
  u.tx = a.tx[i];
  u.T = a.T[i];
  if constexpr (CL) {
#pragma unroll
    for (int k = 1; k < K; ++k) u.cl[(k - 1) * BLOCK] = a.cov[(int64_t)(k - 1) * g.n + i];
  } else {
    u.xr_[0] = 1.0;
#pragma unroll
    for (int k = 1; k < K; ++k) u.xr_[k] = a.cov[(int64_t)(k - 1) * g.n + i];
  }
  const int64_t ci = (int64_t)c * g.n + i;
  u.lam = a.lam[ci];
  u.mu = a.mu[ci];
  u.xi = a.x[i];
  u.gi = (uint32_t)(g.shard_begin + i);
}

// Phase A2a (bi:193-227): draw_z, draw_tau and the log-scale state — independent of the level-2
// state (beta, Sigma), so the persistent kernel runs it for sweep s+1 while sweep s's level-2
// draw is still in flight.
template <int D, int K, bool REPLAY, bool CL>
__device__ __forceinline__ void cust_ztau(Cust<D, K, CL>& u, const SweepArgs& a, int64_t s, uint32_t k0, uint32_t k1,
                                          const double* tape, const double* exp_tab) {
  const Geometry& g = a.g;
  const int64_t i = u.i;
  const double lam = u.lam, mu = u.mu;
  const double tx = u.tx, T = u.T;
  int32_t xi = u.xi;
  asm volatile("" : "+v"(xi));  // keeps the int->double conversion (and its load wait) here
  u.xm = (double)xi;

  // ---- draw_z (bi:193-200)
  // Replay: u_z and the per-customer tau variate (standard exponential if alive, uniform if
  // churned — the reference's consumption order, bi:215-225). Philox: slot SLOT_ZTAU words
  // (x, y) -> u_z, (z, w) -> U in [0,1) for churned / -log(U') with U' in (0,1] for alive.
  double u_z;
  uint32_t rz = 0, rw = 0;
  double v_tau = 0.0;
  if constexpr (REPLAY) {
    u_z = tape[i];
    v_tau = tape[g.n + i];
  } else {
    const u32x4 r = customer_block(k0, k1, u.gi, (uint32_t)s, SLOT_ZTAU);
    u_z = u53(r.x, r.y);
    rz = r.z;
    rw = r.w;
  }
  const double ml = mu + lam;
  const double zz = ml * (T - tx);
  // Philox mode: exp_fast, argument capped at 700 (exp(-700) ~ 1e-304 already makes
  // p(alive) < 2^-53, the smallest nonzero u_z, as exp(-zz) underflowing to 0 does)
  const double e = REPLAY ? exp(-zz) : exp_fast(-min700(zz), exp_tab);
  bool z;
  if constexpr (REPLAY) {
    const double p = (ml * e) / (ml * e + mu * (1.0 - e));
    z = u_z < p;
  } else {  // Philox mode: u_z < a / b as u_z * b < a (b > 0), no fp64 division
    const double ae = ml * e;
    z = u_z * (ae + mu * (1.0 - e)) < ae;
  }
  u.z = z;

  // ---- draw_tau (bi:203-227)
  double tau;
  if constexpr (REPLAY) {
    if (z) {
      tau = T + (1.0 / mu) * v_tau;
    } else {
      const double uu = v_tau;
      const double e_tx = exp(-min700(ml * tx));  // both capped at 700 (bi:223)
      const double e_T = exp(-min700(ml * T));
      tau = -log((1 - uu) * e_tx + uu * e_T) / ml;
    }
  } else {
    // Philox mode, branch-free (the lanes of a wave mix alive and churned customers): one
    // log_fast of either -E's uniform U' in (0, 1] (alive: tau = T + E / mu) or the truncated
    // exponential's argument (churned: tau = -log(.) / ml), one division
    const double uu = u53(rz, rw);
    double e_tx, e_T;
    exp_fast2(-min700(ml * tx), -min700(ml * T), exp_tab, e_tx, e_T);
    const double L = log_fast(z ? u53_open0(rz, rw) : (1 - uu) * e_tx + uu * e_T, exp_tab);
    const double q = L / (z ? mu : ml);
    tau = z ? T - q : -q;
  }
  u.tau = tau;
  u.lc.xm = u.xm;
  u.lc.omz = z ? 0.0 : 1.0;
  u.lc.w = z ? T : tau;
  if constexpr (REPLAY) {
    u.ll = log(lam);
    u.lm = log(mu);
  } else {
    u.ll = log_fast(lam, exp_tab);
    u.lm = log_fast(mu, exp_tab);
  }
}

// Phase A2b (bi:280-290): log-posterior constants from (beta, Sigma) and the current point's
// log posterior.
template <int D, int K, bool REPLAY, bool CL>
__device__ __forceinline__ void cust_coeffs(Cust<D, K, CL>& u, const double* H, const double* exp_tab) {
  // ---- _draw_level_1 (bi:268-339): mv_mean = X @ beta (bi:284)
  double m0 = 0.0, m1 = 0.0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    m0 += u.x(k) * H[H_BETA + k * D + 0];
    m1 += u.x(k) * H[H_BETA + k * D + 1];
  }
  LPConst& lc = u.lc;
  lc.m0 = m0;
  lc.m1 = m1;
  lc.p00 = H[H_P00];
  lc.p01 = H[H_P01];
  lc.p11 = H[H_P11];
  if constexpr (REPLAY) {
    u.cur = log_post(lc, u.ll, u.lm);
  } else {
    LPFast& fc = u.fc;
    fc.A = -0.5 * lc.p00;
    fc.B = -lc.p01;
    fc.C = -0.5 * lc.p11;
    fc.Dl = lc.xm + lc.p00 * lc.m0 + lc.p01 * lc.m1;
    fc.El = lc.omz + lc.p01 * lc.m0 + lc.p11 * lc.m1;
    fc.w = lc.w;
    u.cur = u.lm > 5.0 ? -__builtin_inf() : log_post_fast(fc, u.ll, u.lm, exp_tab);
  }
}

// Phase A2 (bi:193-227, bi:280-290): both of the above.
template <int D, int K, bool REPLAY, bool CL>
__device__ __forceinline__ void cust_prepare(Cust<D, K, CL>& u, const SweepArgs& a, int c, int64_t s, const double* H,
                                             uint32_t k0, uint32_t k1, const double* tape, const double* exp_tab) {
  (void)c;
  cust_ztau<D, K, REPLAY>(u, a, s, k0, k1, tape, exp_tab);
  cust_coeffs<D, K, REPLAY>(u, H, exp_tab);
}

// clip70(a * b + c) as three VALU ops: a VOP3 v_fma_f64 into a fresh register (the compiler
// otherwise emits v_mov_b64 + v_fmac_f64, an accumulator copy, when c stays live) and v_max/v_min
// written out too, so no NaN-canonicalising v_max is inserted after the asm (the operands are never
// NaN).  Separate statements, so the scheduler interleaves the two coordinates' chains.
__device__ __forceinline__ double clip70_fma(double a, double b, double c) {
  double r, lo = -70.0, hi = 70.0;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(r), "s"(lo));  // bounds from SGPRs: no per-step
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(r), "s"(hi));  // v_mov_b64 into VGPRs
  return r;
}

// One Philox-mode MH step (bi:316-335) with lp(proposal) = -inf for pm > 5 (Q3): accept iff
// pm <= 5 and exp(plp - cur) > u  <=>  plp > cur + log(u)  (cur = -inf accepts any finite one;
// cur + log u = fma(log2 u, ln 2, cur) is formed off the dependent chain, alongside the proposal;
// a padded step's log2 u = +inf gives +inf or NaN there, never accepted).
// The log mu proposal needs only the lower bound: a proposal above 5 is rejected by the Q3 cap
// whatever its value (and its log posterior, even NaN, is then never looked at), and an accepted
// one is <= 5 < 70, so max(., -70) accepts exactly what clip(., -70, 70) does.
__device__ __forceinline__ double prop_lm(double a, double b, double c) {
  double r, lo = -70.0;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(r), "s"(lo));
  return r;
}

template <int D, int K, bool CL>
__device__ __forceinline__ void mh_step(Cust<D, K, CL>& u, double s00, double s11, float t_l, float t_m, float l2u,
                                        const double* exp_tab) {
  const double thr = __builtin_fma((double)l2u, 0x1.62e42fefa39efp-1, u.cur);  // cur + ln2 log2 u
  const double pl = clip70_fma(s00, (double)t_l, u.ll);
  const double pm = prop_lm(s11, (double)t_m, u.lm);
  const double plp = log_post_fast(u.fc, pl, pm, exp_tab);
  // The accept as three exec-masked 64-bit moves (3 VALU) instead of six v_cndmask_b32 halves:
  // exec narrowed to the accepting lanes for the moves and restored inside the one asm block (so
  // still no branch: the chunk's steps stay one basic block).  Same predicate as below: 5 >= pm
  // and plp > thr, both false on NaN.
  uint64_t m0, m1, sv;
  const double five = 5.0;
  asm volatile(
      "v_cmp_ge_f64_e64 %[m0], %[five], %[pm]\n\t"
      "v_cmp_gt_f64_e64 %[m1], %[plp], %[thr]\n\t"
      "s_and_saveexec_b64 %[sv], %[m0]\n\t"
      "s_and_b64 exec, exec, %[m1]\n\t"
      "v_mov_b64 %[ll], %[pl]\n\t"
      "v_mov_b64 %[lm], %[pm]\n\t"
      "v_mov_b64 %[cur], %[plp]\n\t"
      "s_mov_b64 exec, %[sv]"
      : [ll] "+v"(u.ll), [lm] "+v"(u.lm), [cur] "+v"(u.cur), [m0] "=&s"(m0), [m1] "=&s"(m1), [sv] "=&s"(sv)
      : [pl] "v"(pl), [pm] "v"(pm), [plp] "v"(plp), [thr] "v"(thr), [five] "s"(five)
      : "scc");
}

// The sweep's S Philox-mode MH steps.  Software pipeline: the Philox blocks and t3 transforms of
// the next chunk of MH_CHUNK_STEPS steps are independent of the state; each full chunk's steps and
// the next chunk's variates form one branch-free basic block, so the scheduler can interleave
// that work with the dependent fp64 accept/reject chain.  The last chunk's steps beyond S are
// padded with log U = +inf (never accepted: the state is unchanged) instead of a branch.
// q0: the first chunk run here (the chunks below it were run from drawn-ahead variates).
template <bool PIPE = (SWEEP_MH_PIPELINE != 0), int D, int K, bool CL>
__device__ __forceinline__ void mh_run(Cust<D, K, CL>& cu, const SlotPhilox& ph, double s00, double s11, int S,
                                       const double* exp_tab, int q0 = 0) {
  constexpr int MC = MH_CHUNK_STEPS;
  const int n_chunks = (S + MC - 1) / MC;
  if (n_chunks <= q0) return;
  float tl[MC], tm[MC], lu[MC];
  // trivariate launch-per-sweep instances (c5): the packed t3 pair — c5 122.8 -> 121.6 us per sweep,
  // bitwise the same variates (the persistent kernels keep the scalar form: c2 measured slower)
  constexpr bool PK = D == 3;
  if constexpr (!PIPE) {
  // no software pipeline (occupancy hides the latency instead): variates, then the chunk's steps
  for (int ch = q0; ch < n_chunks; ++ch) {
    mh_chunk_variates<PK>(ph, (uint32_t)ch, tl, tm, lu);
    const int rem = S - ch * MC;
#pragma unroll
    for (int st = 0; st < MC; ++st) mh_step(cu, s00, s11, tl[st], tm[st], st < rem ? lu[st] : __builtin_inff(), exp_tab);
  }
  return;
  }
  mh_chunk_variates<PK>(ph, (uint32_t)q0, tl, tm, lu);
  for (int ch = q0; ch + 1 < n_chunks; ++ch) {
    float ntl[MC], ntm[MC], nlu[MC];
    mh_chunk_variates<PK>(ph, (uint32_t)(ch + 1), ntl, ntm, nlu);
#pragma unroll
    for (int st = 0; st < MC; ++st) mh_step(cu, s00, s11, tl[st], tm[st], lu[st], exp_tab);
#pragma unroll
    for (int st = 0; st < MC; ++st) {
      tl[st] = ntl[st];
      tm[st] = ntm[st];
      lu[st] = nlu[st];
    }
  }
  const int rem = S - (n_chunks - 1) * MC;
#pragma unroll
  for (int st = 0; st < MC; ++st) mh_step(cu, s00, s11, tl[st], tm[st], st < rem ? lu[st] : __builtin_inff(), exp_tab);
}

// Persistent kernel: the MH variates of a whole sweep (up to PRE_STEPS steps) drawn ahead, while
// the wave would otherwise idle in the level-2 hand-off; the MH phase after (beta, Sigma) arrive is
// then only the dependent fp64 accept/reject chain.  Steps >= S carry log U = +inf (never taken).
// The variates live in LDS, one column per lane (each lane reads back only what it wrote: no
// barrier), not in 60 VGPRs: the persistent kernel's customer path spilled with them in registers.
constexpr int PRE_STEPS = 20;
constexpr int PRE_LDS_BYTES = PRE_STEPS * BLOCK * 12;  // float2 (t_l, t_m) + float log U per step and lane
struct PreVariates {
  float2* t;  // [PRE_STEPS][BLOCK]
  float* u;   // [PRE_STEPS][BLOCK]
  int lane;
};

// S is re-read as an opaque scalar at every call: held loop-invariant, the compiler hoisted the
// per-step "k < S" lane masks out of the sweep loop and spilled them to VGPR lanes (2 v_readlane
// + 1 v_cndmask per step); the padding select now runs only in a partial last chunk.
__device__ __forceinline__ int opaque_uniform(int x) {
  x = __builtin_amdgcn_readfirstlane(x);
  asm volatile("" : "+s"(x));
  return x;
}

template <int NQ = PRE_STEPS / MH_CHUNK_STEPS>
__device__ __forceinline__ void mh_pre_variates(const SlotPhilox& ph, int S_, const PreVariates& v) {
  constexpr int MC = MH_CHUNK_STEPS;
  const int S = opaque_uniform(S_);
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    if (q * MC < S) {  // wave-uniform
      float tl[MC], tm[MC], lu[MC];
      mh_chunk_variates(ph, (uint32_t)q, tl, tm, lu);
      if (q * MC + MC <= S) {  // full chunk
#pragma unroll
        for (int st = 0; st < MC; ++st) {
          const int k = q * MC + st;
          v.t[k * BLOCK + v.lane] = make_float2(tl[st], tm[st]);
          v.u[k * BLOCK + v.lane] = lu[st];
        }
      } else {
#pragma unroll
        for (int st = 0; st < MC; ++st) {
          const int k = q * MC + st;
          v.t[k * BLOCK + v.lane] = make_float2(tl[st], tm[st]);
          v.u[k * BLOCK + v.lane] = k < S ? lu[st] : __builtin_inff();
        }
      }
    }
  }
}

template <int NQ = PRE_STEPS / MH_CHUNK_STEPS, int D, int K, bool CL>
__device__ __forceinline__ void mh_run_pre(Cust<D, K, CL>& cu, const PreVariates& v, double s00, double s11, int S,
                                           const double* exp_tab) {
  constexpr int MC = MH_CHUNK_STEPS;
  S = opaque_uniform(S);
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    if (q * MC < S) {  // wave-uniform
      float2 t[MC];
      float u[MC];
#pragma unroll
      for (int st = 0; st < MC; ++st) {  // the chunk's LDS reads issued together, ahead of the chain
        t[st] = v.t[(q * MC + st) * BLOCK + v.lane];
        u[st] = v.u[(q * MC + st) * BLOCK + v.lane];
      }
#pragma unroll
      for (int st = 0; st < MC; ++st) mh_step(cu, s00, s11, t[st].x, t[st].y, u[st], exp_tab);
    }
  }
}

// Phase C1: state update (bi:337-338), draw_eta (tri:306-333), the likelihood term of stored
// sweeps (bi:423-427) and the customer's sufficient statistics into acc.
template <int D>
struct CustOut {
  double lam, mu, eta, lgl, lgm, leta;  // leta = log(eta) (Philox mode: the exponent itself)
};

// draw_eta's standard normal (tri:333 rng.normal), Philox mode: fp64 Box-Muller from the
// customer's SLOT_ETA block.  Independent of the state, so the persistent kernel draws it for
// sweep s+1 in the level-2 hand-off window (with the MH variates), off the sweep's serial path.
__device__ __forceinline__ double eta_normal(uint32_t k0, uint32_t k1, uint32_t gi, int64_t s, const double* tab) {
  const u32x4 r = customer_block(k0, k1, gi, (uint32_t)s, SLOT_ETA);
  return sqrt(-2.0 * log_fast(u53_open0(r.x, r.y), tab)) * cos2pi_u53(r.z, r.w, tab);  // tab: FAST_TAB_N3
}

template <int D, int K, bool REPLAY, bool CL>
__device__ __forceinline__ CustOut<D> cust_finish(Cust<D, K, CL>& u, const SweepArgs& a, int64_t s, bool stored,
                                                  const double* H, uint32_t k0, uint32_t k1, const double* tape,
                                                  const double* exp_tab, StatGen<D, K>& st,
                                                  const double* zeta_pre = nullptr) {
  const Geometry& g = a.g;
  const int64_t i = u.i;
  // bi:337-338 (state back to natural scale).  Replay reproduces the reference's exp/log round
  // trips (quirk Q5) bit for bit; Philox mode takes log(exp(ll)) = ll (equal to within an ulp).
  double lam, mu;
  if constexpr (REPLAY) {
    lam = exp(u.ll);
    mu = exp(u.lm);
  } else {
    exp_fast2(u.ll, u.lm, exp_tab, lam, mu);
  }
  double eta = 1.0, leta = 0.0, Y[D];
  if constexpr (D == 3) {
    double m2 = 0.0;
#pragma unroll
    for (int k = 0; k < K; ++k) m2 += u.x(k) * H[H_BETA + k * D + 2];
    const double post_var = H[H_POSTVAR];
    // Philox mode: the reciprocals come with the hyper state (no per-customer fp64 division)
    const double post_mean = REPLAY ? post_var * (a.log_s[i] / H[H_OMEGA2] + m2 / H[H_S22])
                                    : post_var * __builtin_fma(a.log_s[i], H[H_INV_OMEGA2], m2 * H[H_INV_S22]);
    double zeta;
    if constexpr (REPLAY) {
      zeta = tape[(int64_t)(2 + 3 * g.S) * g.n + i];
    } else {
      zeta = zeta_pre ? *zeta_pre : eta_normal(k0, k1, u.gi, s, exp_tab);
    }
    const double xe = post_mean + H[H_SQRT_POSTVAR] * zeta;
    if constexpr (REPLAY) {
      eta = exp(xe);
      leta = log(eta);  // tri:534 (level 2 sees log of the natural-scale draw)
    } else {  // Philox mode: the table exp, and log(exp(x)) = x (within an ulp, as for lambda, mu)
      if (__builtin_fabs(xe) <= 700.0) eta = exp_fast(xe, exp_tab);
      else eta = exp(xe);
      leta = xe;
    }
    // tri: level 2 sees log(lambda) before the storage round trip (tri:529-536 before :542)
    Y[0] = REPLAY ? log(lam) : u.ll;
    Y[1] = REPLAY ? log(mu) : u.lm;
    Y[2] = leta;
  }
  double lik = 0.0, lgl = 0.0, lgm = 0.0;
  if (stored) {
    if constexpr (REPLAY) {
      lam = exp(log(lam));  // quirk Q5 (bi:405-406)
      mu = exp(log(mu));
    }
    lgl = REPLAY ? log(lam) : u.ll;
    lgm = REPLAY ? log(mu) : u.lm;
    lik = (u.xm * lgl + u.lc.omz * lgm) - (lam + mu) * u.lc.w;  // bi:423-427
  }
  if constexpr (D == 2) {
    // bi: the next level-2 draw uses log of the carried state (bi:393)
    Y[0] = REPLAY ? log(lam) : u.ll;
    Y[1] = REPLAY ? log(mu) : u.lm;
  }
  u.lam = lam;
  u.mu = mu;
  // ---- sufficient statistics X'Y (K x D), Y'Y (upper triangle), likelihood term: formed in the
  // workgroup reduction (block_reduce_gen), a few at a time
#pragma unroll
  for (int k = 0; k < K; ++k) st.xr[k] = u.x(k);
#pragma unroll
  for (int d = 0; d < D; ++d) st.Y[d] = Y[d];
  st.lik = lik;
  st.on = true;
  return CustOut<D>{lam, mu, eta, lgl, lgm, leta};
}

// The customer's running sums of a stored sweep (summary sinks), loaded ahead of cust_store: the
// launch-per-sweep kernel issues these loads together with the block partial's store, so the
// hand-off's drain covers both in one memory round trip (sweep_body).  Bivariate: the 9 sums
// without ETA / LOG_ETA.
template <int D>
struct SumsPre {
  static constexpr int N = D == 3 ? CLV_N_SUM_STATS : CLV_N_SUM_STATS - 2;
  static __device__ __forceinline__ constexpr int slot(int k) { return (D == 3 || k < CLV_SUM_ETA) ? k : k - 2; }
  double v[N];
};
template <int D>
__device__ __forceinline__ void prefetch_sums(const SweepArgs& a, int c, int64_t i, SumsPre<D>& p) {
  const double* sm = a.sums + (int64_t)c * CLV_N_SUM_STATS * a.g.n + i;
#pragma unroll
  for (int k = 0; k < CLV_N_SUM_STATS; ++k) {
    if (D == 2 && (k == CLV_SUM_ETA || k == CLV_SUM_LOG_ETA)) continue;
    p.v[SumsPre<D>::slot(k)] = sm[(int64_t)k * a.g.n];
  }
}

// Phase C2: storage (bi:402-412, tri:539-571) — issued after the workgroup's partial has been
// handed off, so the hand-off's store drain does not wait for them — and the carried state.
// pre: the running sums loaded ahead (prefetch_sums; the same sums + value, the same bits).
template <int D, int K, bool CL>
__device__ __forceinline__ void cust_store(const Cust<D, K, CL>& u, const CustOut<D>& o, const SweepArgs& a, int c,
                                           int64_t s, bool stored, bool store_state,
                                           const SumsPre<D>* pre = nullptr) {
  const Geometry& g = a.g;
  const int64_t i = u.i;
  if (stored) {
    const int64_t dr = draw_index(s, g);
    if (a.level1) {
      double* w = a.level1 + (((int64_t)c * g.n_draws + dr) * g.n + i) * (D + 2);
      w[0] = o.lam;
      w[1] = o.mu;
      w[2] = u.tau;
      w[3] = u.z ? 1.0 : 0.0;
      if constexpr (D == 3) w[4] = o.eta;
    }
    if (a.sums) {
      double* sm = a.sums + (int64_t)c * CLV_N_SUM_STATS * g.n + i;
      auto acc = [&](int k, double v) {
        if (pre) sm[k * g.n] = pre->v[SumsPre<D>::slot(k)] + v;
        else sm[k * g.n] += v;
      };
      acc(CLV_SUM_LAMBDA, o.lam);
      acc(CLV_SUM_MU, o.mu);
      acc(CLV_SUM_Z, u.z ? 1.0 : 0.0);
      acc(CLV_SUM_LOG_LAMBDA, o.lgl);
      acc(CLV_SUM_LOG_MU, o.lgm);
      acc(CLV_SUM_LAMBDA2, o.lam * o.lam);
      acc(CLV_SUM_MU2, o.mu * o.mu);
      if constexpr (D == 3) {
        acc(CLV_SUM_ETA, o.eta);
        acc(CLV_SUM_LOG_ETA, o.leta);
      }
      acc(CLV_SUM_MU_CAPPED, fmin(o.mu, CLV_SUMMARY_MU_CAP));  // np.clip(mu, None, 0.05)
      acc(CLV_SUM_TAU, u.tau);
    }
    if (a.qstore)  // one coalesced 8-byte store per lane
      a.qstore[((int64_t)c * g.n_draws + dr) * g.n + i] = make_float2((float)o.lam, (float)o.mu);
  }
  if (store_state) {
    const int64_t ci = (int64_t)c * g.n + i;
    a.lam[ci] = o.lam;
    a.mu[ci] = o.mu;
  }
}

static_assert(BLOCK == EXP_TAB_N, "the sweep kernel stages the exp table with one entry per lane");

// FX: the fused peer exchange (world size > 1 after clv_p2p_connect) compiled in — instances of
// their own, launched for sharded runs only (compiled into the world-size-1 kernels it cost c4 /
// c5 1.8% / 1.6% per sweep).
template <int D, int K, bool REPLAY, bool FX>
__device__ __forceinline__ void sweep_body(const SweepArgs& a) {
  constexpr int NT = BLOCK;
  constexpr int NXY = K * D;
  constexpr int NYY = D * (D + 1) / 2;
  constexpr int NS = NXY + NYY + 1;
  __shared__ double red[BLOCK / 64][NS];
  __shared__ double tot[NS];
  __shared__ __attribute__((aligned(16))) double exp_tab[D == 3 ? FAST_TAB_N3 : FAST_TAB_N];
  // the exp/log(/cos) table's global loads are issued first; they are stored to LDS (and the
  // barrier taken) after the customer's own loads are in flight
  static_assert(BLOCK == EXP_TAB_N && BLOCK == LOG_TAB_N && BLOCK == COS_TAB_N, "one table entry per thread");
  double tab_v = 0.0, tab_l0 = 0.0, tab_l1 = 0.0, tab_c0 = 0.0, tab_c1 = 0.0;
  if (!REPLAY) {
    tab_v = exp_tab_entry(threadIdx.x);
    tab_l0 = LOG_TAB[2 * threadIdx.x];
    tab_l1 = LOG_TAB[2 * threadIdx.x + 1];
    if constexpr (D == 3) {
      tab_c0 = COS_TAB[2 * threadIdx.x];
      tab_c1 = COS_TAB[2 * threadIdx.x + 1];
    }
  }

  const Geometry& g = a.g;
  const int c = blockIdx.y;
  const int b = blockIdx.x;
  if constexpr (FX) {  // a wait of an earlier launch of this call timed out: the call fails, and
                       // its remaining launches return at once (the host restores the state)
    if (a.fuse && g.world_size > 1 &&
        __hip_atomic_load(&a.ctrl_rw->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      return;
  }
  // The customer's loads go out first, so that their latency, the exp table's and the sweep
  // index's overlap (one memory round trip before compute instead of several).
  constexpr bool CL = CovLds<D, K>::value;
  __shared__ double cov_s[CL ? (K - 1) * BLOCK : 1];
  Cust<D, K, CL> cu;
  cu.cl = cov_s + threadIdx.x;
  {
    const int64_t i = (int64_t)b * BLOCK + threadIdx.x;
    cu.active = i < g.n;
    cu.i = cu.active ? i : (g.n > 0 ? g.n - 1 : 0);
  }
  if (!a.init && g.n > 0) cust_load(cu, a, c);  // inactive lanes load a clamped valid row
  // The sweep index: a scalar load of the uniform counter (written by the previous launch's tail;
  // this launch's tail overwrites it only after every workgroup has arrived, i.e. read it).
  const int64_t s = a.init ? 0 : a.ctrl->cur + 1;
  const bool stored = !a.init && is_stored(s, g);

  StatGen<D, K> st{};
  if (threadIdx.x == 0 && !a.init) {
    CLV_STAMP(a.stamps, s, 0, true);
#ifndef CLV_STAMP_L2SPLIT
    CLV_STAMP(a.stamps, s, 5, false);
#endif
    CLV_WG_STAMP(a.stamps, (int64_t)c * g.nb_local + b, 0);
    CLV_WG_STAMP(a.stamps, (int64_t)c * g.nb_local + b, 2);
    CLV_WG_STAMP(a.stamps, (int64_t)c * g.nb_local + b, 3);
    CLV_WG_STAMP(a.stamps, (int64_t)c * g.nb_local + b, 4);
  }

  if (a.init) {
    // bi:368-370 / tri:489-491: initial state and the statistics of the first level-2 draw
    if (cu.active) {
      const int64_t i = cu.i;
      const double tx = a.tx[i];
      const double lam = a.lam_init;
      const double mu = 1.0 / (tx + 0.5 / a.lam_init);
      st.xr[0] = 1.0;
#pragma unroll
      for (int k = 1; k < K; ++k) st.xr[k] = a.cov[(int64_t)(k - 1) * g.n + i];
      st.Y[0] = log(lam);
      st.Y[1] = log(mu);
      if constexpr (D == 3) st.Y[2] = 0.0;
      st.on = true;
      const int64_t ci = (int64_t)c * g.n + i;
      a.lam[ci] = lam;
      a.mu[ci] = mu;
    }
  }
  if (!REPLAY) {
    exp_tab[threadIdx.x] = tab_v;
    exp_tab[EXP_TAB_N + 2 * threadIdx.x] = tab_l0;
    exp_tab[EXP_TAB_N + 2 * threadIdx.x + 1] = tab_l1;
    if constexpr (D == 3) {
      exp_tab[FAST_TAB_N + 2 * threadIdx.x] = tab_c0;
      exp_tab[FAST_TAB_N + 2 * threadIdx.x + 1] = tab_c1;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0 && !a.init) CLV_WG_STAMP(a.stamps, (int64_t)c * g.nb_local + b, 8);

  // ---- the next level-2 draw's Philox variates (independent of the statistics): computed by
  // the last wavefront of the chain's last workgroup — the partially filled one — so the draw's
  // serial tail only loads them.  Written with sc1 (write-through) stores.
  if constexpr (!REPLAY) {
    if (a.hvar_out && !a.init && b == g.nb_local - 1 && (int)(threadIdx.x >> 6) == NT / 64 - 1) {
      const int l = threadIdx.x & 63;
      const int64_t hs = (D == 2) ? s + 1 : s;
      uint32_t k0, k1;
      chain_key(a.r.seed, (int64_t)a.r.chain_first + c, &k0, &k1);
      double v = 0.0;
      int slot = -1;
      if (l < D * (D - 1) / 2) {
        v = hyper_normal(k0, k1, HSLOT_NORMAL0 + l, (uint32_t)hs);
        slot = l;
      } else if (l >= 8 && l < 8 + D * K) {
        v = hyper_normal(k0, k1, HSLOT_BETA_NORMAL0 + (l - 8), (uint32_t)hs);
        slot = l;
      } else if (l >= 40 && l < 40 + D) {
        v = chi2_draw(k0, k1, (uint32_t)hs, l - 40, a.h.nu_n - D + 1 + (l - 40));
        slot = 3 + (l - 40);
      }
      if (slot >= 0) __hip_atomic_store(a.hvar_out + (int64_t)c * HV + slot, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }

  CustOut<D> out{};
  if (!a.init && cu.active) {
    const double* H = a.hyper + (int64_t)c * HS;
    uint32_t k0 = 0, k1 = 0;
    const double* tape = nullptr;
    if constexpr (REPLAY) {
      tape = a.r.tape + ((int64_t)c * a.r.tape_sweeps + (s - 1)) * a.r.tape_sweep_stride;
    } else {
      chain_key(a.r.seed, (int64_t)a.r.chain_first + c, &k0, &k1);
    }
    cust_prepare<D, K, REPLAY>(cu, a, c, s, H, k0, k1, tape, exp_tab);
    if (threadIdx.x == 0) CLV_WG_STAMP(a.stamps, (int64_t)c * g.nb_local + b, 9);
    const double s00 = H[H_S00];
    const double s11 = H[H_S11];
    if constexpr (REPLAY) {
      {
        auto& u = cu;
        for (int j = 0; j < g.S; ++j) {
          const double tl = tape[(int64_t)(2 + 3 * j) * g.n + u.i];
          const double tm = tape[(int64_t)(3 + 3 * j) * g.n + u.i];
          const double uu = tape[(int64_t)(4 + 3 * j) * g.n + u.i];
          const double pl = clip70(u.ll + s00 * tl);
          const double pm = clip70(u.lm + s11 * tm);
          const double plp = log_post(u.lc, pl, pm);
          if (exp(plp - u.cur) > uu) {  // bi:329-335
            u.ll = pl;
            u.lm = pm;
            u.cur = plp;
          }
        }
      }
    } else {
      // Software pipeline: the Philox blocks and t3 transforms of the next chunk of 4 MH steps
      // are independent of the state, so they are generated while the current chunk's fp64
      // accept/reject chain runs (ILP for the ~1.5 waves/SIMD of the CDNOW-sized problem).
      if (threadIdx.x == 0) CLV_WG_STAMP(a.stamps, (int64_t)c * g.nb_local + b, 5);
      mh_run(cu, SlotPhilox(k0, k1, cu.gi, (uint32_t)s), s00, s11, g.S, exp_tab);
    }
    if (threadIdx.x == 0) CLV_WG_STAMP(a.stamps, (int64_t)c * g.nb_local + b, 6);
    out = cust_finish<D, K, REPLAY>(cu, a, s, stored, H, k0, k1, tape, exp_tab, st);
  }

  block_reduce_gen<NS, SWEEP_REDUCE_CHUNK>(st, red, tot);
  if (threadIdx.x < NS)  // sc1 (write-through) store: read cross-CU by the fused tail
    __hip_atomic_store(a.blockpart + ((int64_t)c * g.stride + threadIdx.x) * g.blocks_per_rank + b, tot[threadIdx.x],
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // draws / summaries / state: the running sums' loads go out with the partial's store, so the
  // hand-off's drain below waits for both in one memory round trip; the sums' and draws' stores are
  // issued after the hand-off's ticket and never waited for (the tail never reads them).  Was: the
  // whole cust_store between the partial and the drain — two round trips per workgroup, +8.5% per
  // stored sweep at c4 / c5.
  const bool has_store = !a.init && cu.active;
  SumsPre<D> pre;
  const bool pre_sums = !REPLAY && has_store && stored && a.sums != nullptr;
  if (pre_sums) prefetch_sums<D>(a, c, cu.i, pre);
  auto finish_store = [&]() {
    if (has_store) cust_store<D, K>(cu, out, a, c, s, stored, true, pre_sums ? &pre : nullptr);
  };
  if (!a.fuse) finish_store();

  // ---- fused level-2 draw (world_size == 1): no separate hyper launch per sweep.  Two-level
  // hand-off: the last-arriving workgroup of each unit (blocks_per_unit consecutive blocks) sums
  // the unit's block partials in group_kernel's order; the last unit of the chain to complete
  // reduces all unit partials and draws (beta, Sigma).  Hand-off in the fence-free form of the
  // MI355X guide (Guideline 16 / "Valid forms"): partials and variates are stored sc1
  // (write-through), every wave drains its stores, one lane takes an agent-scope ticket; the
  // last arriver reads every handed-off value with sc1 loads (no L1 hit possible).
  if (a.fuse) {
    __shared__ uint32_t s_last;
    __shared__ double var_iw[4], var_chi[4], var_noise[32];
    __shared__ L2Scratch l2;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int bpu = g.blocks_per_unit;
    const double* units = a.blockpart;  // a unit is one block
    // fused peer exchange (world size > 1, clv_p2p_connect): every unit partial goes straight into
    // every rank's mail, [parity][rank][chain][unit][stat], system-scope write-through stores (the
    // value is its own arrival flag); the chain's last unit on this rank then waits in its own mail
    const bool fx = FX && g.world_size > 1;
    const int64_t mail_rank = (int64_t)g.n_chains * g.units_per_rank * NS;
    const int64_t mail_off = ((int64_t)(s & 1) * g.world_size + a.rank) * mail_rank + (int64_t)c * g.units_per_rank * NS;
    if (fx && bpu == 1 && threadIdx.x < NS) {
      const double v = tot[threadIdx.x];
      for (int q = 0; q < g.world_size; ++q) st_sys(a.peers[q] + mail_off + (int64_t)b * NS + threadIdx.x, v);
    }
    if (bpu > 1) {
      const int u = b / bpu;
      const int nbu = min(bpu, g.nb_local - u * bpu);  // blocks of this unit in the launch
      if (threadIdx.x == 0) {
        uint32_t* ctr = a.unit_arrive + (int64_t)c * g.units_per_rank + u;
        const uint32_t old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t last = old == (uint32_t)(nbu - 1) ? 1u : 0u;
        if (last) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = last;
      }
      __syncthreads();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only
      if (!s_last) {
        finish_store();
        return;
      }
      if (threadIdx.x < NS) {  // unit partial: sequential over the unit's blocks (= group_kernel)
        const double* p = a.blockpart + ((int64_t)c * g.stride + threadIdx.x) * g.blocks_per_rank + (int64_t)u * bpu;
        double t = 0.0;
        int bb = 0;
        for (; bb + 8 <= bpu; bb += 8) {  // batch the sc1 loads, add in order
          double v[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) v[q] = __hip_atomic_load(p + bb + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
          for (int q = 0; q < 8; ++q) t += v[q];
        }
        for (; bb < bpu; ++bb) t += __hip_atomic_load(p + bb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (fx) {
          for (int q = 0; q < g.world_size; ++q) st_sys(a.peers[q] + mail_off + (int64_t)u * NS + threadIdx.x, t);
        } else {
          __hip_atomic_store(a.unitpart + ((int64_t)c * g.stride + threadIdx.x) * g.units_per_rank + u, t,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      units = a.unitpart;
    }
    if (bpu > 1 || fx) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      CLV_STAMP(a.stamps, s, 1, false);
      CLV_STAMP(a.stamps, s, 4, true);
      CLV_WG_STAMP(a.stamps, (int64_t)c * g.nb_local + b, 1);
      CLV_WG_STAMP(a.stamps, (int64_t)c * g.nb_local + b, 7);
      const uint32_t n_arrivals = (uint32_t)((g.nb_local + bpu - 1) / bpu);  // units in the launch
      const uint32_t old = __hip_atomic_fetch_add(a.chain_arrive + c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t last = old == n_arrivals - 1 ? 1u : 0u;
      if (last) __hip_atomic_store(a.chain_arrive + c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = last;
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only
    // (storing after the chain's last unit's level-2 draw instead, so that the draw's loads do not
    // wait for these stores in vmcnt order, measured 0.5-1.2 us per sweep slower at c4, round 4)
    finish_store();
    if (s_last) {
      if (threadIdx.x == 0) CLV_STAMP(a.stamps, s, 2, false);
      if (!fx) {
        hyper_body<D, K, REPLAY, NS, NT>(a.h, c, s, 0, units, red, tot, var_iw, var_chi, var_noise, &l2);
      } else {
        hyper_variates<D, K, REPLAY>(a.h, c, s, var_iw, var_chi, var_noise, &l2);
        // every rank's units of sweep s from this rank's mail: lane u reads units u, u + NT
        // (n_units_global <= 2 NT) and sums them in that order — hyper_sum_units' order, so the
        // result is the all-gather path's bit for bit; then it empties its slots for sweep s + 2
        const int64_t u0 = threadIdx.x, u1 = threadIdx.x + NT;
        const bool h0 = u0 < g.n_units_global, h1 = u1 < g.n_units_global;
        const double* mb = a.mail + (int64_t)(s & 1) * g.world_size * mail_rank + (int64_t)c * g.units_per_rank * NS;
        double* p0 = (double*)mb + (u0 / g.units_per_rank) * mail_rank + (u0 % g.units_per_rank) * NS;
        double* p1 = (double*)mb + (u1 / g.units_per_rank) * mail_rank + (u1 % g.units_per_rank) * NS;
        const double* q0 = h0 ? p0 : mb;
        const double* q1 = h1 ? p1 : mb;
        __shared__ uint32_t s_fx_abort;
        if (threadIdx.x == 0) {
          s_fx_abort = 0;
          post_progress(a, a.peers, s);
        }
        __syncthreads();
        // statistics in chunks of FXC (all NS at once for small NS): the polled values of a chunk
        // and the lane's finished sums are live together, not 2 NS polled values (c5: NS = 34)
        constexpr int FXC = NS <= 16 ? NS : 12;
        double acc[NS];
        bool timed_out = false;
#pragma unroll
        for (int j0 = 0; j0 < NS; j0 += FXC) {
          double v0[FXC], v1[FXC];
          const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
          for (uint32_t poll = 0; !timed_out; ++poll) {
            bool ok = true;
#pragma unroll
            for (int q = 0; q < FXC; ++q) {
              if (j0 + q < NS) {
                v0[q] = ld_sys(q0 + j0 + q);
                v1[q] = ld_sys(q1 + j0 + q);
                ok = ok & (!h0 | slot_full(v0[q])) & (!h1 | slot_full(v1[q]));
              }
            }
            if (__all(ok)) break;
            const int ws = wait_state(a, t0, poll, a.wait_ticks);
            if (ws == WAIT_OBSERVED) {
              timed_out = true;
            } else if (ws == WAIT_EXPIRED) {
              timed_out = true;
              int64_t mu_ = -1;
              int mj = -1;
              uint64_t mb = 0;
#pragma unroll
              for (int q = FXC - 1; q >= 0; --q) {  // the lane's first missing slot
                if (j0 + q < NS) {
                  if (h1 && !slot_full(v1[q])) { mu_ = u1; mj = j0 + q; mb = dbits(v1[q]); }
                  if (h0 && !slot_full(v0[q])) { mu_ = u0; mj = j0 + q; mb = dbits(v0[q]); }
                }
              }
              report_wait(a, WAIT_FX_MAIL, s, c, ok, mu_, mj, mb, poll, t0);
              raise_abort(a);
            } else {
              __builtin_amdgcn_s_sleep(1);
            }
          }
#pragma unroll
          for (int q = 0; q < FXC; ++q) {
            if (j0 + q < NS) {
              acc[j0 + q] = 0.0;
              if (h0) acc[j0 + q] += v0[q];
              if (h1) acc[j0 + q] += v1[q];
            }
          }
        }
        if (timed_out) s_fx_abort = 1;
        __syncthreads();
        if (!s_fx_abort) {
          // the slots of sweep s empty again for sweep s + 2 (written only after the next kernel
          // boundary): every rank's [unit][stat] run of this (parity, chain), coalesced, by
          // wavefronts 1-3 while wavefront 0 draws — lane-per-unit resets wrote one double of a
          // different line per lane and instruction ahead of the draw (c5 at 8 ranks: 306 units x
          // 34 statistics; round 6, as the persistent kernel's slots)
          const int nrun = g.units_per_rank * NS;
          hyper_finish<D, K, REPLAY, NS, NT>(a.h, c, s, 0, acc, red, tot, var_iw, var_chi, var_noise, &l2, [&] {
            for (int e = (int)threadIdx.x - 64; e >= 0 && e < g.world_size * nrun; e += NT - 64) {
              const int q = e / nrun;
              st_sys((double*)mb + (int64_t)q * mail_rank + (e - q * nrun), slot_empty());
            }
          });
        }
      }
      if (threadIdx.x == 0) CLV_STAMP(a.stamps, s, 3, false);
    }
  }
}


// The sweep kernel at two occupancy targets (an attribute cannot depend on template arguments
// here): see SweepOcc.
template <int D, int K, bool REPLAY, bool FX>
__global__ __launch_bounds__(BLOCK) void sweep_kernel(SweepArgs a) {
  sweep_body<D, K, REPLAY, FX>(a);
}
template <int D, int K, bool REPLAY, bool FX>
__global__ __launch_bounds__(BLOCK, 4) void sweep_kernel_occ4(SweepArgs a) {
  sweep_body<D, K, REPLAY, FX>(a);
}

// One instance per (D, K, REPLAY, FX): the occupancy variant SweepOcc picks (only that one compiled).
template <int D, int K, bool REPLAY, bool FX>
hipError_t launch_sweep_t(const SweepArgs& a, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  const dim3 grid(a.g.nb_local, a.g.n_chains);
  const dim3 block(BLOCK);
  // e0/e1: hipExtLaunchKernelGGL records the dispatch's own start/end timestamps into the events
  // (no extra marker packets in the stream, unlike hipEventRecord around the launch).
  if constexpr (SweepOcc<D, K>::value >= 4) {
    if (e0) hipExtLaunchKernelGGL((sweep_kernel_occ4<D, K, REPLAY, FX>), grid, block, 0, st, e0, e1, 0, a);
    else hipLaunchKernelGGL((sweep_kernel_occ4<D, K, REPLAY, FX>), grid, block, 0, st, a);
  } else {
    if (e0) hipExtLaunchKernelGGL((sweep_kernel<D, K, REPLAY, FX>), grid, block, 0, st, e0, e1, 0, a);
    else hipLaunchKernelGGL((sweep_kernel<D, K, REPLAY, FX>), grid, block, 0, st, a);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Persistent sweep kernel (world size 1, Philox mode): one launch runs n_sweeps sweeps.  Grid
// (nb_local + 1, chains), every workgroup resident at once (checked at create).  Per chain,
// workgroups 0..nb_local-1 own 256 customers each and keep them in registers for the whole
// launch; workgroup nb_local is the chain's level-2 workgroup.  Per sweep s:
//   customers:  wait for (beta, Sigma) of sweep s -> log-posterior constants -> MH -> state,
//               statistics -> block partial (write-through store) -> draws -> z / tau of s+1
//   level 2:    variates of the next draw -> wait for all block partials of s -> the fused
//               path's fixed-order sum -> level-2 draw -> (beta, Sigma) of s+1 published
// Hand-off without counters or flags: slots are reset to a sentinel (an all-ones NaN, a pattern
// fp64 arithmetic never produces) and a reader polls (write-through loads) until none of its
// slots holds the sentinel.  Block partials: one slot set per chain, reset by the level-2
// workgroup after reading, before it publishes the next (beta, Sigma) — and writers write only
// after seeing that.  (beta, Sigma): two slot sets by sweep parity; set s&1 is reset (after all
// readers of s have delivered their partials) before the set of s+1 is written, so a reader of
// s+2 sees the reset or newer.  Sums are formed in the fused path's order: results are bitwise
// identical to the launch-per-sweep path.  Every wait is bounded (SweepArgs::wait_ticks, 2 s by
// default): a wave that times out raises ctrl->abort (and the host-mapped copy the host reads after
// the launch) and every wave leaves at its next wait.  The carried state (lambda, mu, hyper) is
// written to the *_out buffers, which the host adopts only when no wave aborted: an aborted launch
// leaves the state it started from untouched.
// ---------------------------------------------------------------------------------------------
// The chain's level-2 workgroup of persist_kernel (one per chain, grid column nb_local).
// register arrays (block/unit partials of the chain) do not raise the customer path's pressure.
template <int D, int K, bool P2P>
__device__ __forceinline__ void persist_level2(const SweepArgs& a, int64_t s_first, int64_t n_sweeps, int c, uint32_t k0,
                                            uint32_t k1, int64_t wgi, int64_t it_stamp, double* pool) {
  constexpr int NT = BLOCK;
  constexpr int NXY = K * D;
  constexpr int NYY = D * (D + 1) / 2;
  constexpr int NS = NXY + NYY + 1;
  constexpr int NTRIL = D * (D - 1) / 2;
  (void)NXY;
  __shared__ double red[BLOCK / 64][NS];
  __shared__ double tot[NS];
  __shared__ double Hs[HS];
  __shared__ uint32_t s_abort;
  __shared__ double var_iw[4], var_chi[4], var_noise[32];
  __shared__ L2Scratch l2;
  __shared__ double* s_peers[P2P ? MAX_WORLD : 1];  // every rank's mail (loaded once)
  const Geometry& g = a.g;
  const int tid0 = threadIdx.x;
  (void)wgi;
  double* parts0 = a.pblock + (int64_t)c * g.nb_local * NS;  // [block][stat]
  if (tid0 == 0) s_abort = 0;
  if constexpr (P2P) {
    if (tid0 < g.world_size) s_peers[tid0] = a.peers[tid0];
  }
  __syncthreads();
  // ================= the chain's level-2 workgroup =================
  // It shares its CU with customer workgroups; it is on every sweep's critical path, so its
  // waves take issue priority over theirs (it mostly sleeps in polls otherwise).
  __builtin_amdgcn_s_setprio(3);
  stage_prior(a.h.V, &l2);
  // deferred draws (world size 1): pin = the statistics of sweep s_first - 1 whose draw the
  // previous launch left to this one (iteration -1: no poll, drawn while the customer workgroups
  // load and draw their first variates); pout = where the last sweep's statistics go instead of
  // being drawn from (the next launch's, or a flush's, iteration -1)
  const double* pin = P2P ? nullptr : a.pend_in;
  double* pout = P2P ? nullptr : a.pend_out;
  ClockMark clk_prev = CLV_CLOCK_RECORD && a.clk && c == 0 ? ClockMark::now() : ClockMark{0, 0};  // per-sweep intervals
  for (int64_t it = pin ? -1 : 0; it < n_sweeps; ++it) {
    // the lane's addresses and unit bookkeeping are recomputed every sweep from an opaque copy of
    // the lane index (a few integer ops), not kept live across the loop: registers for the phases
    int tid = tid0;
    double* parts = parts0;
    if constexpr (CLV_L2_OPAQUE(P2P)) {
      asm volatile("" : "+v"(tid));
      asm volatile("" : "+s"(parts));
    }
    const int64_t s = s_first + it;
    const bool stp = tid == 0 && it == it_stamp;
    (void)stp;
    const int64_t hs = (D == 2) ? s + 1 : s;  // sweep the drawn (beta, Sigma) belongs to
    const bool from_pend = it < 0;                           // (uniform)
    const bool defer_now = pout && it == n_sweeps - 1;       // (uniform) this sweep's draw is deferred
    CLV_P_STAMP(a.stamps, wgi, 0, stp);
    // 1. this draw's variates (as hyper_body without precomputed ones): overlap the sweep
    if (!defer_now) {
      if (tid < NTRIL) var_iw[tid] = hyper_normal(k0, k1, HSLOT_NORMAL0 + tid, (uint32_t)hs);
      if (tid >= 32 && tid < 32 + D * K) var_noise[tid - 32] = hyper_normal(k0, k1, HSLOT_BETA_NORMAL0 + (tid - 32), (uint32_t)hs);
      if (tid >= 64 && tid < 64 + D) var_chi[tid - 64] = chi2_draw(k0, k1, (uint32_t)hs, tid - 64, a.h.nu_n - D + 1 + (tid - 64));
    }
    if (from_pend && tid < NS) tot[tid] = pin[(int64_t)c * NS + tid];  // the fixed-order sums, as stored
    __syncthreads();
    if (!defer_now && tid == 0) bartlett_inverse<D>(var_iw, var_chi, l2.Ai);  // read back by this lane only
    CLV_P_STAMP(a.stamps, wgi, 1, stp);
    if (!from_pend) {
    // 2. wait for every block partial of sweep s (lane tid: blocks tid, tid + NT; nb <= 2 NT).
    //    The persistent kernel's partials are [block][stat]: one base address per block and the
    //    statistics at immediate offsets (no per-statistic 64-bit addresses held across the poll).
    double v0[NS], v1[NS];
    const int b0 = tid, b1 = tid + NT;
    const bool hb0 = b0 < g.nb_local, hb1 = b1 < g.nb_local;
    double* pb0 = parts + (int64_t)b0 * NS;
    double* pb1 = parts + (int64_t)b1 * NS;
    // polled unconditionally (no branch per load): lanes without a block / unit read block 0 /
    // their own first mail slot and discard it
    const double* qb0 = hb0 ? pb0 : parts;
    const double* qb1 = hb1 ? pb1 : parts;
    // P2P: the global units this lane sums (u0, u1: as hyper_body, n_units_global <= 2 NT) and
    // where they come from — another rank's (the mail, [unit][stat]) or this rank's own (LDS, below)
    const int64_t per_rank = (int64_t)g.n_chains * NS * g.units_per_rank;  // mail doubles per rank and parity
    const double* mb = a.mail + (int64_t)(s & 1) * g.world_size * per_rank + (int64_t)c * NS * g.units_per_rank;
    const int64_t u0 = tid, u1 = tid + NT;
    const int r0 = (int)(u0 / g.units_per_rank), r1 = (int)(u1 / g.units_per_rank);
    const int l0 = (int)(u0 % g.units_per_rank), l1 = (int)(u1 % g.units_per_rank);
    const double* p0 = mb + r0 * per_rank + (int64_t)l0 * NS;
    const double* p1 = mb + r1 * per_rank + (int64_t)l1 * NS;
    const bool h0 = u0 < g.n_units_global, h1 = u1 < g.n_units_global;
    const bool m0 = P2P && h0 && r0 != a.rank, m1 = P2P && h1 && r1 != a.rank;
    const double* q0 = m0 ? p0 : mb;
    const double* q1 = m1 ? p1 : mb;
    double w0[NS], w1[NS];
    bool mdone = !(m0 || m1);  // this lane's mail slots all full (or none to read)
    if constexpr (P2P) {
      if (tid == 0) post_progress(a, s_peers, s);
    }
    // one bound for the whole wait for sweep s's statistics, local partials and peer mail together,
    // counted from its start: it then expires before the customer workgroups' wait for the (beta,
    // Sigma) this draw would publish (which starts only after their partials), so the record names
    // the missing peer unit rather than the slot that waited on it
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    {  // each wavefront polls on its own (no barrier per poll); a lane stops once its slots are full.
       // P2P: the mail is polled alongside (the other ranks' units of the last rank to finish are
       // then already in registers when its own partials are complete)
      bool done = false;
      for (uint32_t poll = 0;; ++poll) {
        if (!done) {
          bool ok = true;
#pragma unroll
          for (int j = 0; j < NS; ++j) {
            v0[j] = ld_wt(qb0 + j);
            v1[j] = ld_wt(qb1 + j);
          }
#pragma unroll
          for (int j = 0; j < NS; ++j) ok = ok & (!hb0 | slot_full(v0[j])) & (!hb1 | slot_full(v1[j]));
          done = ok;
        }
        if constexpr (P2P) {
          if (!mdone) {
            bool ok = true;
#pragma unroll
            for (int j = 0; j < NS; ++j) {
              w0[j] = ld_sys(q0 + j);
              w1[j] = ld_sys(q1 + j);
            }
#pragma unroll
            for (int j = 0; j < NS; ++j) ok = ok & (!m0 | slot_full(w0[j])) & (!m1 | slot_full(w1[j]));
            mdone = ok;
          }
        }
        if (__all(done)) break;
        const int ws = wait_state(a, t0, poll, a.wait_ticks);
        if (ws == WAIT_OBSERVED) {
          s_abort = 1;
          break;
        }
        if (ws == WAIT_EXPIRED) {
          int64_t mb_ = -1;
          int mj = -1;
          uint64_t mbits = 0;
#pragma unroll
          for (int j = NS - 1; j >= 0; --j) {  // the lane's first missing block partial
            if (hb1 && !slot_full(v1[j])) { mb_ = b1; mj = j; mbits = dbits(v1[j]); }
            if (hb0 && !slot_full(v0[j])) { mb_ = b0; mj = j; mbits = dbits(v0[j]); }
          }
          report_wait(a, WAIT_BLOCKS, s, c, done, mb_, mj, mbits, poll, t0);
          raise_abort(a);
          s_abort = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
    if (s_abort) return;
#pragma unroll
    for (int j = 0; j < NS; ++j) {  // padding blocks contribute 0.0 (group_kernel's zero padding)
      v0[j] = hb0 ? v0[j] : 0.0;
      v1[j] = hb1 ? v1[j] : 0.0;
    }
    CLV_P_STAMP(a.stamps, wgi, 2, stp);
    // 3. the fused path's fixed-order sum (hyper_body: lane u sums units u, u + NT, ... in order)
    double acc[NS];
    if constexpr (!P2P) {
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        acc[j] = 0.0;
        if (hb0) acc[j] += v0[j];
        if (hb1) acc[j] += v1[j];
      }
    } else {
      double* umail = pool;  // [UMAIL]: this rank's unit partials [local unit][stat] (the pool the
                             // customer workgroups use for their drawn-ahead MH variates)
      // 3a. this rank's unit partials: blocks_per_unit consecutive blocks summed in group_kernel's
      //     order (a unit's blocks sit in consecutive lanes of one wavefront: bpu | 64); with one
      //     block per unit the unit partial IS the block partial (the sharded path has no group
      //     kernel then).  One half (blocks tid / tid + NT) at a time: fewer live registers.
      const int bpu = g.blocks_per_unit;
      const int ul = (g.nb_local + bpu - 1) / bpu;
      const int lane = tid & 63;
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const double* v = half ? v1 : v0;
        const int ub = (tid + half * NT) / bpu;  // this lane's local unit (if it leads one)
        double t[NS];
        if (bpu == 1) {
#pragma unroll
          for (int j = 0; j < NS; ++j) t[j] = v[j];
        } else {
#pragma unroll
          for (int j = 0; j < NS; ++j) t[j] = 0.0 + v[j];
          for (int k = 1; k < bpu; ++k) {  // all statistics' shuffles of one k in flight together
#pragma unroll
            for (int j = 0; j < NS; ++j) t[j] += __shfl(v[j], lane + k, 64);  // blocks >= nb_local
          }                                                                  // add 0.0, as
        }                                                                    // group_kernel's padding
        if (tid % bpu == 0 && ub < ul) {
#pragma unroll
          for (int j = 0; j < NS; ++j) umail[ub * NS + j] = t[j];
        }
      }
      lds_barrier();
      CLV_P_STAMP(a.stamps, wgi, 10, stp);
      // 3b. to every OTHER rank's mail slot of sweep s (write-through stores over xGMI; the value
      //     is its own arrival flag — the sentinel never occurs in a partial); own units stay in
      //     LDS.  [unit][stat] on both sides: consecutive lanes store consecutive doubles.
      const int64_t dst = ((int64_t)(s & 1) * g.world_size + a.rank) * per_rank + (int64_t)c * NS * g.units_per_rank;
      for (int e = tid; e < NS * ul; e += NT) {
        const double v = umail[e];
        for (int q = 0; q < g.world_size; ++q)
          if (q != a.rank) st_sys(s_peers[q] + dst + e, v);
      }
      // 3c. the other ranks' units not seen yet (the bound runs from t0, above)
      const uint64_t tw = t0;
      for (uint32_t poll = 0; !__all(mdone); ++poll) {
        if (!mdone) {
          bool ok = true;
#pragma unroll
          for (int j = 0; j < NS; ++j) {
            w0[j] = ld_sys(q0 + j);
            w1[j] = ld_sys(q1 + j);
          }
#pragma unroll
          for (int j = 0; j < NS; ++j) ok = ok & (!m0 | slot_full(w0[j])) & (!m1 | slot_full(w1[j]));
          mdone = ok;
        }
        if (__all(mdone)) break;
        const int ws = wait_state(a, tw, poll, a.wait_ticks);
        if (ws == WAIT_OBSERVED) {
          s_abort = 1;
          break;
        }
        if (ws == WAIT_EXPIRED) {
          int64_t mu_ = -1;
          int mj = -1;
          uint64_t mbits = 0;
#pragma unroll
          for (int j = NS - 1; j >= 0; --j) {  // the lane's first missing unit partial
            if (m1 && !slot_full(w1[j])) { mu_ = u1; mj = j; mbits = dbits(w1[j]); }
            if (m0 && !slot_full(w0[j])) { mu_ = u0; mj = j; mbits = dbits(w0[j]); }
          }
          report_wait(a, WAIT_P2P_MAIL, s, c, mdone, mu_, mj, mbits, poll, tw);
          raise_abort(a);
          s_abort = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      CLV_P_STAMP(a.stamps, wgi, 11, stp);
      lds_barrier();  // (the stores to the peers stay in flight)
      if (s_abort) return;
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        const double x0 = m0 ? w0[j] : (h0 ? umail[l0 * NS + j] : 0.0);
        const double x1 = m1 ? w1[j] : (h1 ? umail[l1 * NS + j] : 0.0);
        acc[j] = 0.0;
        if (h0) acc[j] += x0;
        if (h1) acc[j] += x1;
      }
    }
    block_reduce<NS, NT, P2P>(acc, red, tot);  // also publishes the variates (LDS)
    CLV_P_STAMP(a.stamps, wgi, 6, stp);
    // 4. reset: the partial slots (their writers write again only after step 6) and the
    //    (beta, Sigma) set every reader of s has read (its next write is for s+2; at sweep s_first
    //    of a launch that drew a deferred draw first, its readers took it from this slot too)
    //    Coalesced: consecutive lanes empty consecutive doubles of the chain's [block][stat] slots
    //    (round 6).  Lane-per-block resets (lane b: its block's NS doubles) wrote one double of a
    //    different line per lane and instruction — c4's 8-rank shard (496 blocks x 14 statistics)
    //    queued ~7k partial-line write-throughs ahead of the draw on this wave: 8.2 us of a 20 us
    //    sweep (profiles/r06_c4shard8_stamps_*.txt).  Issued by wavefronts 1-3 only, while wavefront 0
    //    runs the draw (step 5): its instructions queue behind none of them (the vmcnt(0) before
    //    the publish waits for them all).
    const int rt = tid - 64;  // (< 0: wavefront 0)
    if (rt >= 0) {
      const int nrec = g.nb_local * NS;
      for (int e = rt; e < nrec; e += NT - 64) st_wt(parts + e, slot_empty());
      if ((it > 0 || pin) && rt < HS) st_wt(a.hyp2 + ((int64_t)(s & 1) * g.n_chains + c) * HS + rt, slot_empty());
    }
    if constexpr (P2P) {  // this rank's mail slots of sweep s: empty again before any rank can
                          // write sweep s + 2 there (only after this rank's units of s + 1, which
                          // leave after the vmcnt(0) below); every other rank's [unit][stat] run of
                          // this (parity, chain), coalesced like the block slots
      const int nrun = g.units_per_rank * NS;
      for (int e = rt; rt >= 0 && e < g.world_size * nrun; e += NT - 64) {
        const int q = e / nrun;
        if (q != a.rank) st_sys((double*)mb + (int64_t)q * per_rank + (e - q * nrun), slot_empty());
      }
    }
    }  // (!from_pend)
    if (defer_now) {  // the last sweep's statistics to the next launch (kernel boundary: plain
                      // stores), its log-likelihood record now; the slots above are empty again
      if (tid < NS) pout[(int64_t)c * NS + tid] = tot[tid];
      if (tid == 0) {
        if (is_stored(s, g)) a.h.loglik[(int64_t)c * g.n_draws + draw_index(s, g)] = tot[NS - 1] / (double)g.n_global;
        a.ctrl_rw->cur = s;
      }
      return;
    }
    if (tid < HS) Hs[tid] = 0.0;  // unwritten hyper slots publish as 0 (wavefront 0: ordered before the draw's writes)
    // 5. the draw (wavefront 0) while the resets drain
    // P2P: the one-lane form only for the smallest K*D (its registers, added to the exchange's,
    // spilled the peer kernel at K*D = 10); the element-parallel form gives the same bits
    level2_draw<D, K, P2P ? 6 : CLV_L2_LANE0_MAX>(tot, var_iw, var_chi, var_noise, false, &l2, l2.Ai);
    CLV_P_STAMP(a.stamps, wgi, 7, stp);
    if (tid == 0) {
      double Sig[D][D];
#pragma unroll
      for (int p = 0; p < D; ++p)
#pragma unroll
        for (int q = 0; q < D; ++q) Sig[p][q] = l2.Sig[p * D + q];
      finalize_hyper<D, K, true, CLV_L2_NR != 0>(l2.beta, Sig, a.h.omega2, Hs);
    }
    CLV_P_STAMP(a.stamps, wgi, 3, stp);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // resets landed (each wave its own)
    __syncthreads();
    // 6. publish (beta, Sigma) of sweep s+1: one coalesced write-through store per lane
    const bool last = it == n_sweeps - 1;
    if (tid < HS) {
      if (last) a.hyper_out[(int64_t)c * HS + tid] = Hs[tid];  // the carried state (kernel boundary)
      else st_wt(a.hyp2 + ((int64_t)((s + 1) & 1) * g.n_chains + c) * HS + tid, Hs[tid]);
    }
    CLV_P_STAMP(a.stamps, wgi, 4, stp);
    CLV_P_STAMP(a.stamps, wgi, 5, tid == 0 && it + 1 == it_stamp);  // the previous sweep's publish
    if (CLV_CLOCK_RECORD && a.clk && c == 0 && tid == 0) clk_prev = clock_mark(a.clk, s, clk_prev);
#ifdef CLV_STAMPS
    if (tid == 0 && a.stamps && c < 8 && it % 4 == 0 && it / 4 < 1024)  // publish times, every 4th sweep
      a.stamps[(it / 4) * 8 + c] = __builtin_amdgcn_s_memrealtime();
#endif
    // 7. records (off the critical path)
    const bool store_l2 = hs >= 1 && is_stored(hs, g);
    double* o = store_l2 ? a.h.level2 + ((int64_t)c * g.n_draws + draw_index(hs, g)) * g.l2w : nullptr;
    if (tid < K * D && store_l2) o[(tid % D) * K + tid / D] = l2.beta[tid];  // beta.T.ravel() (bi:411)
    if (tid == 0) {
      if (store_l2) {
        int q = K * D;
#pragma unroll
        for (int p = 0; p < D; ++p)
#pragma unroll
          for (int r = p; r < D; ++r) o[q++] = l2.Sig[p * D + r];  // bi:412, tri:550-554
      }
      // (a deferred draw's log-likelihood record was written by the launch that deferred it)
      if (!from_pend && is_stored(s, g)) a.h.loglik[(int64_t)c * g.n_draws + draw_index(s, g)] = tot[NS - 1] / (double)g.n_global;
      if (last) a.ctrl_rw->cur = s;
    }
    __syncthreads();  // LDS (tot, l2, Hs, variates) reused next sweep
  }
  return;
}

// The kernel arguments re-read from the kernarg segment through an opaque pointer: in a loop over
// tasks the compiler otherwise loads every argument once at entry and keeps them all live in SGPRs
// (hundreds of SGPR spills into VGPR lanes), instead of scalar loads where they are used.
__device__ __forceinline__ const SweepArgs& kernargs_fresh() {
  auto p4 = (const __attribute__((address_space(4))) SweepArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p4));
  return *(const SweepArgs*)p4;
}

#ifndef CLV_PERSIST_FRESH_ARGS
#define CLV_PERSIST_FRESH_ARGS 1
#endif
template <bool FRESH>
__device__ __forceinline__ const SweepArgs& loop_args(const SweepArgs& a) {
  if constexpr (FRESH) return kernargs_fresh();
  else return a;
}

// P2P: world size > 1 with the peer exchange (a separate instance, so that the world-size-1
// kernel carries none of its registers or LDS).
template <int D, int K, bool P2P>
__global__ __launch_bounds__(BLOCK, 2) void persist_kernel(SweepArgs a, int64_t s_first, int64_t n_sweeps) {
  constexpr int NXY = K * D;
  constexpr int NYY = D * (D + 1) / 2;
  constexpr int NS = NXY + NYY + 1;
  __shared__ double red[BLOCK / 64][NS];
  __shared__ double tot[NS];
  __shared__ __attribute__((aligned(16))) double exp_tab[D == 3 ? FAST_TAB_N3 : FAST_TAB_N];
  __shared__ double Hs[HS];
  __shared__ uint32_t s_abort;
  // customer workgroups: the drawn-ahead MH variates; the level-2 workgroup (P2P): its unit partials
  __shared__ __attribute__((aligned(16))) char pool[PRE_LDS_BYTES];
  static_assert(UMAIL * sizeof(double) <= PRE_LDS_BYTES, "the level-2 unit partials share the variates' LDS");
  __shared__ double zeta_lds[D == 3 ? BLOCK : 1];  // draw_eta's normal of the next sweep (trivariate)
  const Geometry& g = a.g;
  int c = blockIdx.y, b = blockIdx.x;
  if (a.wg_map) {  // placement (capi.hip persist_wg_map): same-chain workgroups share CUs
    const int32_t m = a.wg_map[blockIdx.y * gridDim.x + blockIdx.x];
    c = m >> 16;
    b = m & 0xFFFF;
  }
  const int tid = threadIdx.x;
  const int64_t wgi = (int64_t)c * (g.nb_local + 1) + b;
  const int64_t it_stamp = n_sweeps >= 2 ? n_sweeps - 2 : 0;  // diagnostic build: one sweep's timeline
  (void)wgi;
  (void)it_stamp;
  uint32_t k0, k1;
  chain_key(a.r.seed, (int64_t)a.r.chain_first + c, &k0, &k1);
  double* parts = a.pblock + (int64_t)c * g.nb_local * NS;  // [block][stat]
  if (tid == 0) s_abort = 0;

  if (b == g.nb_local) {  // the chain's level-2 workgroup
    persist_level2<D, K, P2P>(a, s_first, n_sweeps, c, k0, k1, wgi, it_stamp, (double*)pool);
    return;
  }

  // ================= customer workgroups =================
  CLV_P_STAMP(a.stamps, wgi, 7, tid == 0);  // (diagnostic build) this workgroup's first instruction
  Cust<D, K> cu;
  {
    const int64_t i = (int64_t)b * BLOCK + tid;
    cu.active = i < g.n;
    cu.i = cu.active ? i : (g.n > 0 ? g.n - 1 : 0);
  }
  cust_load(cu, a, c);  // once per launch: CBS row, covariates, state stay in registers
  fast_tab_fill(exp_tab, tid, BLOCK, D == 3);
  if (tid < HS) Hs[tid] = a.hyper[(int64_t)c * HS + tid];  // sweep s_first: from before this launch
  __syncthreads();
  if (cu.active) cust_ztau<D, K, false>(cu, a, s_first, k0, k1, nullptr, exp_tab);
  // MH variates drawn ahead (while the wave waits for the level-2 draw) when S fits the LDS pool
  const bool pre = g.S <= PRE_STEPS;
  const PreVariates pv{(float2*)pool, (float*)(pool + PRE_STEPS * BLOCK * 8), tid};
  if (cu.active && pre) mh_pre_variates(SlotPhilox(k0, k1, cu.gi, (uint32_t)s_first), g.S, pv);
  if constexpr (D == 3) {
    if (cu.active && pre) zeta_lds[tid] = eta_normal(k0, k1, cu.gi, s_first, exp_tab);
  }
  CLV_P_STAMP(a.stamps, wgi, 10, tid == 0);  // (diagnostic build) prologue done
  const SweepArgs& a_launch = a;
  for (int64_t it = 0; it < n_sweeps; ++it) {
    // bivariate: the arguments re-read through an opaque kernarg pointer each sweep (scalar loads
    // where they are used) instead of held across the loop in SGPRs spilled to VGPR lanes (c2: 140
    // -> 101 SGPR spills, 10.79 -> 10.72 us per sweep; c3 measured 12.56 -> 12.63, so not there)
    const SweepArgs& a = loop_args<CLV_PERSIST_FRESH_ARGS && D == 2>(a_launch);
    const Geometry& g = a.g;
    const double* hyp_c = a.hyp2 + (int64_t)c * HS;
    // Philox products of the customer counter word are the same every sweep; hoisted out of the
    // loop they were kept live (and spilled, tri K=3) — recomputed per sweep instead (a few VALU)
    if constexpr (CLV_OPAQUE_GI(D)) asm volatile("" : "+v"(cu.gi));
    const int64_t s = uniform64(s_first + it);  // scalar registers: the sweep's address and index arithmetic on the scalar unit
    const bool stored = is_stored(s, g);
    const bool stp = tid == 0 && it == it_stamp;
    (void)stp;
    CLV_P_STAMP(a.stamps, wgi, 0, stp);
    if (it > 0 || (!P2P && a.pend_in)) {  // wait for (beta, Sigma) of sweep s (wavefront 0 polls, one slot per lane)
      if (tid < 64) {
        const double* src = hyp_c + (int64_t)(s & 1) * g.n_chains * HS;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (uint32_t poll = 0;; ++poll) {
          const double v = ld_wt(src + tid);
          if (__all(slot_full(v))) {
            Hs[tid] = v;
            break;
          }
          const int ws = wait_state(a, t0, poll, hyper_wait_ticks(a));
          if (ws != WAIT_GOING) {
            if (ws == WAIT_EXPIRED) {
              report_wait(a, WAIT_HYPER, s, c, slot_full(v), b, tid, dbits(v), poll, t0);
              raise_abort(a);
            }
            if (tid == 0) s_abort = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      __syncthreads();
      if (s_abort) return;
    }
    CLV_P_STAMP(a.stamps, wgi, 1, stp);
    StatGen<D, K> st{};
    CustOut<D> out{};
    // Wave priority by phase (round 5): from (beta, Sigma) of sweep s to its block partial a customer
    // wave is on the chain's critical path (the level-2 draw waits for the last partial), after it
    // the wave only draws ahead for sweep s + 1.  A SIMD holding two customer waves (c2: 464 of
    // 1,024) used to split its issue between one wave's MH phase and the other's drawing ahead by
    // age; the critical phase now goes first (the level-2 workgroup keeps priority 3):
    // c2 10.62 -> 9.58 us per sweep, c3 12.37 -> 11.1 (tools/ab_env.sh, profiles/r05_ab_priority.txt).
    __builtin_amdgcn_s_setprio(2);
    if (cu.active) {
      cust_coeffs<D, K, false>(cu, Hs, exp_tab);
      CLV_P_STAMP(a.stamps, wgi, 2, stp);
      const double s00 = Hs[H_S00];
      const double s11 = Hs[H_S11];
      if (pre) mh_run_pre(cu, pv, s00, s11, g.S, exp_tab);
      else mh_run(cu, SlotPhilox(k0, k1, cu.gi, (uint32_t)s), s00, s11, g.S, exp_tab);
      CLV_P_STAMP(a.stamps, wgi, 3, stp);
      if constexpr (D == 3) {
        if (!pre) zeta_lds[tid] = eta_normal(k0, k1, cu.gi, s, exp_tab);  // (not drawn ahead: S > PRE_STEPS)
      }
      out = cust_finish<D, K, false>(cu, a, s, stored, Hs, k0, k1, nullptr, exp_tab, st,
                                     D == 3 ? &zeta_lds[tid] : nullptr);
    }
    CLV_P_STAMP(a.stamps, wgi, 4, stp);
#if PERSIST_REDUCE_GEN
    block_reduce_gen<NS, SWEEP_REDUCE_CHUNK>(st, red, tot);
#else
    {
      double acc[NS];
#pragma unroll
      for (int j = 0; j < NS; ++j) acc[j] = st(j);
      block_reduce<NS>(acc, red, tot);
    }
#endif
    if (tid < NS) st_wt(parts + (int64_t)b * NS + tid, tot[tid]);  // one contiguous 8*NS-byte record
    __builtin_amdgcn_s_setprio(0);  // drawing ahead for the next sweep: yield the SIMD
    CLV_P_STAMP(a.stamps, wgi, 5, stp);
    CLV_P_STAMP(a.stamps, wgi, 8, stp);
    CLV_P_STAMP(a.stamps, wgi, 9, stp);
#ifdef CLV_STAMPS
    if (stp && a.stamps) a.stamps[1024 * 8 + wgi * 12 + 11] = blockIdx.y * gridDim.x + blockIdx.x;  // dispatch position
#endif
    if (cu.active) {
      cust_store<D, K>(cu, out, a, c, s, stored, false);
      if (it + 1 < n_sweeps) {
        cust_ztau<D, K, false>(cu, a, s + 1, k0, k1, nullptr, exp_tab);
        if (pre) mh_pre_variates(SlotPhilox(k0, k1, cu.gi, (uint32_t)(s + 1)), g.S, pv);
        if constexpr (D == 3) {
          if (pre) zeta_lds[tid] = eta_normal(k0, k1, cu.gi, s + 1, exp_tab);
        }
      }
    }
    CLV_P_STAMP(a.stamps, wgi, 6, stp);
  }
  if (cu.active) {  // the carried state, once per launch (adopted by the host if nothing aborted)
    const int64_t ci = (int64_t)c * g.n + cu.i;
    a.lam_out[ci] = cu.lam;
    a.mu_out[ci] = cu.mu;
  }
}

// The deferred level-2 draw alone (clv_run's flush before anything reads the hyper state or the
// level-2 records): persist_level2's iteration -1 with no sweeps, one workgroup per chain; it
// writes hyper_out, the level-2 record and ctrl->cur as the end of a launch does.
template <int D, int K>
__global__ __launch_bounds__(BLOCK) void persist_flush_kernel(SweepArgs a, int64_t s_first) {
  __shared__ double pool[1];
  const int c = blockIdx.y;
  uint32_t k0, k1;
  chain_key(a.r.seed, (int64_t)a.r.chain_first + c, &k0, &k1);
  persist_level2<D, K, false>(a, s_first, 0, c, k0, k1, 0, -2, pool);
}

// (beta, Sigma) -> hyper state for every chain: [chain][K*D + D*D] input.
// NR: Philox mode finalises like the level-2 draws do (rcp_nr / rsq_nr), so a state set here
// (clv_create, clv_set_state) carries the same bits as the uninterrupted run's.
template <int D, int K, bool NR>
__global__ void set_hyper_kernel(int n_chains, double* hyper, const double* bs, double omega2) {
  const int c = threadIdx.x;
  if (c >= n_chains) return;
  const double* in = bs + (int64_t)c * (K * D + D * D);
  double Sig[D][D];
  for (int p = 0; p < D; ++p)
    for (int q = 0; q < D; ++q) Sig[p][q] = in[K * D + p * D + q];
  finalize_hyper<D, K, false, NR>(in, Sig, omega2, hyper + (int64_t)c * HS);
}

// ---------------------------------------------------------------------------------------------
// Debug / test kernels
// ---------------------------------------------------------------------------------------------
__global__ void debug_philox_kernel(uint32_t k0, uint32_t k1, const uint32_t* ctr, int64_t n, uint32_t* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const u32x4 r = philox4x32_10(u32x4{ctr[4 * i], ctr[4 * i + 1], ctr[4 * i + 2], ctr[4 * i + 3]}, k0, k1);
  out[4 * i] = r.x;
  out[4 * i + 1] = r.y;
  out[4 * i + 2] = r.z;
  out[4 * i + 3] = r.w;
}

__global__ void debug_variates_kernel(uint64_t seed, int chain, uint32_t sweep, int64_t n, int S, float* tl,
                                      float* tm, float* ua, float* l2u, double* uz, double* ut, double* ea,
                                      double* ez) {
  __shared__ __attribute__((aligned(16))) double tab[FAST_TAB_N3];
  fast_tab_fill(tab, threadIdx.x, blockDim.x, true);
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k0, k1;
  chain_key(seed, chain, &k0, &k1);
  const u32x4 r = customer_block(k0, k1, (uint32_t)i, sweep, SLOT_ZTAU);
  uz[i] = u53(r.x, r.y);
  ut[i] = u53(r.z, r.w);
  ea[i] = -log_fast(u53_open0(r.z, r.w), tab);  // as cust_ztau's alive dropout time
  ez[i] = eta_normal(k0, k1, (uint32_t)i, sweep, tab);
  const SlotPhilox ph(k0, k1, (uint32_t)i, sweep);
  for (int j = 0; j < S; ++j) {
    const u32x4 r = ph(SLOT_MH0 + (uint32_t)j);
    tl[(int64_t)j * n + i] = t3_f32(uf32(r.x), angle_hi(r.z));
    tm[(int64_t)j * n + i] = t3_f32(uf32(r.y), angle_lo(r.z));
    ua[(int64_t)j * n + i] = uf32(r.w);
    l2u[(int64_t)j * n + i] = log2_f32(uf32(r.w));  // the accept threshold's log2 U, as mh_chunk_variates forms it
  }
}

// The accept threshold's log2_f32(uf32(w)) (v_log_f32) against fp64 log2 of the same fp32 uniform
// over the words [w_begin, w_end): per block the max error in fp32 ulps of the exact value, the max
// absolute error, the word of the max ulp error and the max ulp error where U <= 1/2.
__global__ void debug_log2u_scan_kernel(uint64_t w_begin, uint64_t w_end, double* out) {
  double mu = 0.0, ma = 0.0, wu = 0.0, mf = 0.0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t w = w_begin + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < w_end; w += stride) {
    const float u = uf32((uint32_t)w);
    const float y = log2_f32(u);
    const double e = log2((double)u);
    double err_ulp;
    if (e == 0.0) {
      err_ulp = y == 0.0f ? 0.0 : 1e30;
    } else {
      const double ulp = ldexp(1.0, ilogb(e) - 23);  // fp32 ulp at the exact value
      err_ulp = fabs((double)y - e) / ulp;
    }
    const double ae = fabs((double)y - e);
    if (err_ulp > mu) {
      mu = err_ulp;
      wu = (double)w;
    }
    ma = fmax(ma, ae);
    if (u <= 0.5f) mf = fmax(mf, err_ulp);
  }
  __shared__ double red[4][256];
  red[0][threadIdx.x] = mu;
  red[1][threadIdx.x] = ma;
  red[2][threadIdx.x] = wu;
  red[3][threadIdx.x] = mf;
  __syncthreads();
  if (threadIdx.x == 0) {
    double bm = 0.0, ba = 0.0, bw = 0.0, bf = 0.0;
    for (int t = 0; t < 256; ++t) {
      if (red[0][t] > bm) {
        bm = red[0][t];
        bw = red[2][t];
      }
      ba = fmax(ba, red[1][t]);
      bf = fmax(bf, red[3][t]);
    }
    out[4 * blockIdx.x] = bm;
    out[4 * blockIdx.x + 1] = ba;
    out[4 * blockIdx.x + 2] = bw;
    out[4 * blockIdx.x + 3] = bf;
  }
}

// The MH proposal's t3 transforms on caller words (n x 3: radius words x, y and the angle word z),
// exactly as mh_chunk_variates forms them: packed = 0 -> t3_f32 (the bivariate and persistent
// kernels), 1 -> t3_pair (trivariate launch-per-sweep).  Pins the proposal's symmetry (tests).
__global__ void debug_t3_kernel(const uint32_t* w, int64_t n, int packed, float* tl, float* tm) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t x = w[3 * i], y = w[3 * i + 1], z = w[3 * i + 2];
  if (packed) {
    const f32x2 t = t3_pair(x, y, z);
    tl[i] = t.x;
    tm[i] = t.y;
  } else {
    tl[i] = t3_f32(uf32(x), angle_hi(z));
    tm[i] = t3_f32(uf32(y), angle_lo(z));
  }
}

// in: [V 81][cholV 81][A0B0 27][S0B 9] prior block, then xty(K*D) yty(D*D) iwn(3) chi2(3) z(D*K)
template <int D, int K>
__global__ void debug_level2_kernel(const double* prior, const double* in, double* out) {
  constexpr int NXY = K * D;
  __shared__ double tot[NXY + D * (D + 1) / 2 + 1];
  __shared__ L2Scratch sc;
  if (threadIdx.x == 0) {
    for (int q = 0; q < NXY; ++q) tot[q] = in[q];
    int t = NXY;
    for (int p = 0; p < D; ++p)
      for (int q = p; q < D; ++q) tot[t++] = in[NXY + p * D + q];
  }
  __syncthreads();
  const double* iwn = in + NXY + D * D;
  const double* chi = iwn + 3;
  const double* z = chi + 3;
  stage_prior(prior, &sc);
  __syncthreads();
  level2_draw<D, K>(tot, iwn, chi, z, false, &sc);
  if (threadIdx.x == 0) {
    for (int q = 0; q < K * D; ++q) out[q] = sc.beta[q];
    for (int q = 0; q < D * D; ++q) out[K * D + q] = sc.Sig[q];
  }
}

__global__ void debug_hyper_variates_kernel(uint64_t seed, int chain, uint32_t sweep, double df, int64_t n,
                                            double* chi2, double* normals) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k0, k1;
  chain_key(seed, chain, &k0, &k1);
  chi2[i] = chi2_draw(k0, k1, sweep + (uint32_t)i, 0, df);
  normals[i] = hyper_normal(k0, k1, HSLOT_NORMAL0, sweep + (uint32_t)i);
}

template <bool LOG>
__global__ void debug_exp_kernel(const double* x, int64_t n, double* out) {
  __shared__ __attribute__((aligned(16))) double tab[FAST_TAB_N];
  fast_tab_fill(tab, threadIdx.x, blockDim.x);
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = LOG ? log_fast(x[i], tab) : exp_fast(x[i], tab);
}

// The shipped Philox-mode MH step on given inputs (tests only): per lane, the log-posterior
// constants of bi:291-310 (x, z, T, tau, mean row (m0, m1), precision p00/p01/p11), the current
// point (ll, lm), one proposal's t3 noise (t_l, t_m), the scales (s00, s11) and log U.  Runs the
// same cust_coeffs (current log posterior, Q3 cap) and mh_step (fma + clip proposal, accept rule)
// the sweep kernels inline.  out[lane] = {cur, plp, ll', lm', cur'} with plp = log_post_fast of
// the clipped proposal (before the pm > 5 cap).
__global__ void debug_mh_kernel(const int32_t* x, const uint8_t* z, const double* T, const double* tau,
                                const double* m, const double* prec, const double* cur_pt, const float* t3,
                                const double* scale, const float* log_u, int64_t n, double* out) {
  __shared__ __attribute__((aligned(16))) double tab[FAST_TAB_N];
  fast_tab_fill(tab, threadIdx.x, blockDim.x);
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double H[HS];
  for (int j = 0; j < HS; ++j) H[j] = 0.0;
  H[H_BETA + 0] = m[2 * i];      // K = 1: X @ beta = 1 * beta = the given mean row, exactly
  H[H_BETA + 1] = m[2 * i + 1];
  H[H_P00] = prec[0];
  H[H_P01] = prec[1];
  H[H_P11] = prec[2];
  Cust<2, 1> u;
  u.xr_[0] = 1.0;
  u.xm = (double)x[i];
  u.z = z[i] != 0;
  u.lc.xm = u.xm;
  u.lc.omz = u.z ? 0.0 : 1.0;  // as cust_ztau sets them (bi:299-301)
  u.lc.w = u.z ? T[i] : tau[i];
  u.ll = cur_pt[2 * i];
  u.lm = cur_pt[2 * i + 1];
  cust_coeffs<2, 1, false>(u, H, tab);
  const double cur0 = u.cur;
  const double pl = clip70_fma(scale[0], (double)t3[2 * i], u.ll);
  const double pm = prop_lm(scale[1], (double)t3[2 * i + 1], u.lm);
  const double plp = log_post_fast(u.fc, pl, pm, tab);
  mh_step(u, scale[0], scale[1], t3[2 * i], t3[2 * i + 1], log_u[i], tab);
  double* o = out + 7 * i;
  o[0] = cur0;
  o[1] = plp;
  o[2] = pl;
  o[3] = pm;
  o[4] = u.ll;
  o[5] = u.lm;
  o[6] = u.cur;
}

// ---------------------------------------------------------------------------------------------
// Dispatch
// ---------------------------------------------------------------------------------------------
#ifdef CLV_ONLY_K  // analysis builds only (tools/asm_*.py): one covariate count, a fraction of the compile time
#define CLV_FOR_K(M, D, R) M(D, CLV_ONLY_K, R)
#else
#define CLV_FOR_K(M, D, R) \
  M(D, 1, R) M(D, 2, R) M(D, 3, R) M(D, 4, R) M(D, 5, R) M(D, 6, R) M(D, 7, R) M(D, 8, R) M(D, 9, R)
#endif

hipError_t launch_sweep(const SweepArgs& a, bool replay, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  const bool fx = a.fuse && a.g.world_size > 1;  // sharded, fused peer exchange (never in replay mode)
#define CLV_CASE(DD, KK, RR)                                                      \
  if (a.g.D == DD && a.g.K == KK && replay == RR) {                               \
    if constexpr (!RR) {                                                          \
      if (fx) return launch_sweep_t<DD, KK, RR, true>(a, st, e0, e1);             \
    }                                                                             \
    return launch_sweep_t<DD, KK, RR, false>(a, st, e0, e1);                      \
  }
  CLV_FOR_K(CLV_CASE, 2, false)
  CLV_FOR_K(CLV_CASE, 3, false)
  CLV_FOR_K(CLV_CASE, 2, true)
  CLV_FOR_K(CLV_CASE, 3, true)
#undef CLV_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_persist_flush(const SweepArgs& a, int64_t s_first, hipStream_t st) {
  const dim3 grid(1, a.g.n_chains);
#define CLV_CASE(DD, KK, PP)                                                                     \
  if (a.g.D == DD && a.g.K == KK) {                                                              \
    hipLaunchKernelGGL((persist_flush_kernel<DD, KK>), grid, dim3(BLOCK), 0, st, a, s_first);  \
    return hipGetLastError();                                                                  \
  }
  CLV_FOR_K(CLV_CASE, 2, false)
  CLV_FOR_K(CLV_CASE, 3, false)
#undef CLV_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_persist(const SweepArgs& a, int64_t s_first, int64_t n_sweeps, hipStream_t st, hipEvent_t e0,
                          hipEvent_t e1) {
  const dim3 grid(a.g.nb_local + 1, a.g.n_chains);  // + the chain's level-2 workgroup
  const dim3 block(BLOCK);
#define CLV_CASE(DD, KK, PP)                                                                                         \
  if (a.g.D == DD && a.g.K == KK && (a.g.world_size > 1) == PP) {                                                \
    if (e0) hipExtLaunchKernelGGL((persist_kernel<DD, KK, PP>), grid, block, 0, st, e0, e1, 0, a, s_first, n_sweeps); \
    else hipLaunchKernelGGL((persist_kernel<DD, KK, PP>), grid, block, 0, st, a, s_first, n_sweeps);                  \
    return hipGetLastError();                                                                                      \
  }
  CLV_FOR_K(CLV_CASE, 2, false)
  CLV_FOR_K(CLV_CASE, 3, false)
  CLV_FOR_K(CLV_CASE, 2, true)
  CLV_FOR_K(CLV_CASE, 3, true)
#undef CLV_CASE
  return hipErrorInvalidValue;
}

hipError_t persist_occupancy(int D, int K, bool p2p, int* blocks_per_cu) {
#define CLV_CASE(DD, KK, PP) \
  if (D == DD && K == KK && p2p == PP) return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, persist_kernel<DD, KK, PP>, BLOCK, 0);
  CLV_FOR_K(CLV_CASE, 2, false)
  CLV_FOR_K(CLV_CASE, 3, false)
  CLV_FOR_K(CLV_CASE, 2, true)
  CLV_FOR_K(CLV_CASE, 3, true)
#undef CLV_CASE
  return hipErrorInvalidValue;
}

// Private-segment (scratch) bytes per lane of a persistent instance: > 0 where the compiler spilled
// (trivariate K >= 6 at world size 1, large trivariate K in the peer instances).  Such a grid is not
// run persistently: the runtime may cap the waves in flight by the scratch it provisions, and a
// resident grid that is not all resident deadlocks its hand-offs until the wait bound (seen: the
// trivariate K = 9 peer instance at world 2 on one card, round 6).
hipError_t persist_scratch_bytes(int D, int K, bool p2p, size_t* bytes) {
  hipFuncAttributes fa{};
#define CLV_CASE(DD, KK, PP)                                                                     \
  if (D == DD && K == KK && p2p == PP) {                                                         \
    const hipError_t e = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&persist_kernel<DD, KK, PP>)); \
    *bytes = fa.localSizeBytes;                                                                  \
    return e;                                                                                    \
  }
  CLV_FOR_K(CLV_CASE, 2, false)
  CLV_FOR_K(CLV_CASE, 3, false)
  CLV_FOR_K(CLV_CASE, 2, true)
  CLV_FOR_K(CLV_CASE, 3, true)
#undef CLV_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_group(const GroupArgs& a, hipStream_t st) {
  const int units_local = (a.g.nb_local + a.g.blocks_per_unit - 1) / a.g.blocks_per_unit;
  hipLaunchKernelGGL(group_kernel, dim3(units_local, a.g.n_chains), dim3(64), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_hyper(const HyperArgs& a, bool replay, hipStream_t st) {
#define CLV_CASE(DD, KK, RR) \
  if (a.g.D == DD && a.g.K == KK && replay == RR) { hipLaunchKernelGGL((hyper_kernel<DD, KK, RR>), dim3(a.g.n_chains), dim3(256), 0, st, a); return hipGetLastError(); }
  CLV_FOR_K(CLV_CASE, 2, false)
  CLV_FOR_K(CLV_CASE, 3, false)
  CLV_FOR_K(CLV_CASE, 2, true)
  CLV_FOR_K(CLV_CASE, 3, true)
#undef CLV_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_set_hyper(int D, int K, int n_chains, double* hyper, const double* bs, double omega2,
                            bool replay, hipStream_t st) {
#define CLV_CASE(DD, KK, RR) \
  if (D == DD && K == KK && replay == RR) { hipLaunchKernelGGL((set_hyper_kernel<DD, KK, !RR && CLV_L2_NR != 0>), dim3(1), dim3(64), 0, st, n_chains, hyper, bs, omega2); return hipGetLastError(); }
  CLV_FOR_K(CLV_CASE, 2, false)
  CLV_FOR_K(CLV_CASE, 3, false)
  CLV_FOR_K(CLV_CASE, 2, true)
  CLV_FOR_K(CLV_CASE, 3, true)
#undef CLV_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_debug_philox(uint32_t k0, uint32_t k1, const uint32_t* ctr, int64_t n, uint32_t* out,
                               hipStream_t st) {
  hipLaunchKernelGGL(debug_philox_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, k0, k1, ctr, n, out);
  return hipGetLastError();
}

hipError_t launch_debug_variates(uint64_t seed, int chain, uint32_t sweep, int64_t n, int S, float* tl,
                                 float* tm, float* ua, float* l2u, double* uz, double* ut, double* ea, double* ez,
                                 hipStream_t st) {
  hipLaunchKernelGGL(debug_variates_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, seed, chain,
                     sweep, n, S, tl, tm, ua, l2u, uz, ut, ea, ez);
  return hipGetLastError();
}

hipError_t launch_debug_log2u_scan(uint64_t w_begin, uint64_t w_end, int n_blocks, double* out, hipStream_t st) {
  hipLaunchKernelGGL(debug_log2u_scan_kernel, dim3((unsigned)n_blocks), dim3(256), 0, st, w_begin, w_end, out);
  return hipGetLastError();
}

hipError_t launch_debug_t3(const uint32_t* w, int64_t n, int packed, float* tl, float* tm, hipStream_t st) {
  hipLaunchKernelGGL(debug_t3_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, w, n, packed, tl, tm);
  return hipGetLastError();
}

hipError_t launch_debug_level2(int D, int K, const double* prior_dev, const double* in, double* out,
                               hipStream_t st) {
#define CLV_CASE(DD, KK, RR) \
  if (D == DD && K == KK) { hipLaunchKernelGGL((debug_level2_kernel<DD, KK>), dim3(1), dim3(256), 0, st, prior_dev, in, out); return hipGetLastError(); }
  CLV_FOR_K(CLV_CASE, 2, 0)
  CLV_FOR_K(CLV_CASE, 3, 0)
#undef CLV_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_debug_hyper_variates(uint64_t seed, int chain, uint32_t sweep, double df, int64_t n,
                                       double* chi2, double* normals, hipStream_t st) {
  hipLaunchKernelGGL(debug_hyper_variates_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, seed,
                     chain, sweep, df, n, chi2, normals);
  return hipGetLastError();
}

hipError_t launch_debug_exp(const double* x, int64_t n, double* out, hipStream_t st, bool log_fn) {
  if (log_fn) hipLaunchKernelGGL(debug_exp_kernel<true>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, n, out);
  else hipLaunchKernelGGL(debug_exp_kernel<false>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, n, out);
  return hipGetLastError();
}

hipError_t launch_debug_mh(const int32_t* x, const uint8_t* z, const double* T, const double* tau, const double* m,
                           const double* prec, const double* cur_pt, const float* t3, const double* scale,
                           const float* log_u, int64_t n, double* out, hipStream_t st) {
  hipLaunchKernelGGL(debug_mh_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, z, T, tau, m, prec,
                     cur_pt, t3, scale, log_u, n, out);
  return hipGetLastError();
}

}  // namespace clv
