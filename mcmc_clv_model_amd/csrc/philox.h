// Philox4x32-10 counter-based RNG and the variate transforms of the sampler's Philox mode.
//
// The reference draws from numpy's PCG64 stream in a fixed call order
// (bivariate/mcmc.py:200, 217, 225, 258, 261, 316-317, 330; trivariate/mcmc.py:333), which
// cannot be reproduced by a parallel sampler.  Here every variate is a pure function of
//   key     = (lo32(seed + chain), hi32(seed + chain))      (reference: default_rng(seed + ch))
//   counter = (customer, sweep, slot, stream)                 (stream 0 = customers, 1 = hyper)
// so draws do not depend on launch geometry, sharding or GPU count.  The same transforms are
// restated in numpy by oracle/philox.py (test infrastructure) and pinned by tests.
#pragma once
#include <stdint.h>


#define CLV_HD __host__ __device__ __forceinline__

namespace clv {

struct u32x4 { uint32_t x, y, z, w; };

// a ^ b ^ c in one VALU instruction on gfx950 (v_bitop3_b32, truth table 0x96); the compiler
// emits two v_xor_b32 for the plain expression.
CLV_HD uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}

CLV_HD u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c = u32x4{xor3(hi1, c.y, k0), lo1, xor3(hi0, c.w, k1), lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// Stream ids (counter word 3).
enum : uint32_t { STREAM_CUSTOMER = 0u, STREAM_HYPER = 1u };

// Customer-stream slots (counter word 2).
enum : uint32_t { SLOT_ZTAU = 0u, SLOT_ETA = 1u, SLOT_MH0 = 2u };  // MH step j: block SLOT_MH0 + j

// Hyper-stream slots (counter word 0; word 1 = sweep).
enum : uint32_t { HSLOT_NORMAL0 = 0u, HSLOT_BETA_NORMAL0 = 4u, HSLOT_GAMMA0 = 64u, HSLOT_GAMMA_STRIDE = 256u };
constexpr int GAMMA_MAX_ATTEMPTS = 100;

// 53-bit uniform in [0, 1) from two words (numpy's random() resolution).
CLV_HD double u53(uint32_t lo, uint32_t hi) {
  const uint64_t v = (((uint64_t)hi << 32) | lo) >> 11;
  return (double)v * 0x1.0p-53;
}
// 53-bit uniform in (0, 1].
CLV_HD double u53_open0(uint32_t lo, uint32_t hi) {
  const uint64_t v = (((uint64_t)hi << 32) | lo) >> 11;
  return (double)(v + 1) * 0x1.0p-53;
}

CLV_HD u32x4 customer_block(uint32_t k0, uint32_t k1, uint32_t customer, uint32_t sweep, uint32_t slot) {
  return philox4x32_10(u32x4{customer, sweep, slot, STREAM_CUSTOMER}, k0, k1);
}

// Philox4x32-10 of counter (customer, sweep, slot, STREAM_CUSTOMER) with the slot-independent
// products hoisted: round 1's M0*customer and round 2's M1*(hi(M0*customer)^stream^k1) depend only
// on (customer, key), so one sweep's blocks cost 18 instead of 20 multiplies.  Bit-identical to
// customer_block() (checked by the device KAT test through clv_debug_variates).
struct SlotPhilox {
  uint32_t k0, k1, sk0;  // sk0 = sweep ^ k0, made wave-uniform (scalar registers) below
  uint32_t r1z, r1w;     // round-1 outputs that do not depend on the slot
  uint64_t p1r2;         // round-2 product M1 * r1z
  CLV_HD SlotPhilox(uint32_t k0_, uint32_t k1_, uint32_t customer, uint32_t sweep_) : k0(k0_), k1(k1_) {
    sk0 = sweep_ ^ k0_;
#if defined(__HIP_DEVICE_COMPILE__)
    // the sweep and key are uniform, but the compiler may hold them in vector registers (loop-carried
    // sweep counters): without this, round 2's uniform M0 product ran per lane (2 v_mad_u64_u32 +
    // 2 v_xor per block)
    sk0 = __builtin_amdgcn_readfirstlane(sk0);
#endif
    const uint64_t p0 = (uint64_t)0xD2511F53u * customer;
    r1z = (uint32_t)(p0 >> 32) ^ STREAM_CUSTOMER ^ k1_;
    r1w = (uint32_t)p0;
    p1r2 = (uint64_t)0xCD9E8D57u * r1z;
  }
  // `slot` must be uniform across the wavefront (it is at every call site: a loop counter):
  // round 1's M1 * slot and round 2's M0 product then run on the scalar unit.
  CLV_HD u32x4 operator()(uint32_t slot) const {
#if defined(__HIP_DEVICE_COMPILE__)
    slot = __builtin_amdgcn_readfirstlane(slot);
#endif
    // round 1 (key k): words x, y are uniform (plain xor: scalar unit)
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * slot;
    u32x4 c{(uint32_t)(p1 >> 32) ^ sk0, (uint32_t)p1, r1z, r1w};
    uint32_t a0 = k0 + 0x9E3779B9u, a1 = k1 + 0xBB67AE85u;
    // round 2: M0 * x is uniform, M1 * z (= p1r2) is slot-independent and hoisted; the uniform
    // parts of each xor are combined first, so each lane pays one v_xor
    {
      const uint64_t q0 = (uint64_t)0xD2511F53u * c.x;
      const uint32_t ux = c.y ^ a0, uz = (uint32_t)(q0 >> 32) ^ a1;
      c = u32x4{(uint32_t)(p1r2 >> 32) ^ ux, (uint32_t)p1r2, uz ^ c.w, (uint32_t)q0};
      a0 += 0x9E3779B9u;
      a1 += 0xBB67AE85u;
    }
#pragma unroll
    for (int r = 2; r < 10; ++r) {
      const uint64_t q0 = (uint64_t)0xD2511F53u * c.x;
      const uint64_t q1 = (uint64_t)0xCD9E8D57u * c.z;
      c = u32x4{xor3((uint32_t)(q1 >> 32), c.y, a0), (uint32_t)q1, xor3((uint32_t)(q0 >> 32), c.w, a1), (uint32_t)q0};
      a0 += 0x9E3779B9u;
      a1 += 0xBB67AE85u;
    }
    return c;
  }
};
CLV_HD u32x4 hyper_block(uint32_t k0, uint32_t k1, uint32_t slot, uint32_t sweep) {
  return philox4x32_10(u32x4{slot, sweep, 0u, STREAM_HYPER}, k0, k1);
}

CLV_HD void chain_key(uint64_t seed, int64_t chain, uint32_t* k0, uint32_t* k1) {
  const uint64_t s = seed + (uint64_t)chain;
  *k0 = (uint32_t)s;
  *k1 = (uint32_t)(s >> 32);
}

// fp32 uniform in [2^-33, 1] for the proposal-noise transforms (hardware transcendentals).
__device__ __forceinline__ float uf32(uint32_t w) {
  return __builtin_fmaf((float)w, 0x1.0p-32f, 0x1.0p-33f);
}
__device__ __forceinline__ float log2_f32(float u) {  // v_log_f32 (the MH step scales by ln 2 in fp64)
  return __builtin_amdgcn_logf(u);
}
// Student-t(3) by Bailey's trigonometric form of the polar method (Bailey 1994, Math. Comp.
// 62:779-781): R^2 = nu (U^(-2/nu) - 1) is the squared radius of a spherical bivariate t_nu, so
// R cos(2 pi V) is exactly t_nu.  Four hardware transcendentals, no rejection.  The radius
// uniform u is a full 32-bit word; the angle v (revolutions, v_cos_f32) has 16-bit resolution —
// a lattice closed under v -> v + 1/2, and the hardware cosine is odd under that shift bit for bit
// (t(k + 2^15) == -t(k) for all 65,536 angles k, tests/test_gpu_parity.py
// test_t3_proposal_symmetric_over_every_angle), so the proposal is exactly symmetric and the MH
// acceptance without a proposal ratio (bi:329-330) targets the reference's posterior.
__device__ __forceinline__ float t3_f32(float u, float v) {
  const float p = __builtin_amdgcn_exp2f(-(2.0f / 3.0f) * __builtin_amdgcn_logf(u));  // U^(-2/3)
  const float r = __builtin_amdgcn_sqrtf(__builtin_fmaf(3.0f, p, -3.0f));  // 3 (p - 1), one rounding
  return r * __builtin_amdgcn_cosf(v);
}
// The two 16-bit angles of one word, in revolutions: high half -> t_l, low half -> t_m.
// (float) of a 16-bit half is one v_cvt_f32_u32 with an SDWA word select; both are exact, so the
// values equal (w & 0xffff0000) * 2^-32 and (w << 16) * 2^-32.
__device__ __forceinline__ float angle_hi(uint32_t w) { return (float)(w >> 16) * 0x1.0p-16f; }
__device__ __forceinline__ float angle_lo(uint32_t w) { return (float)(w & 0xffffu) * 0x1.0p-16f; }

// The step's two t3 variates (t_l from words x and z's high half, t_m from y and z's low half)
// with every non-transcendental operation on the PAIR in one packed fp32 instruction
// (v_pk_fma_f32 / v_pk_mul_f32: two lanes' worth per issue): the same IEEE operations in the same
// order as two t3_f32 calls, so the same bits, in 17 VALU instead of 21.
// Used by the trivariate launch-per-sweep instances only (c5 122.8 -> 121.6 us per sweep); the
// bivariate and persistent kernels keep t3_f32 (measured slower with the pair: c2 10.80 -> 10.87,
// c4 85.0 -> 87.2).
#if defined(__clang__)  // (clang vector extension; the header is also host-compiled by g++ in tests)
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 t3_pair(uint32_t wl, uint32_t wm, uint32_t wz) {
  const f32x2 c32 = {0x1.0p-32f, 0x1.0p-32f}, c33 = {0x1.0p-33f, 0x1.0p-33f};
  const f32x2 m23 = {-(2.0f / 3.0f), -(2.0f / 3.0f)}, three = {3.0f, 3.0f}, mthree = {-3.0f, -3.0f};
  const f32x2 a16 = {0x1.0p-16f, 0x1.0p-16f};
  f32x2 u = {(float)wl, (float)wm};
  u = __builtin_elementwise_fma(u, c32, c33);                       // uf32 of both radius words
  f32x2 lg = {__builtin_amdgcn_logf(u.x), __builtin_amdgcn_logf(u.y)};
  lg = lg * m23;
  f32x2 p = {__builtin_amdgcn_exp2f(lg.x), __builtin_amdgcn_exp2f(lg.y)};  // U^(-2/3)
  p = __builtin_elementwise_fma(three, p, mthree);                  // 3 (p - 1), one rounding
  f32x2 ang = {(float)(wz >> 16), (float)(wz & 0xffffu)};
  ang = ang * a16;
  const f32x2 r = {__builtin_amdgcn_sqrtf(p.x), __builtin_amdgcn_sqrtf(p.y)};
  const f32x2 cs = {__builtin_amdgcn_cosf(ang.x), __builtin_amdgcn_cosf(ang.y)};
  return r * cs;
}
#endif

// Words of the MH steps: step j uses the four words of Philox block SLOT_MH0 + j:
// x = radius uniform of t_l, y = radius uniform of t_m, z = the two angles (16 bits each),
// w = accept uniform.  Chunk q = steps 4q .. 4q+3.
constexpr int MH_CHUNK_STEPS = 4;

// One chunk's variates: t_l, t_m and log2(U_accept) of 4 consecutive MH steps.  PACKED: the pair
// of t3 transforms as t3_pair (the same bits; the launch-per-sweep trivariate kernel takes it)
template <bool PACKED = false, class PH>
__device__ __forceinline__ void mh_chunk_variates(const PH& ph, uint32_t q, float (&t_l)[4], float (&t_m)[4],
                                                  float (&log2_u)[4]) {
#pragma unroll
  for (int i = 0; i < MH_CHUNK_STEPS; ++i) {
    const u32x4 r = ph(SLOT_MH0 + (uint32_t)MH_CHUNK_STEPS * q + (uint32_t)i);
#if defined(__clang__)
    if constexpr (PACKED) {
      const f32x2 t = t3_pair(r.x, r.y, r.z);
      t_l[i] = t.x;
      t_m[i] = t.y;
    } else {
      t_l[i] = t3_f32(uf32(r.x), angle_hi(r.z));
      t_m[i] = t3_f32(uf32(r.y), angle_lo(r.z));
    }
#else
    t_l[i] = t3_f32(uf32(r.x), angle_hi(r.z));
    t_m[i] = t3_f32(uf32(r.y), angle_lo(r.z));
#endif
    log2_u[i] = log2_f32(uf32(r.w));
  }
}

}  // namespace clv
