// Fast fp64 exp on CDNA4 VALU for arguments |x| <= 700 (the sampler's are clipped: bi:223, bi:323).
//
// exp(x) = 2^(k/256) * exp(r),  k = rint(x * 256/ln2) read from the low word of the "shifter"
// sum x * 256/ln2 + 1.5 * 2^52,  r = x - k ln2/256 (Cody-Waite, two fma), |r| <= ln2/512;
// 2^((k mod 256)/256) from a 256-entry LDS table (correctly rounded entries); expm1(r) by a
// degree-4 Taylor polynomial (truncation < r^5/120 ~ 3.7e-17 relative); the result
// t + t expm1(r) scaled by 2^(k div 256) with v_ldexp_f64 (exact: no overflow/underflow for
// |x| <= 700, the same bits as scaling t first).  Error <= ~1 ulp, like ocml's exp; 11 VALU +
// 1 LDS read instead of ~20 VALU.
// Constants: Python's decimal module at 80 digits, rounded to nearest (tools/gen_exp_table.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace clv {

constexpr int EXP_TAB_N = 256;
constexpr double EXP_INV_L = 0x1.71547652b82fep+8;   // 256 / ln2
constexpr double EXP_L_HI = 0x1.62e42fefa0000p-9;   // ln2 / 256, 38-bit head
constexpr double EXP_L_LO = 0x1.cf79abc9e3b3ap-48;  // ln2 / 256 - EXP_L_HI
constexpr double EXP_SHIFTER = 0x1.8p52;  // x + 1.5 * 2^52 rounds x to an integer held in the low word

__device__ constexpr double EXP2_TAB[EXP_TAB_N] = {
    0x1.0000000000000p+0, 0x1.00b1afa5abcbfp+0, 0x1.0163da9fb3335p+0, 0x1.02168143b0281p+0,
    0x1.02c9a3e778061p+0, 0x1.037d42e11bbccp+0, 0x1.04315e86e7f85p+0, 0x1.04e5f72f654b1p+0,
    0x1.059b0d3158574p+0, 0x1.0650a0e3c1f89p+0, 0x1.0706b29ddf6dep+0, 0x1.07bd42b72a836p+0,
    0x1.0874518759bc8p+0, 0x1.092bdf66607e0p+0, 0x1.09e3ecac6f383p+0, 0x1.0a9c79b1f3919p+0,
    0x1.0b5586cf9890fp+0, 0x1.0c0f145e46c85p+0, 0x1.0cc922b7247f7p+0, 0x1.0d83b23395decp+0,
    0x1.0e3ec32d3d1a2p+0, 0x1.0efa55fdfa9c5p+0, 0x1.0fb66affed31bp+0, 0x1.1073028d7233ep+0,
    0x1.11301d0125b51p+0, 0x1.11edbab5e2ab6p+0, 0x1.12abdc06c31ccp+0, 0x1.136a814f204abp+0,
    0x1.1429aaea92de0p+0, 0x1.14e95934f312ep+0, 0x1.15a98c8a58e51p+0, 0x1.166a45471c3c2p+0,
    0x1.172b83c7d517bp+0, 0x1.17ed48695bbc0p+0, 0x1.18af9388c8deap+0, 0x1.1972658375d2fp+0,
    0x1.1a35beb6fcb75p+0, 0x1.1af99f8138a1cp+0, 0x1.1bbe084045cd4p+0, 0x1.1c82f95281c6bp+0,
    0x1.1d4873168b9aap+0, 0x1.1e0e75eb44027p+0, 0x1.1ed5022fcd91dp+0, 0x1.1f9c18438ce4dp+0,
    0x1.2063b88628cd6p+0, 0x1.212be3578a819p+0, 0x1.21f49917ddc96p+0, 0x1.22bdda27912d1p+0,
    0x1.2387a6e756238p+0, 0x1.2451ffb82140ap+0, 0x1.251ce4fb2a63fp+0, 0x1.25e85711ece75p+0,
    0x1.26b4565e27cddp+0, 0x1.2780e341ddf29p+0, 0x1.284dfe1f56381p+0, 0x1.291ba7591bb70p+0,
    0x1.29e9df51fdee1p+0, 0x1.2ab8a66d10f13p+0, 0x1.2b87fd0dad990p+0, 0x1.2c57e39771b2fp+0,
    0x1.2d285a6e4030bp+0, 0x1.2df961f641589p+0, 0x1.2ecafa93e2f56p+0, 0x1.2f9d24abd886bp+0,
    0x1.306fe0a31b715p+0, 0x1.31432edeeb2fdp+0, 0x1.32170fc4cd831p+0, 0x1.32eb83ba8ea32p+0,
    0x1.33c08b26416ffp+0, 0x1.3496266e3fa2dp+0, 0x1.356c55f929ff1p+0, 0x1.36431a2de883bp+0,
    0x1.371a7373aa9cbp+0, 0x1.37f26231e754ap+0, 0x1.38cae6d05d866p+0, 0x1.39a401b7140efp+0,
    0x1.3a7db34e59ff7p+0, 0x1.3b57fbfec6cf4p+0, 0x1.3c32dc313a8e5p+0, 0x1.3d0e544ede173p+0,
    0x1.3dea64c123422p+0, 0x1.3ec70df1c5175p+0, 0x1.3fa4504ac801cp+0, 0x1.40822c367a024p+0,
    0x1.4160a21f72e2ap+0, 0x1.423fb2709468ap+0, 0x1.431f5d950a897p+0, 0x1.43ffa3f84b9d4p+0,
    0x1.44e086061892dp+0, 0x1.45c2042a7d232p+0, 0x1.46a41ed1d0057p+0, 0x1.4786d668b3237p+0,
    0x1.486a2b5c13cd0p+0, 0x1.494e1e192aed2p+0, 0x1.4a32af0d7d3dep+0, 0x1.4b17dea6db7d7p+0,
    0x1.4bfdad5362a27p+0, 0x1.4ce41b817c114p+0, 0x1.4dcb299fddd0dp+0, 0x1.4eb2d81d8abffp+0,
    0x1.4f9b2769d2ca7p+0, 0x1.508417f4531eep+0, 0x1.516daa2cf6642p+0, 0x1.5257de83f4eefp+0,
    0x1.5342b569d4f82p+0, 0x1.542e2f4f6ad27p+0, 0x1.551a4ca5d920fp+0, 0x1.56070dde910d2p+0,
    0x1.56f4736b527dap+0, 0x1.57e27dbe2c4cfp+0, 0x1.58d12d497c7fdp+0, 0x1.59c0827ff07ccp+0,
    0x1.5ab07dd485429p+0, 0x1.5ba11fba87a03p+0, 0x1.5c9268a5946b7p+0, 0x1.5d84590998b93p+0,
    0x1.5e76f15ad2148p+0, 0x1.5f6a320dceb71p+0, 0x1.605e1b976dc09p+0, 0x1.6152ae6cdf6f4p+0,
    0x1.6247eb03a5585p+0, 0x1.633dd1d1929fdp+0, 0x1.6434634ccc320p+0, 0x1.652b9febc8fb7p+0,
    0x1.6623882552225p+0, 0x1.671c1c70833f6p+0, 0x1.68155d44ca973p+0, 0x1.690f4b19e9538p+0,
    0x1.6a09e667f3bcdp+0, 0x1.6b052fa75173ep+0, 0x1.6c012750bdabfp+0, 0x1.6cfdcddd47645p+0,
    0x1.6dfb23c651a2fp+0, 0x1.6ef9298593ae5p+0, 0x1.6ff7df9519484p+0, 0x1.70f7466f42e87p+0,
    0x1.71f75e8ec5f74p+0, 0x1.72f8286ead08ap+0, 0x1.73f9a48a58174p+0, 0x1.74fbd35d7cbfdp+0,
    0x1.75feb564267c9p+0, 0x1.77024b1ab6e09p+0, 0x1.780694fde5d3fp+0, 0x1.790b938ac1cf6p+0,
    0x1.7a11473eb0187p+0, 0x1.7b17b0976cfdbp+0, 0x1.7c1ed0130c132p+0, 0x1.7d26a62ff86f0p+0,
    0x1.7e2f336cf4e62p+0, 0x1.7f3878491c491p+0, 0x1.80427543e1a12p+0, 0x1.814d2add106d9p+0,
    0x1.82589994cce13p+0, 0x1.8364c1eb941f7p+0, 0x1.8471a4623c7adp+0, 0x1.857f4179f5b21p+0,
    0x1.868d99b4492edp+0, 0x1.879cad931a436p+0, 0x1.88ac7d98a6699p+0, 0x1.89bd0a478580fp+0,
    0x1.8ace5422aa0dbp+0, 0x1.8be05bad61778p+0, 0x1.8cf3216b5448cp+0, 0x1.8e06a5e0866d9p+0,
    0x1.8f1ae99157736p+0, 0x1.902fed0282c8ap+0, 0x1.9145b0b91ffc6p+0, 0x1.925c353aa2fe2p+0,
    0x1.93737b0cdc5e5p+0, 0x1.948b82b5f98e5p+0, 0x1.95a44cbc8520fp+0, 0x1.96bdd9a7670b3p+0,
    0x1.97d829fde4e50p+0, 0x1.98f33e47a22a2p+0, 0x1.9a0f170ca07bap+0, 0x1.9b2bb4d53fe0dp+0,
    0x1.9c49182a3f090p+0, 0x1.9d674194bb8d5p+0, 0x1.9e86319e32323p+0, 0x1.9fa5e8d07f29ep+0,
    0x1.a0c667b5de565p+0, 0x1.a1e7aed8eb8bbp+0, 0x1.a309bec4a2d33p+0, 0x1.a42c980460ad8p+0,
    0x1.a5503b23e255dp+0, 0x1.a674a8af46052p+0, 0x1.a799e1330b358p+0, 0x1.a8bfe53c12e59p+0,
    0x1.a9e6b5579fdbfp+0, 0x1.ab0e521356ebap+0, 0x1.ac36bbfd3f37ap+0, 0x1.ad5ff3a3c2774p+0,
    0x1.ae89f995ad3adp+0, 0x1.afb4ce622f2ffp+0, 0x1.b0e07298db666p+0, 0x1.b20ce6c9a8952p+0,
    0x1.b33a2b84f15fbp+0, 0x1.b468415b749b1p+0, 0x1.b59728de5593ap+0, 0x1.b6c6e29f1c52ap+0,
    0x1.b7f76f2fb5e47p+0, 0x1.b928cf22749e4p+0, 0x1.ba5b030a1064ap+0, 0x1.bb8e0b79a6f1fp+0,
    0x1.bcc1e904bc1d2p+0, 0x1.bdf69c3f3a207p+0, 0x1.bf2c25bd71e09p+0, 0x1.c06286141b33dp+0,
    0x1.c199bdd85529cp+0, 0x1.c2d1cd9fa652cp+0, 0x1.c40ab5fffd07ap+0, 0x1.c544778fafb22p+0,
    0x1.c67f12e57d14bp+0, 0x1.c7ba88988c933p+0, 0x1.c8f6d9406e7b5p+0, 0x1.ca3405751c4dbp+0,
    0x1.cb720dcef9069p+0, 0x1.ccb0f2e6d1675p+0, 0x1.cdf0b555dc3fap+0, 0x1.cf3155b5bab74p+0,
    0x1.d072d4a07897cp+0, 0x1.d1b532b08c968p+0, 0x1.d2f87080d89f2p+0, 0x1.d43c8eacaa1d6p+0,
    0x1.d5818dcfba487p+0, 0x1.d6c76e862e6d3p+0, 0x1.d80e316c98398p+0, 0x1.d955d71ff6075p+0,
    0x1.da9e603db3285p+0, 0x1.dbe7cd63a8315p+0, 0x1.dd321f301b460p+0, 0x1.de7d5641c0658p+0,
    0x1.dfc97337b9b5fp+0, 0x1.e11676b197d17p+0, 0x1.e264614f5a129p+0, 0x1.e3b333b16ee12p+0,
    0x1.e502ee78b3ff6p+0, 0x1.e653924676d76p+0, 0x1.e7a51fbc74c83p+0, 0x1.e8f7977cdb740p+0,
    0x1.ea4afa2a490dap+0, 0x1.eb9f4867cca6ep+0, 0x1.ecf482d8e67f1p+0, 0x1.ee4aaa2188510p+0,
    0x1.efa1bee615a27p+0, 0x1.f0f9c1cb6412ap+0, 0x1.f252b376bba97p+0, 0x1.f3ac948dd7274p+0,
    0x1.f50765b6e4540p+0, 0x1.f6632798844f8p+0, 0x1.f7bfdad9cbe14p+0, 0x1.f91d802243c89p+0,
    0x1.fa7c1819e90d8p+0, 0x1.fbdba3692d514p+0, 0x1.fd3c22b8f71f1p+0, 0x1.fe9d96b2a23d9p+0,
};

__device__ __forceinline__ double exp_tab_entry(int j) { return EXP2_TAB[j]; }
__device__ __forceinline__ double exp_fast(double x, const double* lds_tab) {
  const double t = __builtin_fma(x, EXP_INV_L, EXP_SHIFTER);
  const double k = t - EXP_SHIFTER;                      // rint(x * 256 / ln2)
  const int ki = (int)(uint32_t)__builtin_bit_cast(uint64_t, t);  // the same integer (two's complement)
  double r = __builtin_fma(-k, EXP_L_HI, x);
  r = __builtin_fma(-k, EXP_L_LO, r);
  double p = __builtin_fma(r, 1.0 / 24.0, 1.0 / 6.0);
  p = __builtin_fma(p, r, 0.5);
  p = __builtin_fma(p, r, 1.0);
  p = p * r;                                             // expm1(r)
  const double tab = lds_tab[ki & (EXP_TAB_N - 1)];
  return __builtin_ldexp(__builtin_fma(tab, p, tab), ki >> 8);  // * 2^(k div 256) after the fma
}

// exp_fast of two independent arguments, bit-identical to two exp_fast calls, written so that both
// table reads are in flight before either is waited for: the compiler otherwise finishes the first
// exp (table read, s_waitcnt, scaling) before starting the second, so the MH step's dependent chain
// (both proposal exps, bi:299-301) paid the LDS latency twice.
__device__ __forceinline__ void exp_fast2(double x1, double x2, const double* lds_tab, double& e1, double& e2) {
  const double t1 = __builtin_fma(x1, EXP_INV_L, EXP_SHIFTER);
  const double t2 = __builtin_fma(x2, EXP_INV_L, EXP_SHIFTER);
  const int ki1 = (int)(uint32_t)__builtin_bit_cast(uint64_t, t1);
  const int ki2 = (int)(uint32_t)__builtin_bit_cast(uint64_t, t2);
  const double tab1 = lds_tab[ki1 & (EXP_TAB_N - 1)];
  const double tab2 = lds_tab[ki2 & (EXP_TAB_N - 1)];
  const double k1 = t1 - EXP_SHIFTER, k2 = t2 - EXP_SHIFTER;
  double r1 = __builtin_fma(-k1, EXP_L_HI, x1), r2 = __builtin_fma(-k2, EXP_L_HI, x2);
  r1 = __builtin_fma(-k1, EXP_L_LO, r1);
  r2 = __builtin_fma(-k2, EXP_L_LO, r2);
  double p1 = __builtin_fma(r1, 1.0 / 24.0, 1.0 / 6.0), p2 = __builtin_fma(r2, 1.0 / 24.0, 1.0 / 6.0);
  p1 = __builtin_fma(p1, r1, 0.5);
  p2 = __builtin_fma(p2, r2, 0.5);
  p1 = __builtin_fma(p1, r1, 1.0);
  p2 = __builtin_fma(p2, r2, 1.0);
  p1 = p1 * r1;
  p2 = p2 * r2;
  e1 = __builtin_ldexp(__builtin_fma(tab1, p1, tab1), ki1 >> 8);
  e2 = __builtin_ldexp(__builtin_fma(tab2, p2, tab2), ki2 >> 8);
}

// ---- Fast fp64 log for x > 0 normal (the sampler's Philox-mode logs: lambda, mu, the dropout
// time's uniform or truncated-exponential argument, eta's Box-Muller radius).  ocml's log is ~95
// VALU (double-double reduction); this one is 19 VALU + one 16-byte LDS read, <= 1 ulp
// (tools/gen_log_table.py: method, and a check against 60-digit logs with exact fma).
//   x = 2^k z, z in [0.6865, 1.373) from the high word; bin i of z -> (invc, logc = -log invc);
//   r = fma(z, invc, -1), |r| <= 2^-9;  log x = k ln2 + logc + log1p(r), log1p by its degree-6
//   Taylor polynomial.  The bin around 1 has invc = 1, logc = 0: no cancellation near x = 1.
// Table: LOG_TAB_N (invc, logc) pairs in LDS right after the exp table (FAST_TAB_N doubles).
constexpr int LOG_TAB_N = 256;
constexpr int FAST_TAB_N = EXP_TAB_N + 2 * LOG_TAB_N;
constexpr uint32_t LOG_OFF_HI = 0x3fe5f800u;
constexpr double LOG_LN2_HI = 0x1.62e42fefa3800p-1;
constexpr double LOG_LN2_LO = 0x1.ef35793c76730p-45;
__device__ constexpr double LOG_TAB[2 * LOG_TAB_N] = {  // (invc, logc) per bin
    0x1.745d1745d1746p+0, -0x1.7fafa3bd8151cp-2, 0x1.734f0c541fe8dp+0, -0x1.7cc7f7db46a0ep-2,
    0x1.724287f46debcp+0, -0x1.79e26687cfb3dp-2, 0x1.713786d9c7c09p+0, -0x1.76feecb947176p-2,
    0x1.702e05c0b8170p+0, -0x1.741d876c67bb1p-2, 0x1.6f26016f26017p+0, -0x1.713e33a46a17cp-2,
    0x1.6e1f76b4337c7p+0, -0x1.6e60ee6af1973p-2, 0x1.6d1a62681c861p+0, -0x1.6b85b4cffa3fdp-2,
    0x1.6c16c16c16c17p+0, -0x1.68ac83e9c6a15p-2, 0x1.6b1490aa31a3dp+0, -0x1.65d558d4ce00bp-2,
    0x1.6a13cd1537290p+0, -0x1.630030b3aac48p-2, 0x1.691473a88d0c0p+0, -0x1.602d08af091ecp-2,
    0x1.6816816816817p+0, -0x1.5d5bddf595f31p-2, 0x1.6719f3601671ap+0, -0x1.5a8cadbbedfa1p-2,
    0x1.661ec6a5122f9p+0, -0x1.57bf753c8d1fbp-2, 0x1.6524f853b4aa3p+0, -0x1.54f431b7be1a8p-2,
    0x1.642c8590b2164p+0, -0x1.522ae0738a3d7p-2, 0x1.63356b88ac0dep+0, -0x1.4f637ebba9810p-2,
    0x1.623fa77016240p+0, -0x1.4c9e09e172c3dp-2, 0x1.614b36831ae94p+0, -0x1.49da7f3bcc420p-2,
    0x1.6058160581606p+0, -0x1.4718dc271c41cp-2, 0x1.5f66434292dfcp+0, -0x1.44591e0539f49p-2,
    0x1.5e75bb8d015e7p+0, -0x1.419b423d5e8c6p-2, 0x1.5d867c3ece2a5p+0, -0x1.3edf463c1683ep-2,
    0x1.5c9882b931057p+0, -0x1.3c25277333183p-2, 0x1.5babcc647fa91p+0, -0x1.396ce359bbf53p-2,
    0x1.5ac056b015ac0p+0, -0x1.36b6776be1116p-2, 0x1.59d61f123ccaap+0, -0x1.3401e12aecba0p-2,
    0x1.58ed2308158edp+0, -0x1.314f1e1d35ce3p-2, 0x1.5805601580560p+0, -0x1.2e9e2bce12286p-2,
    0x1.571ed3c506b3ap+0, -0x1.2bef07cdc9355p-2, 0x1.56397ba7c52e2p+0, -0x1.2941afb186b7cp-2,
    0x1.5555555555555p+0, -0x1.269621134db91p-2, 0x1.54725e6bb82fep+0, -0x1.23ec5991eba49p-2,
    0x1.5390948f40febp+0, -0x1.214456d0eb8d5p-2, 0x1.52aff56a8054bp+0, -0x1.1e9e1678899f5p-2,
    0x1.51d07eae2f815p+0, -0x1.1bf99635a6b95p-2, 0x1.50f22e111c4c5p+0, -0x1.1956d3b9bc2f9p-2,
    0x1.5015015015015p+0, -0x1.16b5ccbacfb73p-2, 0x1.4f38f62dd4c9bp+0, -0x1.14167ef367784p-2,
    0x1.4e5e0a72f0539p+0, -0x1.1178e8227e47ap-2, 0x1.4d843bedc2c4cp+0, -0x1.0edd060b78082p-2,
    0x1.4cab88725af6ep+0, -0x1.0c42d676162e2p-2, 0x1.4bd3edda68fe1p+0, -0x1.09aa572e6c6d4p-2,
    0x1.4afd6a052bf5bp+0, -0x1.07138604d5864p-2, 0x1.4a27fad76014ap+0, -0x1.047e60cde83b7p-2,
    0x1.49539e3b2d067p+0, -0x1.01eae5626c691p-2, 0x1.4880522014880p+0, -0x1.feb2233ea07cbp-3,
    0x1.47ae147ae147bp+0, -0x1.f991c6cb3b37ap-3, 0x1.46dce34596066p+0, -0x1.f474b134df228p-3,
    0x1.460cbc7f5cf9ap+0, -0x1.ef5ade4dcffe5p-3, 0x1.453d9e2c776cap+0, -0x1.ea4449f04aaf5p-3,
    0x1.446f86562d9fbp+0, -0x1.e530effe71013p-3, 0x1.43a2730abee4dp+0, -0x1.e020cc6235ab5p-3,
    0x1.42d6625d51f87p+0, -0x1.db13db0d48941p-3, 0x1.420b5265e5951p+0, -0x1.d60a17f903514p-3,
    0x1.4141414141414p+0, -0x1.d1037f2655e7bp-3, 0x1.40782d10e6566p+0, -0x1.cc000c9db3c52p-3,
    0x1.3fb013fb013fbp+0, -0x1.c6ffbc6f00f71p-3, 0x1.3ee8f42a5af07p+0, -0x1.c2028ab17f9b5p-3,
    0x1.3e22cbce4a902p+0, -0x1.bd087383bd8aap-3, 0x1.3d5d991aa75c6p+0, -0x1.b811730b823d4p-3,
    0x1.3c995a47babe7p+0, -0x1.b31d8575bce3bp-3, 0x1.3bd60d9232955p+0, -0x1.ae2ca6f672bd8p-3,
    0x1.3b13b13b13b14p+0, -0x1.a93ed3c8ad9e5p-3, 0x1.3a524387ac822p+0, -0x1.a454082e6ab03p-3,
    0x1.3991c2c187f63p+0, -0x1.9f6c407089663p-3, 0x1.38d22d366088ep+0, -0x1.9a8778debaa3ap-3,
    0x1.3813813813814p+0, -0x1.95a5adcf70182p-3, 0x1.3755bd1c945eep+0, -0x1.90c6db9fcbcdbp-3,
    0x1.3698df3de0748p+0, -0x1.8beafeb38fe8fp-3, 0x1.35dce5f9f2af8p+0, -0x1.871213750e994p-3,
    0x1.3521cfb2b78c1p+0, -0x1.823c16551a3c0p-3, 0x1.34679ace01346p+0, -0x1.7d6903caf5acdp-3,
    0x1.33ae45b57bcb2p+0, -0x1.7898d85444c74p-3, 0x1.32f5ced6a1dfap+0, -0x1.73cb9074fd14dp-3,
    0x1.323e34a2b10bfp+0, -0x1.6f0128b756ab9p-3, 0x1.3187758e9ebb6p+0, -0x1.6a399dabbd383p-3,
    0x1.30d190130d190p+0, -0x1.6574ebe8c1339p-3, 0x1.301c82ac40260p+0, -0x1.60b3100b09474p-3,
    0x1.2f684bda12f68p+0, -0x1.5bf406b543db0p-3, 0x1.2eb4ea1fed14bp+0, -0x1.5737cc9018cddp-3,
    0x1.2e025c04b8097p+0, -0x1.527e5e4a1b58dp-3, 0x1.2d50a012d50a0p+0, -0x1.4dc7b897bc1c7p-3,
    0x1.2c9fb4d812ca0p+0, -0x1.4913d8333b563p-3, 0x1.2bef98e5a3711p+0, -0x1.4462b9dc9b3dcp-3,
    0x1.2b404ad012b40p+0, -0x1.3fb45a59928cap-3, 0x1.2a91c92f3c105p+0, -0x1.3b08b6757f2a7p-3,
    0x1.29e4129e4129ep+0, -0x1.365fcb0159014p-3, 0x1.293725bb804a5p+0, -0x1.31b994d3a4f86p-3,
    0x1.288b01288b013p+0, -0x1.2d1610c86813dp-3, 0x1.27dfa38a1ce4dp+0, -0x1.28753bc11aba2p-3,
    0x1.27350b8812735p+0, -0x1.23d712a49c201p-3, 0x1.268b37cd60127p+0, -0x1.1f3b925f25d44p-3,
    0x1.25e22708092f1p+0, -0x1.1aa2b7e23f729p-3, 0x1.2539d7e9177b2p+0, -0x1.160c8024b27b0p-3,
    0x1.2492492492492p+0, -0x1.1178e8227e47ap-3, 0x1.23eb79717605bp+0, -0x1.0ce7ecdccc28bp-3,
    0x1.23456789abcdfp+0, -0x1.08598b59e3a07p-3, 0x1.22a0122a0122ap+0, -0x1.03cdc0a51ec0dp-3,
    0x1.21fb78121fb78p+0, -0x1.fe89139dbd565p-4, 0x1.21579804855e6p+0, -0x1.f57bc7d9005dbp-4,
    0x1.20b470c67c0d9p+0, -0x1.ec739830a1126p-4, 0x1.2012012012012p+0, -0x1.e3707ee30487bp-4,
    0x1.1f7047dc11f70p+0, -0x1.da7276384469ep-4, 0x1.1ecf43c7fb84cp+0, -0x1.d179788219362p-4,
    0x1.1e2ef3b3fb874p+0, -0x1.c885801bc4b20p-4, 0x1.1d8f5672e4abdp+0, -0x1.bf968769fca18p-4,
    0x1.1cf06ada2811dp+0, -0x1.b6ac88dad5b1dp-4, 0x1.1c522fc1ce059p+0, -0x1.adc77ee5aea8ep-4,
    0x1.1bb4a4046ed29p+0, -0x1.a4e7640b1bc38p-4, 0x1.1b17c67f2bae3p+0, -0x1.9c0c32d4d254dp-4,
    0x1.1a7b9611a7b96p+0, -0x1.9335e5d594988p-4, 0x1.19e0119e0119ep+0, -0x1.8a6477a91dc29p-4,
    0x1.19453808ca29cp+0, -0x1.8197e2f40e3f0p-4, 0x1.18ab083902bdbp+0, -0x1.78d02263d82d7p-4,
    0x1.1811811811812p+0, -0x1.700d30aeac0e8p-4, 0x1.1778a191bd684p+0, -0x1.674f089365a78p-4,
    0x1.16e0689427379p+0, -0x1.5e95a4d9791cdp-4, 0x1.1648d50fc3201p+0, -0x1.55e10050e0382p-4,
    0x1.15b1e5f75270dp+0, -0x1.4d3115d207eacp-4, 0x1.151b9a3fdd5c9p+0, -0x1.4485e03dbdfb0p-4,
    0x1.1485f0e0acd3bp+0, -0x1.3bdf5a7d1ee5ep-4, 0x1.13f0e8d344724p+0, -0x1.333d7f8183f4ap-4,
    0x1.135c81135c811p+0, -0x1.2aa04a44717a1p-4, 0x1.12c8b89edc0acp+0, -0x1.2207b5c7854a1p-4,
    0x1.12358e75d3033p+0, -0x1.1973bd1465561p-4, 0x1.11a3019a74826p+0, -0x1.10e45b3cae829p-4,
    0x1.1111111111111p+0, -0x1.08598b59e3a06p-4, 0x1.107fbbe011080p+0, -0x1.ffa6911ab9309p-5,
    0x1.0fef010fef011p+0, -0x1.eea31c006b87cp-5, 0x1.0f5edfab325a2p+0, -0x1.dda8adc67ee59p-5,
    0x1.0ecf56be69c90p+0, -0x1.ccb73cdddb2d0p-5, 0x1.0e40655826011p+0, -0x1.bbcebfc68f424p-5,
    0x1.0db20a88f4696p+0, -0x1.aaef2d0fb1108p-5, 0x1.0d24456359e3ap+0, -0x1.9a187b573de81p-5,
    0x1.0c9714fbcda3bp+0, -0x1.894aa149fb34bp-5, 0x1.0c0a7868b4171p+0, -0x1.788595a3577c8p-5,
    0x1.0b7e6ec259dc8p+0, -0x1.67c94f2d4bb65p-5, 0x1.0af2f722eecb5p+0, -0x1.5715c4c03cee1p-5,
    0x1.0a6810a6810a7p+0, -0x1.466aed42de3f9p-5, 0x1.09ddba6af8360p+0, -0x1.35c8bfaa13069p-5,
    0x1.0953f39010954p+0, -0x1.252f32f8d1840p-5, 0x1.08cabb37565e2p+0, -0x1.149e3e4005a8dp-5,
    0x1.0842108421084p+0, -0x1.0415d89e74440p-5, 0x1.07b9f29b8eae2p+0, -0x1.e72bf2813ce6ap-6,
    0x1.073260a47f7c6p+0, -0x1.c63d2ec14aad7p-6, 0x1.06ab59c7912fbp+0, -0x1.a55f548c5c427p-6,
    0x1.0624dd2f1a9fcp+0, -0x1.8492528c8cac5p-6, 0x1.059eea0727586p+0, -0x1.63d6178690bbep-6,
    0x1.05197f7d73404p+0, -0x1.432a925980cbcp-6, 0x1.04949cc1664c5p+0, -0x1.228fb1fea2e0ap-6,
    0x1.0410410410410p+0, -0x1.0205658935837p-6, 0x1.038c6b78247fcp+0, -0x1.c317384c75f0dp-7,
    0x1.03091b51f5e1ap+0, -0x1.82448a388a283p-7, 0x1.02864fc7729e9p+0, -0x1.41929f968330cp-7,
    0x1.0204081020408p+0, -0x1.010157588de69p-7, 0x1.0182436517a37p+0, -0x1.8121214586b02p-8,
    0x1.0101010101010p+0, -0x1.0080559588b25p-8, 0x1.0080402010080p+0, -0x1.0040155d5881ep-9,
    0x1.0000000000000p+0, 0x0.0p+0, 0x1.fe01fe01fe020p-1, 0x1.ff00aa2b10ba0p-9,
    0x1.fc07f01fc07f0p-1, 0x1.fe02a6b106799p-8, 0x1.fa11caa01fa12p-1, 0x1.7dc475f810a69p-7,
    0x1.f81f81f81f820p-1, 0x1.fc0a8b0fc03c4p-7, 0x1.f6310aca0dbb5p-1, 0x1.3cea44346a584p-6,
    0x1.f44659e4a4271p-1, 0x1.7b91b07d5b126p-6, 0x1.f25f644230ab5p-1, 0x1.b9fc027af919ap-6,
    0x1.f07c1f07c1f08p-1, 0x1.f829b0e7832f8p-6, 0x1.ee9c7f8458e02p-1, 0x1.1b0d98923d97fp-5,
    0x1.ecc07b301ecc0p-1, 0x1.39e87b9febd68p-5, 0x1.eae807aba01ebp-1, 0x1.58a5bafc8e4d3p-5,
    0x1.e9131abf0b767p-1, 0x1.77458f632dcffp-5, 0x1.e741aa59750e4p-1, 0x1.95c830ec8e3f2p-5,
    0x1.e573ac901e574p-1, 0x1.b42dd711971b9p-5, 0x1.e3a9179dc1a73p-1, 0x1.d276b8adb0b56p-5,
    0x1.e1e1e1e1e1e1ep-1, 0x1.f0a30c01162a8p-5, 0x1.e01e01e01e01ep-1, 0x1.075983598e471p-4,
    0x1.de5d6e3f8868ap-1, 0x1.16536eea37ae3p-4, 0x1.dca01dca01dcap-1, 0x1.253f62f0a1417p-4,
    0x1.dae6076b981dbp-1, 0x1.341d7961bd1d0p-4, 0x1.d92f2231e7f8ap-1, 0x1.42edcbea646eep-4,
    0x1.d77b654b82c34p-1, 0x1.51b073f06183cp-4, 0x1.d5cac807572b2p-1, 0x1.60658a93750c4p-4,
    0x1.d41d41d41d41dp-1, 0x1.6f0d28ae56b4ep-4, 0x1.d272ca3fc5b1ap-1, 0x1.7da766d7b12d0p-4,
    0x1.d0cb58f6ec074p-1, 0x1.8c345d6319b23p-4, 0x1.cf26e5c44bfc6p-1, 0x1.9ab42462033aep-4,
    0x1.cd85689039b0bp-1, 0x1.a926d3a4ad562p-4, 0x1.cbe6d9601cbe7p-1, 0x1.b78c82bb0eda0p-4,
    0x1.ca4b3055ee191p-1, 0x1.c5e548f5bc743p-4, 0x1.c8b265afb8a42p-1, 0x1.d4313d66cb35dp-4,
    0x1.c71c71c71c71cp-1, 0x1.e27076e2af2eap-4, 0x1.c5894d10d4986p-1, 0x1.f0a30c01162a4p-4,
    0x1.c3f8f01c3f8f0p-1, 0x1.fec9131dbeabcp-4, 0x1.c26b5392ea01cp-1, 0x1.0671512ca596fp-3,
    0x1.c0e070381c0e0p-1, 0x1.0d77e7cd08e5bp-3, 0x1.bf583ee868d8bp-1, 0x1.14785846742acp-3,
    0x1.bdd2b899406f7p-1, 0x1.1b72ad52f67a2p-3, 0x1.bc4fd65883e7bp-1, 0x1.2266f190a5acdp-3,
    0x1.bacf914c1bad0p-1, 0x1.29552f81ff521p-3, 0x1.b951e2b18ff23p-1, 0x1.303d718e47fd5p-3,
    0x1.b7d6c3dda338bp-1, 0x1.371fc201e8f75p-3, 0x1.b65e2e3beee05p-1, 0x1.3dfc2b0ecc62ap-3,
    0x1.b4e81b4e81b4fp-1, 0x1.44d2b6ccb7d1cp-3, 0x1.b37484ad806cep-1, 0x1.4ba36f39a55e5p-3,
    0x1.b2036406c80d9p-1, 0x1.526e5e3a1b438p-3, 0x1.b094b31d922a4p-1, 0x1.59338d9982085p-3,
    0x1.af286bca1af28p-1, 0x1.5ff3070a793d6p-3, 0x1.adbe87f94905ep-1, 0x1.66acd4272ad51p-3,
    0x1.ac5701ac5701bp-1, 0x1.6d60fe719d21bp-3, 0x1.aaf1d2f87ebfdp-1, 0x1.740f8f54037a3p-3,
    0x1.a98ef606a63bep-1, 0x1.7ab890210d907p-3, 0x1.a82e65130e159p-1, 0x1.815c0a14357e9p-3,
    0x1.a6d01a6d01a6dp-1, 0x1.87fa06520c911p-3, 0x1.a574107688a4ap-1, 0x1.8e928de886d41p-3,
    0x1.a41a41a41a41ap-1, 0x1.9525a9cf456b6p-3, 0x1.a2c2a87c51ca0p-1, 0x1.9bb362e7dfb85p-3,
    0x1.a16d3f97a4b02p-1, 0x1.a23bc1fe2b561p-3, 0x1.a01a01a01a01ap-1, 0x1.a8becfc882f19p-3,
    0x1.9ec8e951033d9p-1, 0x1.af3c94e80bff3p-3, 0x1.9d79f176b682dp-1, 0x1.b5b519e8fb5a6p-3,
    0x1.9c2d14ee4a102p-1, 0x1.bc286742d8cd4p-3, 0x1.9ae24ea5510dap-1, 0x1.c2968558c18c2p-3,
    0x1.999999999999ap-1, 0x1.c8ff7c79a9a20p-3, 0x1.9852f0d8ec0ffp-1, 0x1.cf6354e09c5ddp-3,
    0x1.970e4f80cb872p-1, 0x1.d5c216b4fbb94p-3, 0x1.95cbb0be377aep-1, 0x1.dc1bca0abec7bp-3,
    0x1.948b0fcd6e9e0p-1, 0x1.e27076e2af2e8p-3, 0x1.934c67f9b2ce6p-1, 0x1.e8c0252aa5a60p-3,
    0x1.920fb49d0e229p-1, 0x1.ef0adcbdc5935p-3, 0x1.90d4f120190d5p-1, 0x1.f550a564b7b37p-3,
    0x1.8f9c18f9c18fap-1, 0x1.fb9186d5e3e29p-3, 0x1.8e6527af1373fp-1, 0x1.00e6c45ad501dp-2,
    0x1.8d3018d3018d3p-1, 0x1.0402594b4d041p-2, 0x1.8bfce8062ff3ap-1, 0x1.071b85fcd590dp-2,
    0x1.8acb90f6bf3aap-1, 0x1.0a324e27390e2p-2, 0x1.899c0f601899cp-1, 0x1.0d46b579ab74bp-2,
    0x1.886e5f0abb04ap-1, 0x1.1058bf9ae4ad4p-2, 0x1.87427bcc092b9p-1, 0x1.136870293a8b0p-2,
    0x1.8618618618618p-1, 0x1.1675cababa60fp-2, 0x1.84f00c2780614p-1, 0x1.1980d2dd4236fp-2,
    0x1.83c977ab2beddp-1, 0x1.1c898c16999fbp-2, 0x1.82a4a0182a4a0p-1, 0x1.1f8ff9e48a2f3p-2,
    0x1.8181818181818p-1, 0x1.22941fbcf7966p-2, 0x1.8060180601806p-1, 0x1.2596010df763ap-2,
    0x1.7f405fd017f40p-1, 0x1.2895a13de86a4p-2, 0x1.7e225515a4f1dp-1, 0x1.2b9303ab89d25p-2,
    0x1.7d05f417d05f4p-1, 0x1.2e8e2bae11d31p-2, 0x1.7beb3922e017cp-1, 0x1.31871c9544185p-2,
    0x1.7ad2208e0ecc3p-1, 0x1.347dd9a987d56p-2, 0x1.79baa6bb6398bp-1, 0x1.3772662bfd85cp-2,
    0x1.78a4c8178a4c8p-1, 0x1.3a64c556945eap-2, 0x1.77908119ac60dp-1, 0x1.3d54fa5c1f710p-2,
    0x1.767dce434a9b1p-1, 0x1.404308686a7e4p-2, 0x1.756cac201756dp-1, 0x1.432ef2a04e813p-2,
};

__device__ __forceinline__ double log_fast(double x, const double* lds_tab) {
  const uint64_t ix = __builtin_bit_cast(uint64_t, x);
  const uint32_t h = (uint32_t)(ix >> 32);
  const uint32_t t = h - LOG_OFF_HI;
  const int k = (int)t >> 20;
  const uint32_t i = (t >> 12) & (LOG_TAB_N - 1);
  const double z = __builtin_bit_cast(double, ((uint64_t)(h - (t & 0xfff00000u)) << 32) | (uint32_t)ix);
  const double2 e = reinterpret_cast<const double2*>(lds_tab + EXP_TAB_N)[i];  // (invc, logc)
  const double r = __builtin_fma(z, e.x, -1.0);
  const double kd = (double)k;
  double p = __builtin_fma(r, -1.0 / 6.0, 1.0 / 5.0);
  p = __builtin_fma(p, r, -1.0 / 4.0);
  p = __builtin_fma(p, r, 1.0 / 3.0);
  p = __builtin_fma(p, r, -0.5);
  const double lp = __builtin_fma(r * r, p, r);  // log1p(r)
  return __builtin_fma(kd, LOG_LN2_HI, e.y) + __builtin_fma(kd, LOG_LN2_LO, lp);
}

// ---- cos(2 pi u) of the 53-bit uniform u53(lo, hi) = v 2^-53, v = (hi:lo) >> 11 (draw_eta's
// Box-Muller angle): the quadrant from v's top 2 bits, a = 2 pi j / 1024 from the next 8 (LDS table
// of (cos a, sin a)), delta = 2 pi (the low 43 bits) 2^-53 < 2 pi / 1024, and
// cos(a + delta) = C (1 + (cos delta - 1)) - S sin delta with the quadrant's (C, S) = (cos, sin) a
// rotated; cos delta - 1 and sin delta by Taylor polynomials (truncation < 1e-19).  ~27 VALU
// instead of ocml cospi's 66; <= ~2 ulp (tools/gen_log_table.py makes the table).
constexpr int COS_TAB_N = 256;
constexpr int FAST_TAB_N3 = FAST_TAB_N + 2 * COS_TAB_N;  // with the cos table (trivariate kernels)
__device__ constexpr double COS_TAB[2 * COS_TAB_N] = {  // (cos, sin) of 2 pi j / 1024
    0x1.0000000000000p+0, 0x0.0p+0, 0x1.fffd8858e8a92p-1, 0x1.921f0fe670071p-8,
    0x1.fff62169b92dbp-1, 0x1.921d1fcdec784p-7, 0x1.ffe9cb44b51a1p-1, 0x1.2d936bbe30efdp-6,
    0x1.ffd886084cd0dp-1, 0x1.92155f7a3667ep-6, 0x1.ffc251df1d3f8p-1, 0x1.f693731d1cf01p-6,
    0x1.ffa72effef75dp-1, 0x1.2d865759455cdp-5, 0x1.ff871dadb81dfp-1, 0x1.5fc00d290cd43p-5,
    0x1.ff621e3796d7ep-1, 0x1.91f65f10dd814p-5, 0x1.ff3830f8d575cp-1, 0x1.c428d12c0d7e3p-5,
    0x1.ff095658e71adp-1, 0x1.f656e79f820e0p-5, 0x1.fed58ecb673c4p-1, 0x1.1440134d709b3p-4,
    0x1.fe9cdad01883ap-1, 0x1.2d52092ce19f6p-4, 0x1.fe5f3af2e3940p-1, 0x1.4661179272096p-4,
    0x1.fe1cafcbd5b09p-1, 0x1.5f6d00a9aa419p-4, 0x1.fdd539ff1f456p-1, 0x1.787586a5d5b21p-4,
    0x1.fd88da3d12526p-1, 0x1.917a6bc29b42cp-4, 0x1.fd37914220b84p-1, 0x1.aa7b724495c03p-4,
    0x1.fce15fd6da67bp-1, 0x1.c3785c79ec2d5p-4, 0x1.fc8646cfeb721p-1, 0x1.dc70ecbae9fc9p-4,
    0x1.fc26470e19fd3p-1, 0x1.f564e56a9730ep-4, 0x1.fbc1617e44186p-1, 0x1.072a047ba831dp-3,
    0x1.fb5797195d741p-1, 0x1.139f0cedaf577p-3, 0x1.fae8e8e46cfbbp-1, 0x1.20116d4ec7bcfp-3,
    0x1.fa7557f08a517p-1, 0x1.2c8106e8e613ap-3, 0x1.f9fce55adb2c8p-1, 0x1.38edbb0cd8d14p-3,
    0x1.f97f924c9099bp-1, 0x1.45576b1293e5ap-3, 0x1.f8fd5ffae41dbp-1, 0x1.51bdf8597c5f2p-3,
    0x1.f8764fa714ba9p-1, 0x1.5e214448b3fc6p-3, 0x1.f7ea629e63d6ep-1, 0x1.6a81304f64ab2p-3,
    0x1.f7599a3a12077p-1, 0x1.76dd9de50bf31p-3, 0x1.f6c3f7df5bbb7p-1, 0x1.83366e89c64c6p-3,
    0x1.f6297cff75cb0p-1, 0x1.8f8b83c69a60bp-3, 0x1.f58a2b1789e84p-1, 0x1.9bdcbf2dc4366p-3,
    0x1.f4e603b0b2f2dp-1, 0x1.a82a025b00451p-3, 0x1.f43d085ff92ddp-1, 0x1.b4732ef3d6722p-3,
    0x1.f38f3ac64e589p-1, 0x1.c0b826a7e4f63p-3, 0x1.f2dc9c9089a9dp-1, 0x1.ccf8cb312b286p-3,
    0x1.f2252f7763adap-1, 0x1.d934fe5454311p-3, 0x1.f168f53f7205dp-1, 0x1.e56ca1e101a1bp-3,
    0x1.f0a7efb9230d7p-1, 0x1.f19f97b215f1bp-3, 0x1.efe220c0b95ecp-1, 0x1.fdcdc1adfedf9p-3,
    0x1.ef178a3e473c2p-1, 0x1.04fb80e37fdaep-2, 0x1.ee482e25a9dbcp-1, 0x1.0b0d9cfdbdb90p-2,
    0x1.ed740e7684963p-1, 0x1.111d262b1f677p-2, 0x1.ec9b2d3c3bf84p-1, 0x1.172a0d7765177p-2,
    0x1.ebbd8c8df0b74p-1, 0x1.1d3443f4cdb3ep-2, 0x1.eadb2e8e7a88ep-1, 0x1.233bbabc3bb71p-2,
    0x1.e9f4156c62ddap-1, 0x1.294062ed59f06p-2, 0x1.e9084361df7f2p-1, 0x1.2f422daec0387p-2,
    0x1.e817bab4cd10dp-1, 0x1.35410c2e18152p-2, 0x1.e7227db6a9744p-1, 0x1.3b3cefa0414b7p-2,
    0x1.e6288ec48e112p-1, 0x1.4135c94176601p-2, 0x1.e529f04729ffcp-1, 0x1.472b8a5571054p-2,
    0x1.e426a4b2bc17ep-1, 0x1.4d1e24278e76ap-2, 0x1.e31eae870ce25p-1, 0x1.530d880af3c24p-2,
    0x1.e212104f686e5p-1, 0x1.58f9a75ab1fddp-2, 0x1.e100cca2980acp-1, 0x1.5ee27379ea693p-2,
    0x1.dfeae622dbe2bp-1, 0x1.64c7ddd3f27c6p-2, 0x1.ded05f7de47dap-1, 0x1.6aa9d7dc77e17p-2,
    0x1.ddb13b6ccc23cp-1, 0x1.7088530fa459fp-2, 0x1.dc8d7cb410260p-1, 0x1.766340f2418f6p-2,
    0x1.db6526238a09bp-1, 0x1.7c3a9311dcce7p-2, 0x1.da383a9668988p-1, 0x1.820e3b04eaac4p-2,
    0x1.d906bcf328d46p-1, 0x1.87de2a6aea963p-2, 0x1.d7d0b02b8ecf9p-1, 0x1.8daa52ec8a4b0p-2,
    0x1.d696173c9e68bp-1, 0x1.9372a63bc93d7p-2, 0x1.d556f52e93eb1p-1, 0x1.993716141bdffp-2,
    0x1.d4134d14dc93ap-1, 0x1.9ef7943a8ed8ap-2, 0x1.d2cb220e0ef9fp-1, 0x1.a4b4127dea1e5p-2,
    0x1.d17e7743e35dcp-1, 0x1.aa6c82b6d3fcap-2, 0x1.d02d4feb2bd92p-1, 0x1.b020d6c7f4009p-2,
    0x1.ced7af43cc773p-1, 0x1.b5d1009e15cc0p-2, 0x1.cd7d9898b32f6p-1, 0x1.bb7cf2304bd01p-2,
    0x1.cc1f0f3fcfc5cp-1, 0x1.c1249d8011ee7p-2, 0x1.cabc169a0b900p-1, 0x1.c6c7f4997000bp-2,
    0x1.c954b213411f5p-1, 0x1.cc66e9931c45ep-2, 0x1.c7e8e52233cf3p-1, 0x1.d2016e8e9db5bp-2,
    0x1.c678b3488739bp-1, 0x1.d79775b86e389p-2, 0x1.c5042012b6907p-1, 0x1.dd28f1481cc58p-2,
    0x1.c38b2f180bdb1p-1, 0x1.e2b5d3806f63bp-2, 0x1.c20de3fa971b0p-1, 0x1.e83e0eaf85114p-2,
    0x1.c08c426725549p-1, 0x1.edc1952ef78d6p-2, 0x1.bf064e15377ddp-1, 0x1.f3405963fd067p-2,
    0x1.bd7c0ac6f952ap-1, 0x1.f8ba4dbf89abap-2, 0x1.bbed7c49380eap-1, 0x1.fe2f64be71210p-2,
    0x1.ba5aa673590d2p-1, 0x1.01cfc874c3eb7p-1, 0x1.b8c38d27504e9p-1, 0x1.0485626ae221ap-1,
    0x1.b728345196e3ep-1, 0x1.073879922ffeep-1, 0x1.b5889fe921405p-1, 0x1.09e907417c5e1p-1,
    0x1.b3e4d3ef55712p-1, 0x1.0c9704d5d898fp-1, 0x1.b23cd470013b4p-1, 0x1.0f426bb2a8e7ep-1,
    0x1.b090a58150200p-1, 0x1.11eb3541b4b23p-1, 0x1.aee04b43c1474p-1, 0x1.14915af336cebp-1,
    0x1.ad2bc9e21d511p-1, 0x1.1734d63dedb49p-1, 0x1.ab7325916c0d4p-1, 0x1.19d5a09f2b9b8p-1,
    0x1.a9b66290ea1a3p-1, 0x1.1c73b39ae68c8p-1, 0x1.a7f58529fe69dp-1, 0x1.1f0f08bbc861bp-1,
    0x1.a63091b02fae2p-1, 0x1.21a799933eb59p-1, 0x1.a4678c8119ac8p-1, 0x1.243d5fb98ac1fp-1,
    0x1.a29a7a0462782p-1, 0x1.26d054cdd12dfp-1, 0x1.a0c95eabaf937p-1, 0x1.2960727629ca8p-1,
    0x1.9ef43ef29af94p-1, 0x1.2bedb25faf3eap-1, 0x1.9d1b1f5ea80d5p-1, 0x1.2e780e3e8ea17p-1,
    0x1.9b3e047f38741p-1, 0x1.30ff7fce17035p-1, 0x1.995cf2ed80d22p-1, 0x1.338400d0c8e57p-1,
    0x1.9777ef4c7d742p-1, 0x1.36058b10659f3p-1, 0x1.958efe48e6dd7p-1, 0x1.3884185dfeb22p-1,
    0x1.93a22499263fbp-1, 0x1.3affa292050b9p-1, 0x1.91b166fd49da2p-1, 0x1.3d78238c58344p-1,
    0x1.8fbcca3ef940dp-1, 0x1.3fed9534556d4p-1, 0x1.8dc45331698ccp-1, 0x1.425ff178e6bb1p-1,
    0x1.8bc806b151741p-1, 0x1.44cf325091dd6p-1, 0x1.89c7e9a4dd4aap-1, 0x1.473b51b987347p-1,
    0x1.87c400fba2ebfp-1, 0x1.49a449b9b0939p-1, 0x1.85bc51ae958ccp-1, 0x1.4c0a145ec0004p-1,
    0x1.83b0e0bff976ep-1, 0x1.4e6cabbe3e5e9p-1, 0x1.81a1b33b57accp-1, 0x1.50cc09f59a09bp-1,
    0x1.7f8ece3571771p-1, 0x1.5328292a35596p-1, 0x1.7d7836cc33db2p-1, 0x1.5581038975137p-1,
    0x1.7b5df226aafafp-1, 0x1.57d69348ceca0p-1, 0x1.79400574f55e5p-1, 0x1.5a28d2a5d7250p-1,
    0x1.771e75f037261p-1, 0x1.5c77bbe65018cp-1, 0x1.74f948da8d28dp-1, 0x1.5ec3495837074p-1,
    0x1.72d0837efff96p-1, 0x1.610b7551d2cdfp-1, 0x1.70a42b3176d7ap-1, 0x1.63503a31c1be9p-1,
    0x1.6e74454eaa8afp-1, 0x1.6591925f0783dp-1, 0x1.6c40d73c18275p-1, 0x1.67cf78491af10p-1,
    0x1.6a09e667f3bcdp-1, 0x1.6a09e667f3bcdp-1, 0x1.67cf78491af10p-1, 0x1.6c40d73c18275p-1,
    0x1.6591925f0783dp-1, 0x1.6e74454eaa8afp-1, 0x1.63503a31c1be9p-1, 0x1.70a42b3176d7ap-1,
    0x1.610b7551d2cdfp-1, 0x1.72d0837efff96p-1, 0x1.5ec3495837074p-1, 0x1.74f948da8d28dp-1,
    0x1.5c77bbe65018cp-1, 0x1.771e75f037261p-1, 0x1.5a28d2a5d7250p-1, 0x1.79400574f55e5p-1,
    0x1.57d69348ceca0p-1, 0x1.7b5df226aafafp-1, 0x1.5581038975137p-1, 0x1.7d7836cc33db2p-1,
    0x1.5328292a35596p-1, 0x1.7f8ece3571771p-1, 0x1.50cc09f59a09bp-1, 0x1.81a1b33b57accp-1,
    0x1.4e6cabbe3e5e9p-1, 0x1.83b0e0bff976ep-1, 0x1.4c0a145ec0004p-1, 0x1.85bc51ae958ccp-1,
    0x1.49a449b9b0939p-1, 0x1.87c400fba2ebfp-1, 0x1.473b51b987347p-1, 0x1.89c7e9a4dd4aap-1,
    0x1.44cf325091dd6p-1, 0x1.8bc806b151741p-1, 0x1.425ff178e6bb1p-1, 0x1.8dc45331698ccp-1,
    0x1.3fed9534556d4p-1, 0x1.8fbcca3ef940dp-1, 0x1.3d78238c58344p-1, 0x1.91b166fd49da2p-1,
    0x1.3affa292050b9p-1, 0x1.93a22499263fbp-1, 0x1.3884185dfeb22p-1, 0x1.958efe48e6dd7p-1,
    0x1.36058b10659f3p-1, 0x1.9777ef4c7d742p-1, 0x1.338400d0c8e57p-1, 0x1.995cf2ed80d22p-1,
    0x1.30ff7fce17035p-1, 0x1.9b3e047f38741p-1, 0x1.2e780e3e8ea17p-1, 0x1.9d1b1f5ea80d5p-1,
    0x1.2bedb25faf3eap-1, 0x1.9ef43ef29af94p-1, 0x1.2960727629ca8p-1, 0x1.a0c95eabaf937p-1,
    0x1.26d054cdd12dfp-1, 0x1.a29a7a0462782p-1, 0x1.243d5fb98ac1fp-1, 0x1.a4678c8119ac8p-1,
    0x1.21a799933eb59p-1, 0x1.a63091b02fae2p-1, 0x1.1f0f08bbc861bp-1, 0x1.a7f58529fe69dp-1,
    0x1.1c73b39ae68c8p-1, 0x1.a9b66290ea1a3p-1, 0x1.19d5a09f2b9b8p-1, 0x1.ab7325916c0d4p-1,
    0x1.1734d63dedb49p-1, 0x1.ad2bc9e21d511p-1, 0x1.14915af336cebp-1, 0x1.aee04b43c1474p-1,
    0x1.11eb3541b4b23p-1, 0x1.b090a58150200p-1, 0x1.0f426bb2a8e7ep-1, 0x1.b23cd470013b4p-1,
    0x1.0c9704d5d898fp-1, 0x1.b3e4d3ef55712p-1, 0x1.09e907417c5e1p-1, 0x1.b5889fe921405p-1,
    0x1.073879922ffeep-1, 0x1.b728345196e3ep-1, 0x1.0485626ae221ap-1, 0x1.b8c38d27504e9p-1,
    0x1.01cfc874c3eb7p-1, 0x1.ba5aa673590d2p-1, 0x1.fe2f64be71210p-2, 0x1.bbed7c49380eap-1,
    0x1.f8ba4dbf89abap-2, 0x1.bd7c0ac6f952ap-1, 0x1.f3405963fd067p-2, 0x1.bf064e15377ddp-1,
    0x1.edc1952ef78d6p-2, 0x1.c08c426725549p-1, 0x1.e83e0eaf85114p-2, 0x1.c20de3fa971b0p-1,
    0x1.e2b5d3806f63bp-2, 0x1.c38b2f180bdb1p-1, 0x1.dd28f1481cc58p-2, 0x1.c5042012b6907p-1,
    0x1.d79775b86e389p-2, 0x1.c678b3488739bp-1, 0x1.d2016e8e9db5bp-2, 0x1.c7e8e52233cf3p-1,
    0x1.cc66e9931c45ep-2, 0x1.c954b213411f5p-1, 0x1.c6c7f4997000bp-2, 0x1.cabc169a0b900p-1,
    0x1.c1249d8011ee7p-2, 0x1.cc1f0f3fcfc5cp-1, 0x1.bb7cf2304bd01p-2, 0x1.cd7d9898b32f6p-1,
    0x1.b5d1009e15cc0p-2, 0x1.ced7af43cc773p-1, 0x1.b020d6c7f4009p-2, 0x1.d02d4feb2bd92p-1,
    0x1.aa6c82b6d3fcap-2, 0x1.d17e7743e35dcp-1, 0x1.a4b4127dea1e5p-2, 0x1.d2cb220e0ef9fp-1,
    0x1.9ef7943a8ed8ap-2, 0x1.d4134d14dc93ap-1, 0x1.993716141bdffp-2, 0x1.d556f52e93eb1p-1,
    0x1.9372a63bc93d7p-2, 0x1.d696173c9e68bp-1, 0x1.8daa52ec8a4b0p-2, 0x1.d7d0b02b8ecf9p-1,
    0x1.87de2a6aea963p-2, 0x1.d906bcf328d46p-1, 0x1.820e3b04eaac4p-2, 0x1.da383a9668988p-1,
    0x1.7c3a9311dcce7p-2, 0x1.db6526238a09bp-1, 0x1.766340f2418f6p-2, 0x1.dc8d7cb410260p-1,
    0x1.7088530fa459fp-2, 0x1.ddb13b6ccc23cp-1, 0x1.6aa9d7dc77e17p-2, 0x1.ded05f7de47dap-1,
    0x1.64c7ddd3f27c6p-2, 0x1.dfeae622dbe2bp-1, 0x1.5ee27379ea693p-2, 0x1.e100cca2980acp-1,
    0x1.58f9a75ab1fddp-2, 0x1.e212104f686e5p-1, 0x1.530d880af3c24p-2, 0x1.e31eae870ce25p-1,
    0x1.4d1e24278e76ap-2, 0x1.e426a4b2bc17ep-1, 0x1.472b8a5571054p-2, 0x1.e529f04729ffcp-1,
    0x1.4135c94176601p-2, 0x1.e6288ec48e112p-1, 0x1.3b3cefa0414b7p-2, 0x1.e7227db6a9744p-1,
    0x1.35410c2e18152p-2, 0x1.e817bab4cd10dp-1, 0x1.2f422daec0387p-2, 0x1.e9084361df7f2p-1,
    0x1.294062ed59f06p-2, 0x1.e9f4156c62ddap-1, 0x1.233bbabc3bb71p-2, 0x1.eadb2e8e7a88ep-1,
    0x1.1d3443f4cdb3ep-2, 0x1.ebbd8c8df0b74p-1, 0x1.172a0d7765177p-2, 0x1.ec9b2d3c3bf84p-1,
    0x1.111d262b1f677p-2, 0x1.ed740e7684963p-1, 0x1.0b0d9cfdbdb90p-2, 0x1.ee482e25a9dbcp-1,
    0x1.04fb80e37fdaep-2, 0x1.ef178a3e473c2p-1, 0x1.fdcdc1adfedf9p-3, 0x1.efe220c0b95ecp-1,
    0x1.f19f97b215f1bp-3, 0x1.f0a7efb9230d7p-1, 0x1.e56ca1e101a1bp-3, 0x1.f168f53f7205dp-1,
    0x1.d934fe5454311p-3, 0x1.f2252f7763adap-1, 0x1.ccf8cb312b286p-3, 0x1.f2dc9c9089a9dp-1,
    0x1.c0b826a7e4f63p-3, 0x1.f38f3ac64e589p-1, 0x1.b4732ef3d6722p-3, 0x1.f43d085ff92ddp-1,
    0x1.a82a025b00451p-3, 0x1.f4e603b0b2f2dp-1, 0x1.9bdcbf2dc4366p-3, 0x1.f58a2b1789e84p-1,
    0x1.8f8b83c69a60bp-3, 0x1.f6297cff75cb0p-1, 0x1.83366e89c64c6p-3, 0x1.f6c3f7df5bbb7p-1,
    0x1.76dd9de50bf31p-3, 0x1.f7599a3a12077p-1, 0x1.6a81304f64ab2p-3, 0x1.f7ea629e63d6ep-1,
    0x1.5e214448b3fc6p-3, 0x1.f8764fa714ba9p-1, 0x1.51bdf8597c5f2p-3, 0x1.f8fd5ffae41dbp-1,
    0x1.45576b1293e5ap-3, 0x1.f97f924c9099bp-1, 0x1.38edbb0cd8d14p-3, 0x1.f9fce55adb2c8p-1,
    0x1.2c8106e8e613ap-3, 0x1.fa7557f08a517p-1, 0x1.20116d4ec7bcfp-3, 0x1.fae8e8e46cfbbp-1,
    0x1.139f0cedaf577p-3, 0x1.fb5797195d741p-1, 0x1.072a047ba831dp-3, 0x1.fbc1617e44186p-1,
    0x1.f564e56a9730ep-4, 0x1.fc26470e19fd3p-1, 0x1.dc70ecbae9fc9p-4, 0x1.fc8646cfeb721p-1,
    0x1.c3785c79ec2d5p-4, 0x1.fce15fd6da67bp-1, 0x1.aa7b724495c03p-4, 0x1.fd37914220b84p-1,
    0x1.917a6bc29b42cp-4, 0x1.fd88da3d12526p-1, 0x1.787586a5d5b21p-4, 0x1.fdd539ff1f456p-1,
    0x1.5f6d00a9aa419p-4, 0x1.fe1cafcbd5b09p-1, 0x1.4661179272096p-4, 0x1.fe5f3af2e3940p-1,
    0x1.2d52092ce19f6p-4, 0x1.fe9cdad01883ap-1, 0x1.1440134d709b3p-4, 0x1.fed58ecb673c4p-1,
    0x1.f656e79f820e0p-5, 0x1.ff095658e71adp-1, 0x1.c428d12c0d7e3p-5, 0x1.ff3830f8d575cp-1,
    0x1.91f65f10dd814p-5, 0x1.ff621e3796d7ep-1, 0x1.5fc00d290cd43p-5, 0x1.ff871dadb81dfp-1,
    0x1.2d865759455cdp-5, 0x1.ffa72effef75dp-1, 0x1.f693731d1cf01p-6, 0x1.ffc251df1d3f8p-1,
    0x1.92155f7a3667ep-6, 0x1.ffd886084cd0dp-1, 0x1.2d936bbe30efdp-6, 0x1.ffe9cb44b51a1p-1,
    0x1.921d1fcdec784p-7, 0x1.fff62169b92dbp-1, 0x1.921f0fe670071p-8, 0x1.fffd8858e8a92p-1,
};

__device__ __forceinline__ double cos2pi_u53(uint32_t lo, uint32_t hi, const double* lds_tab) {
  constexpr double TWO_PI = 0x1.921fb54442d18p+2;
  const double dl = __builtin_fma((double)(hi & 0x3fffffu), TWO_PI * 0x1.0p-32, (double)(lo >> 11) * (TWO_PI * 0x1.0p-53));
  const double2 cs = reinterpret_cast<const double2*>(lds_tab + FAST_TAB_N)[(hi >> 22) & (COS_TAB_N - 1)];
  const bool swap = (hi >> 30) & 1u;  // quadrants 1, 3: (C, S) = (-+sin, +-cos)
  double C = swap ? cs.y : cs.x;
  double S = swap ? cs.x : cs.y;
  // sign of C: quadrants 1, 2 (hi bits 31 ^ 30); sign of S: quadrants 2, 3 (hi bit 31)
  const uint64_t cneg = (uint64_t)((hi ^ (hi << 1)) & 0x80000000u) << 32;
  const uint64_t sneg = (uint64_t)(hi & 0x80000000u) << 32;
  C = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, C) ^ cneg);
  S = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, S) ^ sneg);
  const double d2 = dl * dl;
  double p = __builtin_fma(d2, -1.0 / 720.0, 1.0 / 24.0);
  p = __builtin_fma(p, d2, -0.5);
  const double cm1 = p * d2;                                   // cos delta - 1
  const double sn = __builtin_fma(d2 * dl, __builtin_fma(d2, 1.0 / 120.0, -1.0 / 6.0), dl);  // sin delta
  return __builtin_fma(-S, sn, __builtin_fma(C, cm1, C));
}

// Fills the LDS table of exp_fast / log_fast (FAST_TAB_N doubles; with_cos: FAST_TAB_N3, adding
// cos2pi_u53's) from nt threads.
__device__ __forceinline__ void fast_tab_fill(double* lds_tab, int tid, int nt, bool with_cos = false) {
  for (int j = tid; j < EXP_TAB_N; j += nt) lds_tab[j] = exp_tab_entry(j);
  for (int j = tid; j < 2 * LOG_TAB_N; j += nt) lds_tab[EXP_TAB_N + j] = LOG_TAB[j];
  if (with_cos)
    for (int j = tid; j < 2 * COS_TAB_N; j += nt) lds_tab[FAST_TAB_N + j] = COS_TAB[j];
}

}  // namespace clv
