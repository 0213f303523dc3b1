// Host-compiled check of csrc/philox.h (test infrastructure): the Random123 known-answer vectors
// and bit-identity of the hoisted SlotPhilox with the plain Philox4x32-10 counter form.
#include <cstdint>
#include <cstdio>
#include <initializer_list>
#define __host__
#define __device__
#define __forceinline__ inline
#define __builtin_amdgcn_logf(x) (x)
#define __builtin_amdgcn_sqrtf(x) (x)
#define __builtin_amdgcn_cosf(x) (x)
#define __builtin_amdgcn_sinf(x) (x)
#define __builtin_amdgcn_rsqf(x) (x)
#define __builtin_amdgcn_exp2f(x) (x)
#include "../../mcmc_clv_model_amd/csrc/philox.h"

int main() {
  using namespace clv;
  int bad = 0;
  const u32x4 k1 = philox4x32_10(u32x4{0, 0, 0, 0}, 0, 0);
  bad += !(k1.x == 0x6627e8d5u && k1.y == 0xe169c58du && k1.z == 0xbc57ac4cu && k1.w == 0x9b00dbd8u);
  const u32x4 k2 = philox4x32_10(u32x4{~0u, ~0u, ~0u, ~0u}, ~0u, ~0u);
  bad += !(k2.x == 0x408f276du && k2.y == 0x41c83b0eu && k2.z == 0xa20bc7c6u && k2.w == 0x6d5451fdu);
  const u32x4 k3 = philox4x32_10(u32x4{0x243f6a88u, 0x85a308d3u, 0x13198a2eu, 0x03707344u}, 0xa4093822u, 0x299f31d0u);
  bad += !(k3.x == 0xd16cfe09u && k3.y == 0x94fdccebu && k3.z == 0x5001e420u && k3.w == 0x24126ea1u);
  long checks = 0;
  for (uint32_t cust : {0u, 1u, 255u, 12345u, 0x7fffffffu, 0xffffffffu})
    for (uint32_t sw : {1u, 77u, 20000u})
      for (uint32_t k : {0u, 0xa4093822u, 0xffffffffu}) {
        const SlotPhilox ph(k, k * 3u + 1u, cust, sw);
        for (uint32_t slot = 0; slot < 64; ++slot) {
          const u32x4 a = ph(slot), b = customer_block(k, k * 3u + 1u, cust, sw, slot);
          bad += !(a.x == b.x && a.y == b.y && a.z == b.z && a.w == b.w);
          ++checks;
        }
      }
  std::printf("checks %ld mismatches %d\n", checks, bad);
  return bad != 0;
}
