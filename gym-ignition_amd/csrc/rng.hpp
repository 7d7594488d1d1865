// rng.hpp -- Philox4x32-10 (Random123) and its uniform float mapping, shared
// by the device tasks' resets and randomisation (kernels.hip, group_kernel.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mw {
namespace dev {

__device__ __forceinline__ void philox(uint32_t seed_lo, uint32_t seed_hi, uint32_t world,
                                       uint32_t episode, uint32_t (&out)[4], uint32_t block = 0u) {
    uint32_t c0 = world, c1 = episode, c2 = block, c3 = 0u, k0 = seed_lo, k1 = seed_hi;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
        const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}
__device__ __forceinline__ float unif(uint32_t x, float lo, float hi) {
    return lo + (hi - lo) * (static_cast<float>(x >> 8) * (1.f / 16777216.f));
}

}  // namespace dev
}  // namespace mw
