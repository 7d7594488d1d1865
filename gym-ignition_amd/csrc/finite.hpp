// finite.hpp -- a non-finite test that survives the kernels' finite-math
// build.  Built with -ffinite-math-only, isfinite() folds to true, and so
// does a plain exponent-bit test of an arithmetic result: the compiler knows
// such a value is finite and drops the comparison (checked in the ISA).  The
// bits go through an empty asm first, which is opaque to that reasoning and
// emits no instruction.
#pragma once

#include <cstdint>
#ifdef MW_HOST_TEST
#include <cmath>
#endif

namespace mw {
namespace dev {

__device__ __forceinline__ bool nonfinite_bits(float x) {
#ifdef MW_HOST_TEST
    return !std::isfinite(x);
#else
    uint32_t u = __float_as_uint(x);
    asm("" : "+v"(u));
    return (u & 0x7f800000u) == 0x7f800000u;
#endif
}

}  // namespace dev
}  // namespace mw
