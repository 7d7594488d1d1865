// pid.hpp -- the JointController PID update of the device kernels.
#pragma once

#include <hip/hip_runtime.h>

#include "chain_params.hpp"
#include "finite.hpp"

namespace mw {
namespace dev {

// ignition::math::PID::Update [EXT: ign-math6, restated in oracle.c
// or_pid_update]; returns false (and leaves the state) for a non-finite error
__device__ __forceinline__ bool pid_update(const PidF& g, float err, float inv_dt, float dt, float& e_last,
                                           float& ierr, float& cmd) {
    // the kernels are built finite-math-only: finite.hpp's exponent-bit test
    if (nonfinite_bits(err)) return false;
    const float pterm = g.p * err;
    ierr = ierr + g.i * dt * err;
    if (g.imax >= g.imin) ierr = fminf(fmaxf(ierr, g.imin), g.imax);
    const float derr = (err - e_last) * inv_dt;
    e_last = err;
    float u = -pterm - ierr - g.d * derr + g.offset;
    if (g.cmdmax >= g.cmdmin) u = fminf(fmaxf(u, g.cmdmin), g.cmdmax);
    cmd = u;
    return true;
}

}  // namespace dev
}  // namespace mw
