// pid.hpp -- the JointController PID update of the device kernels.
#pragma once

#include <hip/hip_runtime.h>

#include "chain_params.hpp"

namespace mw {
namespace dev {

// ignition::math::PID::Update [EXT: ign-math6, restated in oracle.c
// or_pid_update]; returns false (and leaves the state) for a non-finite error
__device__ __forceinline__ bool pid_update(const PidF& g, float err, float inv_dt, float dt, float& e_last,
                                           float& ierr, float& cmd) {
    // exponent-bits test: the kernels are built finite-math-only, where
    // isfinite() folds to true
    if ((__float_as_uint(err) & 0x7f800000u) == 0x7f800000u) return false;
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
