// chain_params.hpp -- device-side (float32) model parameters of a fixed-base
// chain, shared by every world of a simulator (read-only, uniform across a
// wave, so the compiler keeps them on the scalar path).
#pragma once

#include <cstdint>

namespace mw {

constexpr int kMaxBodies = 48;      // model compiler limit
constexpr int kMaxKernelDofs = 12;  // chain kernels are instantiated for 1..12 dofs

// One moving body: the joint that connects it to its parent plus its inertia.
// 40 words (160 B); the first 16 are read by every substep's forward kinematics.
struct BodyF {
    float E[9];        // joint origin rotation in the parent frame (row-major)
    float r[3];        // joint origin translation in the parent frame
    float axis[3];     // joint axis, child frame
    int32_t jtype;     // 0 revolute, 1 prismatic
    float mass;
    float com[3];      // COM in the body frame
    float Io[6];       // rotational inertia about the body ORIGIN: xx yy zz xy xz yz
    float damping;     // viscous (implicit in the ABA, DART semantics)
    float friction;    // Coulomb (LCP row)
    float lower, upper;
    float effort;      // |tau| clip and servo impulse bound
    float vel_limit;   // servo command clip
    int32_t limited;   // position limits enforced (LCP row)
    float Ea[3];       // E * axis (prismatic translation direction in the parent)
    float pad_[4];
};
static_assert(sizeof(BodyF) == 40 * 4, "BodyF layout");

enum : int32_t { kHasDamping = 1, kHasLimits = 2, kHasFriction = 4 };

struct ChainF {
    int32_t n;
    int32_t flags;     // kHas* bits
    int32_t pad_[2];
    float g[4];        // gravity in the base frame
    BodyF b[kMaxBodies];
};

// Per-dof actuation inside the engine (DART actuator types).
enum : uint8_t { kActForce = 0, kActServo = 1 };

}  // namespace mw
