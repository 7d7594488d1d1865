// chain_params.hpp -- device-side (float32) model parameters of a fixed-base
// kinematic tree, shared by every world of a simulator (read-only, uniform
// across a wave, so the compiler keeps them on the scalar path).
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
    int32_t parent;    // parent body (< own index), -1 = base
    // row topology for the lane-group kernels (group_tree.hpp), filled by
    // group_topology_words(): ancestor bit mask, subtree end (bodies are
    // numbered depth-first, the subtree of i is [i, end)), lane-order chain
    // segment (bits 0-7: distance to the segment head, 8-15: the head's
    // parent + 1, 16-23: segment nesting level)
    uint32_t anc;
    int32_t end;
    int32_t seg;
};
static_assert(sizeof(BodyF) == 40 * 4, "BodyF layout");

enum : int32_t { kHasDamping = 1, kHasLimits = 2, kHasFriction = 4 };

struct ChainF {
    int32_t n;
    int32_t flags;     // kHas* bits
    // lane-group kernels: bits 0-7 body whose origin is the common frame's,
    // 8-15 segment nesting levels, 16-23 Hillis-Steele steps of the segmented
    // scans; gtopo2: bits 0-7 the head parent of every level-1 segment + 1
    // when there is exactly one (a DPP broadcast replaces the shuffle), 8-15
    // the end of every subtree that ends before n + 1 when there is exactly
    // one, bit 16 set when some subtree ends before n
    int32_t gtopo;
    int32_t gtopo2;
    float g[4];        // gravity in the base frame
    BodyF b[kMaxBodies];
};

// Per-dof actuation of a world's joint.  Force / Servo are DART actuator
// types; PidPos / PidVel are joints in Position / Velocity control mode whose
// force comes from the JointController PID (a force actuator to the engine).
enum : uint8_t { kActForce = 0, kActServo = 1, kActPidPos = 2, kActPidVel = 3 };

// ignition::math::PID parameters of one joint (float32 copy of the fp64
// values; Joint::setPID, Joint.cpp:479-525).  Ranges with max < min disable
// the corresponding clamp (ign-math semantics).
struct PidF {
    float p, i, d, imax, imin, cmdmax, cmdmin, offset;
};

// PIDs of every dof of a simulator (kernel argument, passed by value).
struct PidSet {
    PidF g[kMaxKernelDofs];
};

// Kinematic topology as a compile-time constant: 4 bits per body holding
// parent + 1 (so 0 = the base).  Kernels are instantiated per topology.
using Topo = uint64_t;
constexpr Topo chain_topo(int n) {
    Topo t = 0;
    for (int i = 0; i < n; ++i) t |= static_cast<Topo>(i) << (4 * i);
    return t;
}
constexpr int parent_of(Topo t, int i) { return static_cast<int>((t >> (4 * i)) & 15u) - 1; }
// i has at least one child among bodies i+1..n-1
constexpr bool has_child(Topo t, int n, int i) {
    for (int k = i + 1; k < n; ++k)
        if (parent_of(t, k) == i) return true;
    return false;
}
// i is the highest-numbered child of its parent, i.e. the first one an
// inward (n-1 .. 0) pass reaches
constexpr bool first_inward(Topo t, int n, int i) {
    for (int k = i + 1; k < n; ++k)
        if (parent_of(t, k) == parent_of(t, i)) return false;
    return true;
}
// i == j or i is an ancestor of j
constexpr bool on_path(Topo t, int i, int j) {
    for (int k = j; k >= 0; k = parent_of(t, k))
        if (k == i) return true;
    return false;
}
// Fill the lane-group topology words of a depth-first numbered tree
// (P.n bodies, P.b[i].parent set).  The common frame's origin is the body
// half-way up the deepest chain (group_tree.hpp).
inline void group_topology_words(ChainF& P) {
    const int n = P.n;
    int depth[kMaxBodies] = {}, level[kMaxBodies] = {};
    int deepest = 0, levels = 0, maxh = 0;
    for (int i = 0; i < n; ++i) {
        const int pa = P.b[i].parent;
        depth[i] = (pa >= 0) ? depth[pa] + 1 : 0;
        if (depth[i] > depth[deepest]) deepest = i;
        uint32_t anc = 0;
        for (int k = pa; k >= 0; k = P.b[k].parent) anc |= 1u << (k & 31);
        P.b[i].anc = anc;
        int end = i + 1;
        while (end < n) {
            bool desc = false;
            for (int k = P.b[end].parent; k >= 0; k = P.b[k].parent) desc = desc || (k == i);
            if (!desc) break;
            ++end;
        }
        P.b[i].end = end;
        int h = 0;  // lanes i-h..i form a parent chain in lane order
        while (i - h > 0 && P.b[i - h].parent == i - h - 1) ++h;
        const int head = i - h, hp = P.b[head].parent;
        level[i] = (hp >= 0) ? level[hp] + 1 : 0;
        levels = level[i] > levels ? level[i] : levels;
        maxh = h > maxh ? h : maxh;
        P.b[i].seg = h | ((hp + 1) << 8) | (level[i] << 16);
    }
    int ref = deepest;
    while (depth[ref] > depth[deepest] / 2) ref = P.b[ref].parent;
    int steps = 0;  // Hillis-Steele steps of the segmented scans: 2^steps > maxh
    while ((1 << steps) <= maxh) ++steps;
    P.gtopo = ref | (levels << 8) | (steps << 16);
    int fix = -2, dend = -2;  // -2: none yet, -1: more than one
    bool diff = false;
    for (int i = 0; i < n; ++i) {
        const int hp = ((P.b[i].seg >> 8) & 0xff) - 1;
        if (level[i] == 1) fix = (fix == -2 || fix == hp) ? hp : -1;
        if (P.b[i].end < n) {
            diff = true;
            dend = (dend == -2 || dend == P.b[i].end) ? P.b[i].end : -1;
        }
    }
    const int fixw = (levels == 1 && fix >= 0) ? fix + 1 : 0;
    const int dendw = dend >= 0 ? dend + 1 : 0;
    P.gtopo2 = fixw | (dendw << 8) | ((diff ? 1 : 0) << 16);
}

// the Franka Panda: joints 1..7 in a chain, both fingers hang off the hand
constexpr Topo kPandaTopo = chain_topo(7) | (static_cast<Topo>(7) << 28) | (static_cast<Topo>(7) << 32);
// four 2-dof legs hanging off a floating base (models/quadruped.urdf):
// parents [-1, 0, -1, 2, -1, 4, -1, 6]
constexpr Topo kQuadrupedTopo = (static_cast<Topo>(1) << 4) | (static_cast<Topo>(3) << 12) |
                                (static_cast<Topo>(5) << 20) | (static_cast<Topo>(7) << 28);

}  // namespace mw
