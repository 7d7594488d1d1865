// wave_tree.hpp -- one engine step of an articulated model on a floating
// base, ONE WORLD PER WAVEFRONT (large trees: the iCub-class models of
// BASELINE config 5).  Same physics as float_tree.hpp / oracle.c
// or_float_step (DART 6 World::step restated [EXT]); different mapping:
//
//   ABA              level-parallel (runtime topology, bodies in depth-first
//                    order): lane = body, the passes walk the tree by depth
//                    level; child -> parent sums go through per-parent LDS
//                    accumulators one sibling rank at a time (deterministic).
//                    Per-body records (R, p, U, psi, depth, world pose) are
//                    left in LDS for the later phases (uniform broadcasts).
//   lane phases      joint commands / PID (lane = dof), contact detection
//                    (lane = slot), row responses M^-1 J^T (lane = row, contact
//                    and joint rows in one pass; each walks its body's
//                    ancestor mask to the base, then the outward pass with a
//                    per-lane stack indexed by body depth), the nu update
//                    (lane = component).
//   Delassus         J (M^-1 J^T)^T on the matrix cores (32x32x2 f32 MFMA
//                    tiles), rearranged so lane c holds column c in registers.
//   PGS              rows in order (the oracle's order); impulses uniform in
//                    registers, the residual sum_c A_rc x_c distributed over
//                    the lanes and updated by one column per row.
//
// Capacities (checked on the host): bodies <= MAXN, tree depth <= kWaveMaxDepth,
// contact slots <= 32, active rows <= 64 per step (beyond: the step's extra
// rows are dropped and counted in the world's overflow counter).
#pragma once

#include "float_tree.hpp"

namespace mw {
namespace dev {

// Which register widths of the exact solve take the matrix-core LDL^T
// (wave_lcp.hpp kLcpMfma*): the <= 16-body instance every width (it runs
// without scratch: contacts 121.9 -> 115.7 us, quadruped 580 -> 567 us,
// profiles/r05ak), the larger instances the 17-32-row width only (the 64-row
// tiles made their legs slower through spills)
constexpr int kWaveLcpMfmaSmall = 7;  // kLcpMfmaAll
constexpr int kWaveLcpMfmaLarge = 2;  // kLcpMfma32
constexpr int kWaveLanes = 64;
constexpr int kWaveMaxRows = 64;
constexpr int kWaveMaxDepth = 12;
// warm-start record of the PGS impulses by row identity: contact slot rows
// 3 slot + d (d: normal, t1, t2), joint rows kWaveWarmJoint0 + 3 dof + t (t:
// limit, servo, Coulomb) -- oracle.h OR_WARM_* (its slot capacity is larger)
constexpr int kWaveWarmJoint0 = 3 * kMaxFloatSlots;
constexpr int kWaveWarmWords = kWaveWarmJoint0 + 3 * kMaxBodies;
// the record holds two such blocks: the final impulses, then the exact
// solve's stage-1 impulses (wave_lcp.hpp: DART's frictionless first stage)
constexpr int kWaveWarmRecord = 2 * kWaveWarmWords;

typedef float v16f __attribute__((ext_vector_type(16)));

struct alignas(16) F4 {
    float x, y, z, w;
};

// per-body record, 45 words (odd: lane-strided gathers of parent records are
// conflict-free); the articulated inertias live in the accumulators below
struct WaveBody {
    M3 R;        // joint transform (parent -> body)
    f3 p;
    SV U;        // AI S
    float psi;   // (S^T AI S)^-1
    float tt;    // total joint force (ABA u)
    SV V;        // body velocity, then acceleration
    M3 Rw;       // world pose (contact detection)
    f3 pw;
    int32_t depth;
    int32_t parent;  // the responses' outward walk reads it here (no model-block load per body)
    float pad_;
    f3 ax;       // joint axis (child frame) and type: the lane-varying walks read
    int32_t jt;  // them here instead of from the model block in global memory
};
static_assert(sizeof(WaveBody) == 45 * 4, "WaveBody layout");

// S and S^T of a body's joint from its LDS record (motion / proj of chain_dyn.hpp)
__device__ __forceinline__ SV motion_rec(const WaveBody& s, float q) {
    const bool rev = ((s.jt & 1) == 0);
    const float sw = rev ? q : 0.f, sv = rev ? 0.f : q;
    return {{s.ax.x * sw, s.ax.y * sw, s.ax.z * sw}, {s.ax.x * sv, s.ax.y * sv, s.ax.z * sv}};
}
__device__ __forceinline__ float proj_rec(const WaveBody& s, const SV& x) {
    const float dw = dot(s.ax, x.w), dv = dot(s.ax, x.v);
    return ((s.jt & 1) == 0) ? dw : dv;
}

// component-wise selects (a select between two records is lowered to a
// scratch round trip; a conditional record load to an exec-masked read that
// is waited on at once)
__device__ __forceinline__ f3 sel3(bool c, const f3& a, const f3& b) {
    return {c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z};
}
__device__ __forceinline__ SV selv(bool c, const SV& a, const SV& b) { return {sel3(c, a.w, b.w), sel3(c, a.v, b.v)}; }
__device__ __forceinline__ M3 selm(bool c, const M3& a, const M3& b) {
    M3 r;
#pragma unroll
    for (int k = 0; k < 9; ++k) r.m[k] = c ? a.m[k] : b.m[k];
    return r;
}

// child -> parent accumulator of the inward pass (48 words, float4-aligned):
// articulated inertia with DART's implicit joint damping, bias, and the
// non-implicit articulated inertia (models with damping: impulses propagate
// through it)
struct alignas(16) WaveAcc {
    SI I;
    SV B;
    SI In;
};
static_assert(sizeof(WaveAcc) == 48 * 4, "WaveAcc layout");

template <int MAXN>
struct WaveWorld {
    static constexpr int kNv = 6 + MAXN;
    static constexpr int kRowStride = kNv | 1;  // odd: lane-strided row access is conflict-free
    // odd like MJ: the response pass writes, and the Delassus tiles read, one
    // row per lane (a stride of 24/40/56 put 8 lanes on each bank)
    static constexpr int kJStride = kNv | 1;
    // the response stack's depth: the <= 16-body instance takes trees of
    // depth <= 10 (the host routes deeper ones to the 32-body instance), so
    // that its world record fits 4 waves per CU (LDS <= 40 KiB)
    static constexpr int kDepth = (MAXN <= 16) ? 10 : kWaveMaxDepth;
    WaveBody body[MAXN];
    // the inward ABA's accumulators are dead once the base solve has read
    // them; J is written from the response pass on: one LDS region
    union {
        WaveAcc acc[MAXN + 1];   // [MAXN] = the base
        alignas(16) float J[kWaveMaxRows][kJStride];
    };
    float q[MAXN], qd[MAXN], qdd[MAXN], tau[MAXN], vc[MAXN];
    uint32_t act[MAXN];
    float ext[MAXN + 1][6];      // this substep's world wrenches: [0] the base, [1 + i] body i (f, tau)
    float nu[kNv];
    float MJ[kWaveMaxRows][kRowStride];
    float b[kWaveMaxRows], lo[kWaveMaxRows], hi[kWaveMaxRows];
    F4 rc[kWaveMaxRows];         // PGS row constants {b, 1/A_rr, lo, hi}
    int32_t src[kWaveMaxRows];   // 3 slot + d, or kJointRow + 3 dof + type
    // contact slots
    float s_b[kMaxFloatSlots][3];   // body-frame point
    float s_xw[kMaxFloatSlots][3];  // world point
    float s_depth[kMaxFloatSlots];
    float s_R[kMaxFloatSlots][9];   // body rotation
    float s_x[kMaxFloatSlots][3];   // impulses (output)
    // per-lane outward stack of the responses: [depth][7][lane] (dv 6, u)
    alignas(16) float stack[kDepth][7][kWaveLanes];
    float xw[kWaveWarmRecord];   // warm-start impulses (RunArgs::warm): final, then stage 1
};

// The lane index through a volatile asm: every call is a fresh value, so the
// lane-dependent constants the phases derive from it (masks, identity
// patterns, LDS addresses) are formed where they are used instead of being
// hoisted out of the substep loop by LICM, where hundreds of them stayed live
// across the whole step and spilled to scratch.
#if defined(MW_HOST_TEST) || defined(MW_LANE_PLAIN)
__device__ __forceinline__ int lane_id() { return static_cast<int>(threadIdx.x & 63u); }
#else
__device__ __forceinline__ int lane_id() {
    int l;
    asm volatile("v_and_b32 %0, 63, %1" : "=v"(l) : "v"(threadIdx.x));
    return l;
}
#endif

// Phase timing (debug builds only: EXTRA=-DMW_WAVE_PROF, scripts/wave_prof.py):
// shader-clock cycles per phase, summed over the worlds of a launch.
constexpr int kWaveProfPhases = 22;  // [8] exact-LCP linear solves, [9] its rounds, [10] stage-2 solves,
                                     // [11] / [12] max solves / stage-2 solves of a world-step, [13] world-steps > 4 solves,
                                     // [14] cycles in the linear solves, [15] in the PGS sweeps / the exact solve,
                                     // [16] in the exact solve's per-stage sweeps, [17] in its stage 1,
                                     // [18] / [19] ABA pass 1 / inward, [20] the kernel's prologue (entry
                                     // to the first substep: state and warm-record loads)
#ifdef MW_WAVE_PROF
__device__ unsigned long long g_wave_prof[kWaveProfPhases];
// up to kDumpSlots hard exact LCPs (world-steps with >= 8 linear solves, or
// with -DMW_DUMP_FAIL the unconverged ones): n, A, b, lo, hi, kind, both warm
// records, both results (scripts/wave_prof.py, scripts/lcp_dump_check.py)
constexpr int kDumpSlots = 8;
constexpr int kWaveDumpFloats = 8 + 64 * 64 + 9 * 64;
__device__ float g_wave_dump[kDumpSlots * kWaveDumpFloats];
#ifdef MW_DUMP_FAIL
#define MW_DUMP_WHEN(ok, ns) (!(ok))
#else
#define MW_DUMP_WHEN(ok, ns) ((ns) >= 8)
#endif
__device__ unsigned int g_wave_dump_claim;
#define MW_PROF_T(var) const long long var = clock64()
#define MW_PROF_ACC(k, a, b) (prof[k] += static_cast<unsigned long long>((b) - (a)))
#else
#define MW_PROF_T(var)
#define MW_PROF_ACC(k, a, b)
#endif

// min(max(v, lo), hi) for lo <= hi (every PGS bound pair is ordered): one
// v_med3_f32 on the device
__device__ __forceinline__ float clamp_ordered(float v, float lo, float hi) {
#ifdef MW_HOST_TEST
    return fminf(fmaxf(v, lo), hi);
#else
    return __builtin_amdgcn_fmed3f(v, lo, hi);
#endif
}

__device__ __forceinline__ float read_lane(float x, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), l));
}

}  // namespace dev
}  // namespace mw
#include "wave_lcp.hpp"
namespace mw {
namespace dev {

// the whole wave runs these with identical values; lane 0 stores
#define MW_LANE0 if (lane_id() == 0)

// Floating-base ABA, level-parallel (runtime topology): lane i owns body i
// and keeps its quantities in registers; the passes walk the tree by depth
// level (all bodies of one level at once), so a step costs `levels` body
// updates instead of N.  Parent -> child data (velocity, world pose,
// acceleration) goes through the body records in LDS; child -> parent
// articulated inertias and biases are added into the parent's accumulator
// one sibling rank at a time, highest body index first (the order of the
// serial inward pass), so the sums are deterministic.  Every lane then has
// IA0 and B0 of the base (broadcast reads) and solves a0 itself.  Returns a0
// and leaves qdd_i in qdd_out (L.qdd, LDS) and the per-body records that the
// later phases read (R, p, U, psi, depth, Rw, pw) in L.body.
template <int MAXN>
__device__ __forceinline__ SV wave_aba(const ChainF* __restrict__ P, const FloatF* __restrict__ F, int N,
                                       const M3& R0, const f3& p0, const SV& V0, WaveWorld<MAXN>& L, Chol6& L0,
                                       float dt, float* qdd_out, bool ext, unsigned long long* prof) {
    (void)prof;
    MW_PROF_T(ta0);
    const int lane = lane_id();
    const bool own = lane < N;
    const int i = own ? lane : 0;
    const BodyF b = P->b[i];  // by value: one load up front, not one per level
    const int pa = b.parent;
    const int depth = own ? F->body_depth[i] : -1;
    const int srank = F->body_srank[i];
    const int levels = F->levels, fanout = F->fanout;
    const f3 gw = mk(F->g[0], F->g[1], F->g[2]);
    const int slot = (pa >= 0) ? pa : MAXN;  // accumulator of the parent (MAXN = the base)
    // accumulators start empty
    if (lane <= MAXN) L.acc[lane] = WaveAcc{};
    // joint transforms and joint velocities: independent of the parent, every
    // body at once
    M3 R, Rw;
    f3 p, pw;
    SV V, eta, B, Sq;
    float tau = 0.f;
    if (own) {
        joint_pose_tree(b, L.q, i, R, p);
        Sq = motion(b, L.qd[i]);
        L.body[i].ax = mk(b.axis[0], b.axis[1], b.axis[2]);
        L.body[i].jt = b.jtype;
        L.body[i].parent = pa;
    }
    // outward: velocities and world poses, the only parent chain, level by level
    for (int d = 0; d < levels; ++d) {
        if (depth == d) {
            // the parent's record loads unconditionally (the base: record 0, unused)
            const bool hp = pa >= 0;
            const int pai = hp ? pa : 0;
            const SV Vp = selv(hp, L.body[pai].V, V0);
            const M3 Rwp = selm(hp, L.body[pai].Rw, R0);
            const f3 pwp = sel3(hp, L.body[pai].pw, p0);
            V = ad_inv(R, p, Vp) + Sq;
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int c = 0; c < 3; ++c)
                    Rw.m[r * 3 + c] =
                        Rwp.m[r * 3] * R.m[c] + Rwp.m[r * 3 + 1] * R.m[3 + c] + Rwp.m[r * 3 + 2] * R.m[6 + c];
            pw = pwp + mul(Rwp, p);
            L.body[i].V = V;
            L.body[i].Rw = Rw;
            L.body[i].pw = pw;
        }
    }
    // velocity-product terms and bias forces: every body at once
    float qdi = 0.f;
    SV extB = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};  // -(this substep's world wrench), body frame
    if (own) {
        const SV Ve = ball_bias_velocity(b, L.qd, i, V);
        eta = {cross(Ve.w, Sq.w), cross(Ve.w, Sq.v) + cross(Ve.v, Sq.w)};
        B = rigid_bias(b.mass, mk(b.com[0], b.com[1], b.com[2]), inertia_origin(b, b.mass), V, mulT(Rw, gw));
        tau = L.tau[i];
        qdi = L.qd[i];
        if (ext) {
            // this substep's world wrenches (L.ext, mw_apply_link_wrench) enter
            // as the starting bias of each body's sum, in its own frame
            const float* e = L.ext[1 + i];
            extB = (-1.f) * SV{mulT(Rw, mk(e[3], e[4], e[5])), mulT(Rw, mk(e[0], e[1], e[2]))};
            L.acc[i].B = L.acc[i].B + extB;
        }
    }
    SV extB0 = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
    if (ext) {
        const float* e = L.ext[0];
        extB0 = (-1.f) * SV{mulT(R0, mk(e[3], e[4], e[5])), mulT(R0, mk(e[0], e[1], e[2]))};
        if (lane == 0) L.acc[MAXN].B = L.acc[MAXN].B + extB0;
    }
    MW_PROF_T(ta1);
    MW_PROF_ACC(18, ta0, ta1);
    // DART's implicit joint damping (Psi = (S^T AI S + dt d)^-1, force
    // tau - d qd) for the free motion; with damping the impulses use the
    // non-implicit articulated inertias, a second recursion (F->dual)
    const bool dual = F->dual != 0;
    // inward, deepest level first
    SV U, Un;
    float psi = 0.f, tt = 0.f, psin = 0.f;
    for (int d = levels - 1; d >= 0; --d) {
        const bool mine = (depth == d);
        SI c, cn;
        SV cb;
        if (mine) {
            SI AI = rigid(b, b.mass);
            AI += L.acc[i].I;
            const SV Bt = B + L.acc[i].B;
            U = ais(AI, b);
            psi = rcp(proj(b, U) + dt * b.damping);
            const SV AIeta = mul(AI, eta);
            tt = tau - b.damping * qdi - proj(b, AIeta + Bt);
            c = to_parent(R, p, downdate(AI, U, psi));
            cb = dad_inv(R, p, Bt + AIeta + (psi * tt) * U);
            if (dual) {
                SI AIn = rigid(b, b.mass);
                AIn += L.acc[i].In;
                Un = ais(AIn, b);
                psin = rcp(proj(b, Un));
                cn = to_parent(R, p, downdate(AIn, Un, psin));
            }
        }
        // children add into the parent's accumulator one sibling rank at a
        // time, highest body index first (a parent gathering its children's
        // slots instead measured slower: profiles/r05b)
        // (sibling ranks at one level are contiguous from 0: the rounds stop
        // at the level's own fan-out instead of the model's -- most levels of
        // a humanoid are chains, one round instead of five)
        for (int k = 0; k < fanout; ++k) {
            const bool me = mine && srank == k;
            if (__ballot(me) == 0ull) break;
            if (me) {
                WaveAcc& acc = L.acc[slot];
                SI I = acc.I;
                I += c;
                acc.I = I;
                acc.B = acc.B + cb;
                if (dual) {
                    SI In = acc.In;
                    In += cn;
                    acc.In = In;
                }
            }
        }
    }
    const SI IA0s = L.acc[MAXN].I, IA0ns = L.acc[MAXN].In;
    const SV B0s = L.acc[MAXN].B;
    (void)extB0;
    MW_PROF_T(ta2);
    MW_PROF_ACC(19, ta1, ta2);
    // a welded base (F->fixed: generic fixed-base trees) does not move: a0 = 0
    // and it absorbs every impulse (wave_response), V0 stays 0
    SV a0 = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
    if (!F->fixed) {
        SI IA0 = rigid_base(*F);
        IA0 += IA0s;
        const SV B0 = rigid_bias(F->mass, mk(F->com[0], F->com[1], F->com[2]),
                                 Sy{F->Io[0], F->Io[1], F->Io[2], F->Io[3], F->Io[4], F->Io[5]}, V0, mulT(R0, gw)) +
                      B0s;

        L0.factor(IA0);
        a0 = L0.solve(-1.f * B0);
        if (dual) {
            SI IA0n = rigid_base(*F);
            IA0n += IA0ns;
            L0.factor(IA0n);  // L0 leaves with the impulses' (non-implicit) base inertia
        }
    }
    // outward: accelerations (the V record now carries a)
    for (int d = 0; d < levels; ++d) {
        if (depth == d) {
            const SV ap = ad_inv(R, p, selv(pa >= 0, L.body[(pa >= 0) ? pa : 0].V, a0));
            const float qdd = psi * (tt - dot(U, ap));
            L.body[i].V = ap + eta + motion(b, qdd);
            qdd_out[i] = qdd;
        }
    }
    if (own) {
        WaveBody& s = L.body[i];
        s.R = R;
        s.p = p;
        // the responses are impulse dynamics; component selects (a select
        // between two SV objects is lowered to a scratch round trip)
        s.U = {{dual ? Un.w.x : U.w.x, dual ? Un.w.y : U.w.y, dual ? Un.w.z : U.w.z},
               {dual ? Un.v.x : U.v.x, dual ? Un.v.y : U.v.y, dual ? Un.v.z : U.v.z}};
        s.psi = dual ? psin : psi;
        s.tt = tt;
        s.depth = depth;
    }
    return a0;
}

// Per-lane response to a spatial impulse f on body k (k = -1: base) and/or
// a unit impulse on dof j: J = J_k^T f (generalized row), MJ = M^-1 (J^T + e_j).
// Writes J (if Jrow) and MJ to the lane's LDS rows and returns J nu.
// The path to the base comes from the model's ancestor masks (no dependent
// parent loads); on the outward pass a body whose parent is the previous
// body takes the parent's response from registers, so only branch points
// wait on the lane's LDS stack.
template <int MAXN>
__device__ __forceinline__ float wave_response(const ChainF* __restrict__ P, const FloatF* __restrict__ F, int N,
                                               WaveWorld<MAXN>& L, const Chol6& L0, int k, int j, const SV& f,
                                               float* Jrow, float* MJrow) {
    const int lane = lane_id();
    const int start = (k >= 0) ? k : j;
    const uint64_t path = (start >= 0) ? F->body_path[start] : uint64_t{0};
    for (int e = 0; e < WaveWorld<MAXN>::kJStride; ++e) Jrow[e] = 0.f;
    // inward along the path: articulated bias impulse Bi and the kinematic
    // force Fi (for J); u_i parked in the lane's depth stack
    SV Bi = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}}, Fi = Bi;
    if (k >= 0 || (k < 0 && j < 0)) { Bi = -1.f * f; Fi = f; }
    float jv = 0.f;
    // (unrolled by 2 like the outward walk below: the next path body's record
    // gathers are independent of this body's transform chain)
#pragma unroll 2
    for (uint64_t m = path; m != 0;) {
        const int i = 63 - __builtin_clzll(m);
        m &= ~(uint64_t{1} << i);
        const WaveBody& s = L.body[i];
        const float ji = proj_rec(s, Fi);
        Jrow[6 + i] = ji;
        jv += ji * L.nu[6 + i];
        const float u = ((i == j) ? 1.f : 0.f) - proj_rec(s, Bi);
        L.stack[s.depth][6][lane] = u;
        Bi = dad_inv(s.R, s.p, Bi + (s.psi * u) * s.U);
        Fi = dad_inv(s.R, s.p, Fi);
    }
    Jrow[0] = Fi.w.x; Jrow[1] = Fi.w.y; Jrow[2] = Fi.w.z; Jrow[3] = Fi.v.x; Jrow[4] = Fi.v.y; Jrow[5] = Fi.v.z;
    jv += Fi.w.x * L.nu[0] + Fi.w.y * L.nu[1] + Fi.w.z * L.nu[2] + Fi.v.x * L.nu[3] + Fi.v.y * L.nu[4] +
          Fi.v.z * L.nu[5];
    const SV dV0 = F->fixed ? SV{{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}} : L0.solve(-1.f * Bi);
    MJrow[0] = dV0.w.x; MJrow[1] = dV0.w.y; MJrow[2] = dV0.w.z;
    MJrow[3] = dV0.v.x; MJrow[4] = dV0.v.y; MJrow[5] = dV0.v.z;
    SV dv_prev = dV0;
    (void)P;
    // unrolled by 4: the next bodies' LDS records load while this one's
    // transform runs (the loop waited on each record's broadcast reads)
#pragma unroll 4
    for (int i = 0; i < N; ++i) {
        const WaveBody& s = L.body[i];
        const int pa = s.parent;
        SV dvp_in;
        if (pa == i - 1) {
            dvp_in = dv_prev;  // the previous body (or the base for i = 0)
        } else if (pa >= 0) {
            const int dp = L.body[pa].depth;
            dvp_in = {{L.stack[dp][0][lane], L.stack[dp][1][lane], L.stack[dp][2][lane]},
                      {L.stack[dp][3][lane], L.stack[dp][4][lane], L.stack[dp][5][lane]}};
        } else {
            dvp_in = dV0;
        }
        const SV dvp = ad_inv(s.R, s.p, dvp_in);
        // (an unconditional read here, a select instead of the masked read,
        // measured slower: 32.4k -> 34.5k cycles, profiles/r05ad)
        const float u = ((path >> i) & 1u) ? L.stack[s.depth][6][lane] : 0.f;
        const float mm = s.psi * (u - dot(s.U, dvp));
        MJrow[6 + i] = mm;
        const SV dv = dvp + motion_rec(s, mm);
        dv_prev = dv;
        float* st = &L.stack[s.depth][0][lane];
        st[0 * kWaveLanes] = dv.w.x; st[1 * kWaveLanes] = dv.w.y; st[2 * kWaveLanes] = dv.w.z;
        st[3 * kWaveLanes] = dv.v.x; st[4 * kWaveLanes] = dv.v.y; st[5 * kWaveLanes] = dv.v.z;
    }
    return jv;
}

// Projected Gauss-Seidel sweeps over the rows (see wave_step): impulses x[r]
// uniform in registers, residual w_c = sum_r A[c][r] x_r in lane c, rows in
// order, padded to blocks of 8 with inert rows.  TOL: end once a sweep changed
// no row's constraint velocity w_r = (A x)_r by more than pgs_tol -- measured
// in velocity space, where the redundant contact corners' null directions (A
// conditioned ~1e5 by CFM 1e-5: impulse changes there move nothing, and fp32
// round-off keeps them moving) do not count.  One wave max per sweep; a
// separate instance so the fixed-count solve pays nothing for it.
template <int MAXN, bool TOL>
__device__ __forceinline__ void wave_pgs(const WaveWorld<MAXN>& L, const float (&a)[kWaveMaxRows],
                                         float (&x)[kWaveMaxRows], int Rpad, int ncr, float mu, int pgs_iters,
                                         float pgs_tol) {
    for (int it = 0; it < pgs_iters; ++it) {
        float w = 0.f;
#pragma unroll
        for (int rb = 0; rb < kWaveMaxRows; rb += 8) {
            if (rb >= Rpad) break;
#pragma unroll
            for (int k = 0; k < 8; ++k) w += a[rb + k] * x[rb + k];
        }
        const float w_start = w;
        float h = 0.f;  // mu x_normal of the current contact (set by its normal row)
#pragma unroll
        for (int rb = 0; rb < kWaveMaxRows; rb += 8) {
            if (rb >= Rpad) break;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int r = rb + k;
                // dependent chain per row: lane read of w_r, one fma, the
                // clamp, one fma into w (x + b/A_rr and w - A[.][r] x_r are
                // formed off the chain)
                const F4 c = L.rc[r];
                const float xb = fmaf(c.x, c.y, x[r]);
                const float wpre = fmaf(-a[r], x[r], w);
                float v = fmaf(-read_lane(w, r), c.y, xb);
                if (r % 3 == 0) {
                    v = clamp_ordered(v, c.z, c.w);  // normal row (0, inf) or joint row
                    h = mu * v;                      // friction bound of this contact
                } else {  // friction row |x| <= mu x_normal, or joint row
                    const bool fr = r < ncr;
                    v = clamp_ordered(v, fr ? -h : c.z, fr ? h : c.w);
                }
                w = fmaf(a[r], v, wpre);
                x[r] = v;
            }
        }
        if (TOL) {
            if (wave_fmax(fabsf(w - w_start)) <= pgs_tol) break;
        }
    }
}

// One engine step of world L (state in L.q / L.qd / base; joint forces in
// L.tau).  Returns the active slot mask; *overflow += rows dropped.
template <int MAXN, bool CONS>
__device__ __forceinline__ uint32_t wave_step(const ChainF* __restrict__ P, const FloatF* __restrict__ F, int N,
                                              FreeState& base, WaveWorld<MAXN>& L, float dt, int pgs_iters,
                                              float pgs_tol, bool warm, int lcp_solves, float* qdd_out, int* overflow,
                                              int* unconverged, unsigned long long* prof, bool ext) {
    const int lane = lane_id();
    const int NV = 6 + N;
    MW_PROF_T(t0);
    const M3 R0 = quat_to_R(base.qw, base.qx, base.qy, base.qz);
    Chol6 L0;  // on return: the factorisation the impulses use
    const SV a0 = wave_aba<MAXN>(P, F, N, R0, base.p, base.V, L, L0, dt, qdd_out, ext, prof);
    MW_PROF_T(t1);
    MW_PROF_ACC(1, t0, t1);
    // integrateVelocities (lane e: nu component e)
    if (lane < NV) {
        float v;
        if (lane < 6) {
            const float a[6] = {a0.w.x, a0.w.y, a0.w.z, a0.v.x, a0.v.y, a0.v.z};
            const float V0[6] = {base.V.w.x, base.V.w.y, base.V.w.z, base.V.v.x, base.V.v.y, base.V.v.z};
            float ae = 0.f, ve = 0.f;
#pragma unroll
            for (int e = 0; e < 6; ++e) {
                ae = (lane == e) ? a[e] : ae;
                ve = (lane == e) ? V0[e] : ve;
            }
            v = ve + dt * ae;
        } else {
            v = L.qd[lane - 6] + dt * qdd_out[lane - 6];
        }
        L.nu[lane] = v;
    }

    // ---- contact detection (lane = slot) -----------------------------------
    uint32_t active = 0u;
    if (F->ground) {
        bool hit = false;
        if (lane < F->n_slots) {
            int sh = 0;
            while (sh + 1 < F->n_shapes && F->shape_slot0[sh + 1] <= lane) ++sh;
            const int c = lane - F->shape_slot0[sh];
            const int bi = F->shape_body[sh];
            M3 Rb;
            f3 pb;
            if (bi < 0) { Rb = R0; pb = base.p; }
            else { Rb = L.body[bi].Rw; pb = L.body[bi].pw; }
            const bool sphere = (F->shape_type[sh] == 1);
            const float* h = F->shape_size[sh];
            const float* SR = F->shape_R[sh];
            const f3 lp = shape_slot_point(F->shape_type[sh], h, shape_plane_normal(Rb, SR), c);
            const float lx = lp.x, ly = lp.y, lz = lp.z;
            f3 bb = {F->shape_p[sh][0] + SR[0] * lx + SR[1] * ly + SR[2] * lz,
                     F->shape_p[sh][1] + SR[3] * lx + SR[4] * ly + SR[5] * lz,
                     F->shape_p[sh][2] + SR[6] * lx + SR[7] * ly + SR[8] * lz};
            f3 xw = pb + mul(Rb, bb);
            float depth = -xw.z;
            if (sphere) {
                depth = h[0] - xw.z;
                xw.z -= h[0];
                bb = mulT(Rb, xw - pb);
            }
            if (depth > 0.f) {
                hit = true;
                L.s_b[lane][0] = bb.x; L.s_b[lane][1] = bb.y; L.s_b[lane][2] = bb.z;
                L.s_xw[lane][0] = xw.x; L.s_xw[lane][1] = xw.y; L.s_xw[lane][2] = xw.z;
                L.s_depth[lane] = depth;
#pragma unroll
                for (int e = 0; e < 9; ++e) L.s_R[lane][e] = Rb.m[e];
                L.s_x[lane][0] = L.s_x[lane][1] = L.s_x[lane][2] = 0.f;
            }
        }
        active = static_cast<uint32_t>(__ballot(hit));
    }

    // ---- rows: contacts (slot order), then joint rows (dof order) ----------
    // joint rows of dof `lane`: bit t of jbits = limit / servo / friction
    uint32_t jbits = 0u;
    float jb[3] = {0.f, 0.f, 0.f}, jlo[3] = {0.f, 0.f, 0.f}, jhi[3] = {0.f, 0.f, 0.f};
    if (CONS && lane < N) {
        const BodyF& b = P->b[lane];
        const float qdi = L.nu[6 + lane];
        if (b.limited) {
            float viol = L.q[lane] - b.lower;
            bool lim = false, up = false;
            if (viol <= 0.f) {
                lim = true;
            } else {
                viol = L.q[lane] - b.upper;
                if (viol >= 0.f) { lim = true; up = true; }
            }
            if (lim) {
                jbits |= 1u;
                jb[0] = fminf(fmaxf(-viol * kErp * rcp(dt), -kMaxErv), kMaxErv) - qdi;
                jlo[0] = up ? -kBig : 0.f;
                jhi[0] = up ? 0.f : kBig;
            }
        }
        if (L.act[lane] == kActServo) {
            const float vc = fminf(fmaxf(L.vc[lane], -b.vel_limit), b.vel_limit);
            if (vc - qdi != 0.f) {
                jbits |= 2u;
                jb[1] = vc - qdi;
                jhi[1] = b.effort * dt;
                jlo[1] = -jhi[1];
            }
        }
        if (b.friction != 0.f && qdi != 0.f) {
            jbits |= 4u;
            jb[2] = -qdi;
            jhi[2] = b.friction * dt;
            jlo[2] = -jhi[2];
        }
    }
    const int n_contact_rows = 3 * __builtin_popcount(active);
    // prefix count of the joint rows in dof order
    const int my_j = __builtin_popcount(jbits);
    int before = 0, total_j = 0;
    for (int d = 0; d < N; ++d) {
        const int cnt = __builtin_amdgcn_readlane(my_j, d);
        before += (d < lane) ? cnt : 0;
        total_j += cnt;
    }
    int R = n_contact_rows + total_j;
    if (R > kWaveMaxRows) {
        MW_LANE0 { *overflow += R - kWaveMaxRows; }
        R = kWaveMaxRows;
    }
    // contact rows: lane = slot -> rows 3 rank + d
    if (lane < 32 && ((active >> lane) & 1u)) {
        const int rank = __builtin_popcount(active & ((1u << lane) - 1u));
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            const int r = 3 * rank + d;
            if (r < R) {
                L.src[r] = 3 * lane + d;
                L.lo[r] = 0.f;
                L.hi[r] = kBig;
            }
        }
    }
    if (CONS && lane < N) {
        int r = n_contact_rows + before;
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            if (((jbits >> t) & 1u) && r < R) {
                L.src[r] = kJointRow + 3 * lane + t;
                L.b[r] = jb[t];
                L.lo[r] = jlo[t];
                L.hi[r] = jhi[t];
                ++r;
            }
        }
    }

    MW_PROF_T(t2);
    MW_PROF_ACC(2, t1, t2);
    if (R > 0) {
        // ---- responses (lane = row) ------------------------------------------
        for (int r0 = 0; r0 < R; r0 += kWaveLanes) {
            const int r = r0 + lane;
            if (r < R) {
                // contact rows (impulse f on body k) and joint rows (unit
                // impulse on dof j) share one response pass: the lanes of a
                // mixed row set do not diverge into two serial passes
                const int src = L.src[r];
                const bool contact = src < kJointRow;
                int k = -2, j = -1;
                SV f = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
                int slot = 0, d = 0;
                if (contact) {
                    slot = src / 3;
                    d = src % 3;
                    int sh = 0;
                    while (sh + 1 < F->n_shapes && F->shape_slot0[sh + 1] <= slot) ++sh;
                    k = F->shape_body[sh];
                    const f3 bpt = {L.s_b[slot][0], L.s_b[slot][1], L.s_b[slot][2]};
                    // body-frame direction R_k^T d: n -> row 2, t1 -> -row 1, t2 -> row 0
                    const int row = (d == 0) ? 2 : ((d == 1) ? 1 : 0);
                    const float sg = (d == 1) ? -1.f : 1.f;
                    const f3 dir = {sg * L.s_R[slot][row * 3], sg * L.s_R[slot][row * 3 + 1],
                                    sg * L.s_R[slot][row * 3 + 2]};
                    f = {cross(bpt, dir), dir};
                } else {
                    j = (src - kJointRow) / 3;
                }
                const float jv = wave_response<MAXN>(P, F, N, L, L0, k, j, f, L.J[r], L.MJ[r]);
                if (contact) {
                    const float bounce =
                        (d == 0) ? fminf(kContactErp * L.s_depth[slot] * rcp(dt), kContactMaxErv) : 0.f;
                    L.b[r] = bounce - jv;
                } else {
                    L.J[r][6 + j] = 1.f;  // the response pass left the joint row's J zero
                }
            }
        }
        MW_PROF_T(t3);
        MW_PROF_ACC(3, t2, t3);
        // ---- Delassus matrix A = J (M^-1 J^T)^T on the matrix cores ------------
        // v_mfma_f32_32x32x2_f32 tiles (fp32 operands, fp32 accumulate): in
        // k-step k, lane l supplies J[m0 + l%32][2k + l/32] and
        // MJ[n0 + l%32][2k + l/32]; the 32x32 result holds column n0 + l%32 in
        // lane l, rows 8(i/4) + 4(l/32) + i%4 in accumulator i.  One exchange
        // of the two 32-lane halves then gives lane c all of column c (= row
        // c: A is symmetric), a[r] = A[r][c], the layout the PGS keeps in
        // registers.  Rows / columns >= R (stale LDS) are masked to zero.
        const int ncr = (n_contact_rows < R) ? n_contact_rows : R;
        const int lr = lane & 31, lh = lane >> 5;
        const bool two = R > 32;
        v16f t00 = {}, t01 = {}, t10 = {}, t11 = {};
        // unrolled to the instance's coordinate count (the operand loads go
        // out ahead of the MFMA chain; a loop to the runtime NV waited on each
        // k-step's loads: 14.6k -> see DESIGN.md cycles per world-step);
        // columns >= NV: J is zero there, MJ masked.  Chunks of 8 coordinates
        // (4 k-steps) end at the world's own NV (a uniform branch), so a
        // floating box (NV 6) in a MAXN-16 instance runs 4 k-steps, not 11.
        // The chunk's operands load unconditionally (MJ columns >= NV are
        // in-bounds stale LDS, masked by a select after the load): written as
        // `ev ? MJ[..] : 0` the load itself was conditional, an exec-masked
        // ds_read waited on right before each MFMA, one LDS round trip per
        // k-step.  `two` (R > 32) selects one of two loops outside.
        constexpr int kKs = (WaveWorld<MAXN>::kNv + 1) / 2;
        if (!two) {
#pragma unroll
            for (int k0 = 0; k0 < kKs; k0 += 4) {
                if (2 * k0 >= NV) break;
                float jv[4], mv[4];
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    const int e = 2 * (k0 + kk) + lh;
                    jv[kk] = (k0 + kk < kKs) ? L.J[lr][e] : 0.f;
                    mv[kk] = (k0 + kk < kKs) ? L.MJ[lr][e] : 0.f;
                }
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    if (k0 + kk >= kKs) break;
                    const bool ev = 2 * (k0 + kk) + lh < NV;
                    t00 = __builtin_amdgcn_mfma_f32_32x32x2f32(jv[kk], ev ? mv[kk] : 0.f, t00, 0, 0, 0);
                }
            }
        } else {
#pragma unroll
            for (int k0 = 0; k0 < kKs; k0 += 4) {
                if (2 * k0 >= NV) break;
                float jv0[4], mv0[4], jv1[4], mv1[4];
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    const int e = 2 * (k0 + kk) + lh;
                    const bool in = k0 + kk < kKs;
                    jv0[kk] = in ? L.J[lr][e] : 0.f;
                    mv0[kk] = in ? L.MJ[lr][e] : 0.f;
                    jv1[kk] = in ? L.J[32 + lr][e] : 0.f;
                    mv1[kk] = in ? L.MJ[32 + lr][e] : 0.f;
                }
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    if (k0 + kk >= kKs) break;
                    const bool ev = 2 * (k0 + kk) + lh < NV;
                    const float m0 = ev ? mv0[kk] : 0.f, m1 = ev ? mv1[kk] : 0.f;
                    t00 = __builtin_amdgcn_mfma_f32_32x32x2f32(jv0[kk], m0, t00, 0, 0, 0);
                    t01 = __builtin_amdgcn_mfma_f32_32x32x2f32(jv0[kk], m1, t01, 0, 0, 0);
                    t10 = __builtin_amdgcn_mfma_f32_32x32x2f32(jv1[kk], m0, t10, 0, 0, 0);
                    t11 = __builtin_amdgcn_mfma_f32_32x32x2f32(jv1[kk], m1, t11, 0, 0, 0);
                }
            }
        }
        float a[kWaveMaxRows];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            // this half's row r0; the other half holds r0 + 4.  One
            // v_permlane32_swap per tile pair: lanes < 32 get t00 of their
            // own and of lane + 32, lanes >= 32 t01 of lane - 32 and their own
            // (a ds_bpermute __shfl_xor + selects before)
            const int r0 = 8 * (i / 4) + (i % 4);
            float x0 = t00[i], y0 = t01[i];
            lane_swap32(x0, y0);
            a[r0] = x0;
            a[r0 + 4] = y0;
            float x1 = t10[i], y1 = t11[i];
            lane_swap32(x1, y1);
            a[32 + r0] = x1;
            a[32 + r0 + 4] = y1;
        }
        float dg = 1.f;
#pragma unroll
        for (int r = 0; r < kWaveMaxRows; ++r) {
            a[r] = (r < R && lane < R) ? a[r] : 0.f;
            if (lane == r && r < R) {
                a[r] *= 1.f + ((r >= ncr) ? kJointCfm : kContactCfm);
                dg = a[r];
            }
        }
        MW_PROF_T(t4);
        MW_PROF_ACC(4, t3, t4);
        // ---- PGS: impulses x[r] uniform (registers), residual w_c = sum_r A[c][r] x_r
        // in lane c.  Rows in order (the oracle's Gauss-Seidel order), padded
        // to blocks of 8 with inert rows (zero column, b = 0, bounds [0, 0]) so
        // the sweep is branch-free inside a block.  The residual is rebuilt at
        // the start of every sweep and updated by column r (= a[r], symmetry)
        // after row r moves, so a row costs one lane read of w, one uniform
        // LDS broadcast of its constants {b, 1/A_rr, lo, hi} (off the chain)
        // and a handful of dependent VALU ops.  A contact's normal row sets
        // the bound mu x_normal its two friction rows clamp to.
        const int Rpad = (R + 7) & ~7;
        if (lane < Rpad) {
            F4 c = {0.f, 0.f, 0.f, 0.f};
            if (lane < R) {
                c.x = L.b[lane];
                c.y = rcp(dg);
                if (lane < ncr) {
                    const bool normal = (lane % 3) == 0;
                    c.z = normal ? 0.f : -1.f;
                    c.w = normal ? kBig : 1.f;
                } else {
                    c.z = L.lo[lane];
                    c.w = L.hi[lane];
                }
            }
            L.rc[lane] = c;
        }
        const float mu = F->mu;
        float x[kWaveMaxRows];
        // warm start: every row from the previous step's impulse of the same
        // row identity (contact slot / joint row), else 0; x1w: its stage-1
        // impulse (exact solve)
        float x0 = 0.f, x1w = 0.f;
        const int wid = (lane < R) ? ((L.src[lane] < kJointRow) ? L.src[lane]
                                                                 : kWaveWarmJoint0 + (L.src[lane] - kJointRow))
                                   : 0;
        if (warm && lane < R) {
            x0 = L.xw[wid];
            x1w = L.xw[kWaveWarmWords + wid];
        }
        float x1s = 0.f;  // this step's stage-1 impulse (exact solve)
        if (lcp_solves > 0) {
            // DART's boxed LCP (wave_lcp.hpp; oracle OR_PGS_CONVERGED): lane r =
            // row r, each of its two stages from the previous step's solution,
            // then PGS sweeps on the stage's box problem, then the exact solve
            LcpRow Rw;
            Rw.live = lane < R;
            const F4 c = L.rc[lane < Rpad ? lane : 0];
            Rw.kind = (lane < ncr) ? ((lane % 3 == 0) ? 0 : 1) : 2;
            Rw.nrow = (Rw.kind == 1) ? lane - lane % 3 : lane;
            Rw.b = Rw.live ? c.x : 0.f;
            Rw.lo = Rw.live ? c.z : 0.f;
            Rw.hi = Rw.live ? c.w : 0.f;
            float xe = x0;
            x1s = x1w;
            // (skipping the stages' sweeps when every contact has a warm
            // record: C5 72.2 -> 68.0 us, but a resting cube's friction
            // answer then drifts by 1.7e-4 m/s (test_cube_contact_kat): kept)
            const int sweeps = pgs_iters;
            // the elimination's pivot rows go to the responses' stack (dead here)
            static_assert(sizeof(L.stack) >= kLcpWorkFloats * sizeof(float), "LCP workspace");
            float* U = &L.stack[0][0][0];
            int nsolve = 0, nround = 0, nsolve1 = 0;
            long long cyc[3] = {0, 0, 0};
            constexpr int kLcpSmall = 32;
            // the matrix-core solves this instance takes (wave_lcp.hpp: the
            // <= 16-body instance and the 64-row width eliminate over the lanes)
            constexpr int kWaveLcpMfma = (MAXN <= 16) ? kWaveLcpMfmaSmall : kWaveLcpMfmaLarge;
            // three register widths (wave_lcp.hpp: the elimination runs the
            // whole register row): a free body's 4-corner LCP (12 rows) on 16
            // columns took contacts_floating 195 -> 167 us (gpurun_out r04z)
            bool ok;
            if (R <= 16 && kLcpSmall > 0)
                ok = wave_lcp_exact<16, false, kLcpStageSweeps, kWaveLcpMfma>(a, Rw, mu, R, lcp_solves, sweeps, pgs_tol, L.rc, U, x1s, xe, nsolve, nround,
                                        nsolve1, cyc);
            else if (R <= kLcpSmall)
                ok = wave_lcp_exact<32, false, kLcpStageSweeps, kWaveLcpMfma>(a, Rw, mu, R, lcp_solves, sweeps, pgs_tol, L.rc, U, x1s, xe, nsolve, nround,
                                        nsolve1, cyc);
            else
                ok = wave_lcp_exact<kWaveMaxRows, false, kLcpStageSweeps, kWaveLcpMfma>(a, Rw, mu, R, lcp_solves, sweeps, pgs_tol, L.rc, U, x1s, xe,
                                                  nsolve, nround, nsolve1, cyc);
#ifdef MW_WAVE_PROF
            if (MW_DUMP_WHEN(ok, nsolve)) {
                unsigned int claim = 0u;
                if (lane == 0) claim = atomicAdd(&g_wave_dump_claim, 1u);
                claim = __builtin_amdgcn_readfirstlane(claim);
                if (claim < static_cast<unsigned int>(kDumpSlots)) {
                    float* D0 = g_wave_dump + claim * kWaveDumpFloats;
                    for (int r = 0; r < R; ++r) D0[8 + r * 64 + lane] = (lane < R) ? a[r] : 0.f;
                    float* V = D0 + 8 + 64 * 64;
                    if (lane < R) {
                        V[lane] = Rw.b;
                        V[64 + lane] = Rw.lo;
                        V[128 + lane] = Rw.hi;
                        V[192 + lane] = static_cast<float>(Rw.kind);
                        V[256 + lane] = x0;
                        V[320 + lane] = x1w;
                        V[384 + lane] = xe;
                        V[448 + lane] = x1s;
                    }
                    if (lane == 0) {
                        D0[0] = static_cast<float>(R);
                        D0[1] = static_cast<float>(nsolve);
                        D0[2] = static_cast<float>(nsolve1);
                        D0[3] = mu;
                        D0[4] = ok ? 1.f : 0.f;
                    }
                }
            }
            prof[8] += static_cast<unsigned long long>(nsolve);
            prof[9] += static_cast<unsigned long long>(nround);
            prof[10] += static_cast<unsigned long long>(nsolve1);
            prof[11] = prof[11] > static_cast<unsigned long long>(nsolve) ? prof[11] : nsolve;
            prof[12] = prof[12] > static_cast<unsigned long long>(nsolve1) ? prof[12] : nsolve1;
            prof[13] += nsolve > 4 ? 1ull : 0ull;
            prof[14] += static_cast<unsigned long long>(cyc[0]);
            prof[16] += static_cast<unsigned long long>(cyc[1]);
            prof[17] += static_cast<unsigned long long>(cyc[2]);
#else
            (void)nsolve1;
            (void)cyc;
#endif
#pragma unroll
            for (int r = 0; r < kWaveMaxRows; ++r) {
                if ((r & 7) == 0 && r >= Rpad) break;
                x[r] = read_lane(xe, r);
            }
            if (!ok) MW_LANE0 { *unconverged += 1; }
            MW_PROF_T(t45);
            MW_PROF_ACC(15, t4, t45);
        } else {
#pragma unroll
            for (int r = 0; r < kWaveMaxRows; ++r) x[r] = warm ? read_lane(x0, r) : 0.f;
            if (pgs_tol > 0.f)
                wave_pgs<MAXN, true>(L, a, x, Rpad, ncr, mu, pgs_iters, pgs_tol);
            else
                wave_pgs<MAXN, false>(L, a, x, Rpad, ncr, mu, pgs_iters, 0.f);
            MW_PROF_T(t45);
            MW_PROF_ACC(15, t4, t45);
        }
        MW_PROF_T(t5);
        MW_PROF_ACC(5, t4, t5);
        // ---- nu += MJ^T x (lane = component); impulses to the slots ----------------
        float xl = 0.f, dnu = 0.f;
#pragma unroll
        for (int rb = 0; rb < kWaveMaxRows; rb += 8) {
            if (rb >= Rpad) break;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int r = rb + k;
                xl = (lane == r) ? x[r] : xl;
                if (r < R && lane < NV) dnu += x[r] * L.MJ[r][lane];
            }
        }
        if (lane < R) {
            const int src = L.src[lane];
            if (src < kJointRow) L.s_x[src / 3][src % 3] = xl;
        }
        if (lane < NV) L.nu[lane] += dnu;
        if (warm) {
            for (int e = lane; e < kWaveWarmRecord; e += kWaveLanes) L.xw[e] = 0.f;
            wave_lds_sync();
            if (lane < R) {
                L.xw[wid] = xl;
                L.xw[kWaveWarmWords + wid] = x1s;
            }
        }
    } else if (warm) {
        for (int e = lane; e < kWaveWarmRecord; e += kWaveLanes) L.xw[e] = 0.f;
    }

    // ---- integratePositions ---------------------------------------------------
    // (a ball joint's three lanes read each other's coordinates: every lane
    // forms its new q before any is stored)
    float q_new = 0.f;
    if (lane < N) {
        const float qd_new = L.nu[6 + lane];
        qdd_out[lane] = (qd_new - L.qd[lane]) * rcp(dt);
        L.qd[lane] = qd_new;
        q_new = L.q[lane] + dt * qd_new;
        const int bp = ball_part(P->b[lane]);
        if (bp) {
            const int i0 = lane - bp + 1;
            q_new = ball_integrate(L.q[i0], L.q[i0 + 1], L.q[i0 + 2], L.nu[6 + i0], L.nu[7 + i0], L.nu[8 + i0], dt,
                                   bp - 1);
        }
    }
    wave_lds_sync();
    if (lane < N) L.q[lane] = q_new;
    const SV V = {{L.nu[0], L.nu[1], L.nu[2]}, {L.nu[3], L.nu[4], L.nu[5]}};
    integrate_pose(R0, V, dt, base);
    base.V = V;
    MW_PROF_T(t6);
    MW_PROF_ACC(6, t2, t6);
    return active;
}

#undef MW_LANE0

}  // namespace dev
}  // namespace mw

