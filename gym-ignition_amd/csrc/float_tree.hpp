// float_tree.hpp -- one engine step of an articulated model on a floating
// base (a DART skeleton whose root joint is a FreeJoint) with ground-plane
// contacts on any body, float32, one world per lane.  Restates, like oracle.c
// or_float_step (fp64, dense), DART 6.x World::step as driven by the
// reference's Physics system (Physics.cpp:1824-1835) [EXT]:
//
//   forward dynamics      ABA over the joint tree with a free 6-dof root:
//                         the root's articulated inertia IA0 is factored
//                         (6x6 Cholesky) and a0 = -IA0^-1 pA0; gravity enters
//                         as the body force I [0; g_body]
//   integrateVelocities   nu += dt nu',  nu = [V0 (base twist, base frame); qd]
//   constraint rows       ContactConstraint (normal + two ODE plane-space
//                         tangents per point, ERP 0.01 / max 1e-3 m/s, CFM
//                         1e-5) first, then the joint rows (limit, servo,
//                         Coulomb friction), the order of DART's
//                         ConstraintSolver; projected Gauss-Seidel on the
//                         impulses x with the Delassus matrix J M^-1 J^T
//                         (the oracle's form)
//   integratePositions    q += dt qd;  T0 <- T0 exp(dt V0)
//
// Layout for CDNA4:
//   - per-body factorisation (R, p, U, psi, ...) in LDS (LdsStage records,
//     stride 64 lanes), indexed by runtime body numbers where a contact's
//     body is a model parameter (uniform across the wave);
//   - constraint rows in a per-world global workspace laid out [word][W]
//     (coalesced: a wave's access to one word of one row is 256 contiguous
//     bytes): per contact slot its point, depth, body rotation, the three
//     rows' J, M^-1 J^T and J M^-1 J^T, and per dof a column M^-1 e_j.
//     Rows live in the workspace, not LDS, so a model's slot count is not
//     capped by the 160 KB of LDS per CU.
//   - the PGS itself runs on a compacted table of the active rows in LDS
//     (RowsLds: A, b, bounds, x for up to kLdsRows rows), assembled once per
//     step; every sweep is then LDS-only.  A step with more active rows falls
//     back to sequential impulses on nu over the workspace rows (the same
//     iteration; each row then costs dependent global round trips).
//   - contact slots are fixed per model (8 corners of a box, 1 per sphere),
//     an active bitmask selects them; the loops over slots and their bodies
//     are uniform (model data), only the active test diverges.
#pragma once

#include "chain_dyn.hpp"
#include "free_body.hpp"

namespace mw {

constexpr int kMaxFloatShapes = 16;
constexpr int kMaxFloatSlots = 32;  // active-slot bitmask
constexpr float kJointCfm = 1e-9f;  // DART JointConstraint CFM [EXT] (oracle OR_CFM)

// Floating base + collision shapes of an articulated floating model; the
// joints are the ChainF bodies (their parent -1 is this base).
struct FloatF {
    float mass;
    float com[3];
    float Io[6];           // base rotational inertia about its origin: xx yy zz xy xz yz
    float g[3];            // world gravity
    float mu;              // Coulomb friction with the ground
    int32_t ground;
    int32_t n_shapes;
    int32_t n_slots;
    int32_t pad_;
    // shapes ordered base first, then by body (oracle FloatWorld order)
    int32_t shape_body[kMaxFloatShapes];   // -1 = base
    int32_t shape_type[kMaxFloatShapes];   // 0 box (half extents), 1 sphere (radius)
    int32_t shape_slot0[kMaxFloatShapes];  // first contact slot of the shape
    uint64_t shape_path[kMaxFloatShapes];  // bit i: body i is the shape's body or one of its ancestors
    float shape_size[kMaxFloatShapes][3];
    float shape_R[kMaxFloatShapes][9];
    float shape_p[kMaxFloatShapes][3];
    // tree levels for the level-parallel ABA of the wave kernel (wave_tree.hpp):
    // depth of every body (0 = child of the base), its rank among the
    // children of its parent counted from the highest index (the order the
    // serial inward pass adds them in), the number of levels and the largest
    // number of children of one body (or of the base)
    int32_t levels;
    int32_t fanout;
    int32_t dual;          // some joint has damping: impulses need the non-implicit inertias
    int32_t fixed;         // the base is welded to the world (generic fixed-base trees, wave kernel)
    int8_t body_depth[kMaxBodies];
    int8_t body_srank[kMaxBodies];
    uint64_t body_path[kMaxBodies];  // bit k: body k is body i or one of its ancestors
};

namespace dev {

// ---- workspace layout (floats per world, each word strided by W) --------
template <int N>
struct FloatWs {
    static constexpr int kNv = 6 + N;
    // slot record: b(3) body-frame point, xw(3) world point, depth, Rk(9)
    // body rotation, x(3) impulses, arr(3) J M^-1 J^T, then 3 x (J, MJ)
    static constexpr int kSlotHead = 22;
    static constexpr int kSlotWords = kSlotHead + 3 * 2 * kNv;
    static constexpr int kColWords = kNv;  // M^-1 e_j per dof
    static int words(int n_slots) { return n_slots * kSlotWords + N * kColWords; }
};

struct WsRef {
    float* base;  // &ws[0 * W + w]
    int W;
    __device__ __forceinline__ float& at(int word) const { return base[static_cast<size_t>(word) * W]; }
};

// Compacted active rows of one world in LDS for the x-space PGS (the
// oracle's form): the Delassus matrix A = J M^-1 J^T with the CFM on its
// diagonal, right-hand sides, bounds, impulses and each row's source (a
// contact row 3 slot + d, or a joint row kJointRow + 3 dof + type).  Word k
// of lane l at [k * 64 + l].  A PGS sweep then touches LDS only.
constexpr int kLdsRows = 16;
constexpr int kJointRow = 128;
constexpr int kRowsLdsWords = kLdsRows * kLdsRows + 5 * kLdsRows;
struct RowsLds {
    float* base;  // &words[0][lane]
    __device__ __forceinline__ float& A(int r, int c) const { return base[(r * kLdsRows + c) * kLdsLanes]; }
    __device__ __forceinline__ float& b(int r) const { return base[(kLdsRows * kLdsRows + r) * kLdsLanes]; }
    __device__ __forceinline__ float& x(int r) const { return base[(kLdsRows * (kLdsRows + 1) + r) * kLdsLanes]; }
    __device__ __forceinline__ float& lo(int r) const { return base[(kLdsRows * (kLdsRows + 2) + r) * kLdsLanes]; }
    __device__ __forceinline__ float& hi(int r) const { return base[(kLdsRows * (kLdsRows + 3) + r) * kLdsLanes]; }
    __device__ __forceinline__ int32_t& src(int r) const {
        return reinterpret_cast<int32_t*>(base)[(kLdsRows * (kLdsRows + 4) + r) * kLdsLanes];
    }
};

// 6x6 SPD factorisation (Cholesky, lower, packed row-major) of a root
// articulated inertia; solve() returns IA^-1 b
struct Chol6 {
    float l[21];
    float id[6];  // 1 / L_ii
    __device__ __forceinline__ static int ix(int r, int c) { return r * (r + 1) / 2 + c; }
    __device__ __forceinline__ void factor(const SI& I) {
        float a[6][6];
        const float A9[9] = {I.A.xx, I.A.xy, I.A.xz, I.A.xy, I.A.yy, I.A.yz, I.A.xz, I.A.yz, I.A.zz};
        const float C9[9] = {I.C.xx, I.C.xy, I.C.xz, I.C.xy, I.C.yy, I.C.yz, I.C.xz, I.C.yz, I.C.zz};
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                a[r][c] = A9[r * 3 + c];
                a[r][c + 3] = I.B.m[r * 3 + c];
                a[r + 3][c] = I.B.m[c * 3 + r];
                a[r + 3][c + 3] = C9[r * 3 + c];
            }
#pragma unroll
        for (int c = 0; c < 6; ++c) {
            float d = a[c][c];
#pragma unroll
            for (int k = 0; k < c; ++k) d -= l[ix(c, k)] * l[ix(c, k)];
            const float s = sqrtf(d);
            l[ix(c, c)] = s;
            id[c] = rcp(s);
#pragma unroll
            for (int r = c + 1; r < 6; ++r) {
                float v = a[r][c];
#pragma unroll
                for (int k = 0; k < c; ++k) v -= l[ix(r, k)] * l[ix(c, k)];
                l[ix(r, c)] = v * id[c];
            }
        }
    }
    __device__ __forceinline__ SV solve(const SV& b) const {
        float y[6] = {b.w.x, b.w.y, b.w.z, b.v.x, b.v.y, b.v.z};
#pragma unroll
        for (int r = 0; r < 6; ++r) {
            float v = y[r];
#pragma unroll
            for (int k = 0; k < r; ++k) v -= l[ix(r, k)] * y[k];
            y[r] = v * id[r];
        }
#pragma unroll
        for (int r = 5; r >= 0; --r) {
            float v = y[r];
#pragma unroll
            for (int k = r + 1; k < 6; ++k) v -= l[ix(k, r)] * y[k];
            y[r] = v * id[r];
        }
        return {{y[0], y[1], y[2]}, {y[3], y[4], y[5]}};
    }
};

__device__ __forceinline__ SI rigid_base(const FloatF& F) {
    SI I;
    const float m = F.mass, cx = F.com[0], cy = F.com[1], cz = F.com[2];
    I.A = {F.Io[0], F.Io[1], F.Io[2], F.Io[3], F.Io[4], F.Io[5]};
    I.B.m[0] = 0.f;     I.B.m[1] = -m * cz; I.B.m[2] = m * cy;
    I.B.m[3] = m * cz;  I.B.m[4] = 0.f;     I.B.m[5] = -m * cx;
    I.B.m[6] = -m * cy; I.B.m[7] = m * cx;  I.B.m[8] = 0.f;
    I.C = {m, m, m, 0.f, 0.f, 0.f};
    return I;
}

// -dad(V, I V) - I [0; g] of a rigid body (bias force, body frame)
__device__ __forceinline__ SV rigid_bias(float m, f3 c, const Sy& Io, const SV& V, f3 g) {
    const f3 hw = mul(Io, V.w) + m * cross(c, V.v);
    const f3 hv = m * (V.v - cross(c, V.w));
    return {cross(V.w, hw) + cross(V.v, hv) - m * cross(c, g), cross(V.w, hv) - m * g};
}

// Floating-base ABA (no joint damping: the impulse passes reuse U / psi).
// Fills the stage (R, p, U, psi per body) and L0; returns a0 (base twist
// derivative, base frame) and qdd.
template <int N, Topo TOPO, class WK>
__device__ __forceinline__ void aba_float(const ChainF* __restrict__ P, const FloatF* __restrict__ F, const M3& R0,
                                          const SV& V0, const float (&q)[N], const float (&qd)[N],
                                          const float (&tau)[N], SV& a0, float (&qdd)[N], WK& W, Chol6& L0) {
    const f3 g0 = mulT(R0, mk(F->g[0], F->g[1], F->g[2]));
    SV V[N];
    f3 g[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const BodyF& b = P->b[i];
        BodyState& s = W.bs(i);
        const int pa = parent_of(TOPO, i);
        joint_pose(b, q[i], s.R, s.p);
        const SV Sq = motion(b, qd[i]);
        V[i] = ad_inv(s.R, s.p, pa >= 0 ? V[pa] : V0) + Sq;
        g[i] = mulT(s.R, pa >= 0 ? g[pa] : g0);
        const SV& Vi = V[i];
        s.eta = {cross(Vi.w, Sq.w), cross(Vi.w, Sq.v) + cross(Vi.v, Sq.w)};
        const float m = b.mass;
        W.own(i) = rigid_bias(m, mk(b.com[0], b.com[1], b.com[2]), inertia_origin(b, m), Vi, g[i]);
    }
    SI carry[N];
    SV carryB[N];
    SI IA0 = rigid_base(*F);
    SV B0 = rigid_bias(F->mass, mk(F->com[0], F->com[1], F->com[2]),
                       Sy{F->Io[0], F->Io[1], F->Io[2], F->Io[3], F->Io[4], F->Io[5]}, V0, g0);
#pragma unroll
    for (int i = N - 1; i >= 0; --i) {
        const BodyF& b = P->b[i];
        BodyState& s = W.bs(i);
        const int pa = parent_of(TOPO, i);
        SI AI = rigid(b, b.mass);
        SV Bi = W.own(i);
        if (has_child(TOPO, N, i)) {
            AI += carry[i];
            Bi = Bi + carryB[i];
        }
        s.U = ais(AI, b);
        s.psi = rcp(proj(b, s.U));
        const SV AIeta = mul(AI, s.eta);
        s.tt = tau[i] - proj(b, AIeta + Bi);
        const SI c = to_parent(s.R, s.p, downdate(AI, s.U, s.psi));
        const SV cb = dad_inv(s.R, s.p, Bi + AIeta + (s.psi * s.tt) * s.U);
        if (pa >= 0) {
            if (first_inward(TOPO, N, i)) { carry[pa] = c; carryB[pa] = cb; }
            else { carry[pa] += c; carryB[pa] = carryB[pa] + cb; }
        } else {
            IA0 += c;
            B0 = B0 + cb;
        }
    }
    L0.factor(IA0);
    a0 = L0.solve(-1.f * B0);
    SV a[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const BodyF& b = P->b[i];
        const BodyState& s = W.bs(i);
        const int pa = parent_of(TOPO, i);
        const SV ap = ad_inv(s.R, s.p, pa >= 0 ? a[pa] : a0);
        qdd[i] = s.psi * (s.tt - dot(s.U, ap));
        a[i] = ap + s.eta + motion(b, qdd[i]);
    }
}

// Response of nu to a spatial impulse f on body k (k = -1: the base; body
// frame, force-like) and/or a unit impulse on dof j (j = -1: none):
//   MJ = M^-1 (J_k^T f + e_j),  J = J_k^T f  (the generalized row of f).
// k, j and path (bit i: body i lies on the injection's path to the base)
// are uniform; every loop is unrolled over the compile-time bodies.
template <int N, Topo TOPO, class WK>
__device__ __forceinline__ void response(const ChainF* __restrict__ P, const WK& W, const Chol6& L0, int k, int j,
                                         uint32_t path, const SV& f, float (&J)[6 + N], float (&MJ)[6 + N]) {
    float u[N];
    SV Bimp[N], Fk[N];
    SV B0 = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}}, F0 = B0;
    if (k < 0 && j < 0) { B0 = -1.f * f; F0 = f; }
#pragma unroll
    for (int i = N - 1; i >= 0; --i) {
        J[6 + i] = 0.f;
        u[i] = 0.f;
        if (!((path >> i) & 1u)) continue;
        const BodyF& b = P->b[i];
        const BodyState& s = W.bs(i);
        SV Bi, Fi;
        if (i == k) { Bi = -1.f * f; Fi = f; }
        else if (i == j) { Bi = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}}; Fi = Bi; }
        else { Bi = Bimp[i]; Fi = Fk[i]; }
        J[6 + i] = proj(b, Fi);
        u[i] = ((i == j) ? 1.f : 0.f) - proj(b, Bi);
        const SV up = dad_inv(s.R, s.p, Bi + (s.psi * u[i]) * s.U);
        const SV fp = dad_inv(s.R, s.p, Fi);
        const int pa = parent_of(TOPO, i);
        if (pa >= 0) { Bimp[pa] = up; Fk[pa] = fp; }
        else { B0 = up; F0 = fp; }
    }
    J[0] = F0.w.x; J[1] = F0.w.y; J[2] = F0.w.z; J[3] = F0.v.x; J[4] = F0.v.y; J[5] = F0.v.z;
    const SV dV0 = L0.solve(-1.f * B0);
    MJ[0] = dV0.w.x; MJ[1] = dV0.w.y; MJ[2] = dV0.w.z; MJ[3] = dV0.v.x; MJ[4] = dV0.v.y; MJ[5] = dV0.v.z;
    SV dv[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const BodyState& s = W.bs(i);
        const int pa = parent_of(TOPO, i);
        const SV dvp = ad_inv(s.R, s.p, pa >= 0 ? dv[pa] : dV0);
        MJ[6 + i] = s.psi * (u[i] - dot(s.U, dvp));
        dv[i] = dvp + motion(P->b[i], MJ[6 + i]);
    }
}

template <int N>
struct FloatBody {  // per-world floating state in registers
    FreeState base;  // p, quaternion, V0
    float q[N], qd[N];
};

// One engine step.  act / vcmd as substep(); tau holds the joint forces of
// this step (commands and PID already applied).  Returns the active slots.
template <int N, Topo TOPO, bool CONS, class WK>
__device__ __forceinline__ uint32_t float_step(const ChainF* __restrict__ P, const FloatF* __restrict__ F,
                                               FloatBody<N>& X, const float (&tau)[N], const uint8_t (&act)[N],
                                               const float (&vcmd)[N], float dt, int pgs_iters, float (&qdd)[N],
                                               WK& W, const WsRef& ws, const RowsLds& RL) {
    using L = FloatWs<N>;
    constexpr int NV = L::kNv;
    const M3 R0 = quat_to_R(X.base.qw, X.base.qx, X.base.qy, X.base.qz);
    SV a0;
    Chol6 L0;
    aba_float<N, TOPO>(P, F, R0, X.base.V, X.q, X.qd, tau, a0, qdd, W, L0);
    float nu[NV];
    nu[0] = X.base.V.w.x + dt * a0.w.x; nu[1] = X.base.V.w.y + dt * a0.w.y; nu[2] = X.base.V.w.z + dt * a0.w.z;
    nu[3] = X.base.V.v.x + dt * a0.v.x; nu[4] = X.base.V.v.y + dt * a0.v.y; nu[5] = X.base.V.v.z + dt * a0.v.z;
#pragma unroll
    for (int i = 0; i < N; ++i) nu[6 + i] = X.qd[i] + dt * qdd[i];

    // ---- contact detection at the start-of-step poses --------------------
    uint32_t active = 0u;
    if (F->ground) {
        M3 Rw[N];
        f3 pw[N];
#pragma unroll
        for (int i = -1; i < N; ++i) {
            M3 Rb;
            f3 pb;
            if (i < 0) {
                Rb = R0;
                pb = X.base.p;
            } else {
                const BodyState& s = W.bs(i);
                const int pa = parent_of(TOPO, i);
                const M3& Rp = pa >= 0 ? Rw[pa] : R0;
                const f3 pp = pa >= 0 ? pw[pa] : X.base.p;
#pragma unroll
                for (int r = 0; r < 3; ++r)
#pragma unroll
                    for (int c = 0; c < 3; ++c)
                        Rw[i].m[r * 3 + c] =
                            Rp.m[r * 3] * s.R.m[c] + Rp.m[r * 3 + 1] * s.R.m[3 + c] + Rp.m[r * 3 + 2] * s.R.m[6 + c];
                pw[i] = pp + mul(Rp, s.p);
                Rb = Rw[i];
                pb = pw[i];
            }
            for (int sh = 0; sh < F->n_shapes; ++sh) {
                if (F->shape_body[sh] != i) continue;
                const bool sphere = (F->shape_type[sh] == 1);
                const int corners = sphere ? 1 : 8;
                for (int c = 0; c < corners; ++c) {
                    const float* h = F->shape_size[sh];
                    const float* SR = F->shape_R[sh];
                    const f3 lp = shape_slot_point(F->shape_type[sh], h, shape_plane_normal(Rb, SR), c);
                    const float lx = lp.x, ly = lp.y, lz = lp.z;
                    f3 b = {F->shape_p[sh][0] + SR[0] * lx + SR[1] * ly + SR[2] * lz,
                            F->shape_p[sh][1] + SR[3] * lx + SR[4] * ly + SR[5] * lz,
                            F->shape_p[sh][2] + SR[6] * lx + SR[7] * ly + SR[8] * lz};
                    f3 xw = pb + mul(Rb, b);
                    float depth = -xw.z;
                    if (sphere) {
                        depth = h[0] - xw.z;
                        xw.z -= h[0];
                        b = mulT(Rb, xw - pb);
                    }
                    if (depth > 0.f) {
                        const int slot = F->shape_slot0[sh] + c;
                        active |= 1u << slot;
                        const int o = slot * L::kSlotWords;
                        ws.at(o + 0) = b.x; ws.at(o + 1) = b.y; ws.at(o + 2) = b.z;
                        ws.at(o + 3) = xw.x; ws.at(o + 4) = xw.y; ws.at(o + 5) = xw.z;
                        ws.at(o + 6) = depth;
#pragma unroll
                        for (int e = 0; e < 9; ++e) ws.at(o + 7 + e) = Rb.m[e];
                    }
                }
            }
        }
    }

    // ---- rows: J, M^-1 J^T, diagonal --------------------------------------
    if (active) {
        for (int sh = 0; sh < F->n_shapes; ++sh) {
            const int k = F->shape_body[sh];
            const uint32_t path = static_cast<uint32_t>(F->shape_path[sh]);  // N <= 32 here
            const int corners = (F->shape_type[sh] == 1) ? 1 : 8;
            for (int c = 0; c < corners; ++c) {
                const int slot = F->shape_slot0[sh] + c;
                if (!((active >> slot) & 1u)) continue;
                const int o = slot * L::kSlotWords;
                const f3 b = {ws.at(o + 0), ws.at(o + 1), ws.at(o + 2)};
                // body-frame directions R_k^T d: n = +z -> row 2 of R_k,
                // t1 = (0, -1, 0) -> -row 1, t2 = (1, 0, 0) -> row 0
                const f3 r0 = {ws.at(o + 7), ws.at(o + 8), ws.at(o + 9)};
                const f3 r1 = {ws.at(o + 10), ws.at(o + 11), ws.at(o + 12)};
                const f3 r2 = {ws.at(o + 13), ws.at(o + 14), ws.at(o + 15)};
                const f3 db[3] = {r2, -r1, r0};
#pragma unroll
                for (int d = 0; d < 3; ++d) {
                    const SV f = {cross(b, db[d]), db[d]};
                    float J[NV], MJ[NV];
                    W.fence();
                    response<N, TOPO>(P, W, L0, k, -1, path, f, J, MJ);
                    float arr = 0.f;
#pragma unroll
                    for (int e = 0; e < NV; ++e) arr += J[e] * MJ[e];
                    const int ro = o + L::kSlotHead + d * 2 * NV;
#pragma unroll
                    for (int e = 0; e < NV; ++e) { ws.at(ro + e) = J[e]; ws.at(ro + NV + e) = MJ[e]; }
                    ws.at(o + 19 + d) = arr;
                    ws.at(o + 16 + d) = 0.f;
                }
            }
        }
    }
    uint32_t on = 0u, at_upper = 0u, need = 0u;
    float bb[N][3];
    if constexpr (CONS) {
#pragma unroll
        for (int i = 0; i < N; ++i) {
            const BodyF& b = P->b[i];
            const float qdi = nu[6 + i];
            bb[i][0] = bb[i][1] = bb[i][2] = 0.f;
            if (b.limited) {
                float viol = X.q[i] - b.lower;
                bool lim = false;
                if (viol <= 0.f) {
                    lim = true;
                } else {
                    viol = X.q[i] - b.upper;
                    if (viol >= 0.f) { lim = true; at_upper |= 1u << i; }
                }
                if (lim) {
                    on |= 1u << (3 * i);
                    bb[i][0] = fminf(fmaxf(-viol * kErp * rcp(dt), -kMaxErv), kMaxErv);  // target velocity
                }
            }
            if (act[i] == kActServo) {
                const float vc = fminf(fmaxf(vcmd[i], -b.vel_limit), b.vel_limit);
                if (vc - qdi != 0.f) { on |= 1u << (3 * i + 1); bb[i][1] = vc; }
            }
            if (b.friction != 0.f && qdi != 0.f) on |= 1u << (3 * i + 2);
            if ((on >> (3 * i)) & 7u) need |= 1u << i;
        }
        if (need) {
            constexpr PathMasks<N> paths = path_masks<N, TOPO>();
            const SV zero = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
#pragma unroll
            for (int i = 0; i < N; ++i) {
                if (!((need >> i) & 1u)) continue;
                float J[NV], MJ[NV];
                W.fence();
                response<N, TOPO>(P, W, L0, -2, i, paths.m[i], zero, J, MJ);
                const int co = F->n_slots * L::kSlotWords + i * L::kColWords;
#pragma unroll
                for (int e = 0; e < NV; ++e) ws.at(co + e) = MJ[e];
            }
        }
    }

    // ---- projected Gauss-Seidel ---------------------------------------------
    const int n_rows = 3 * __builtin_popcount(active) + __builtin_popcount(on);
    const float inv_dt_c = rcp(dt);
    if (n_rows > 0 && n_rows <= kLdsRows) {
        // x-space PGS on the compacted rows, A in LDS (the oracle's order:
        // contacts by slot, then joint rows by dof: limit, servo, friction)
        int R = 0;
        for (uint32_t m = active; m; m &= m - 1u) {
            const int slot = __builtin_ctz(m);
            const int o = slot * L::kSlotWords;
            const float bounce = fminf(kContactErp * ws.at(o + 6) * inv_dt_c, kContactMaxErv);
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                const int ro = o + L::kSlotHead + d * 2 * NV;
                float jv = 0.f;
#pragma unroll
                for (int e = 0; e < NV; ++e) jv += ws.at(ro + e) * nu[e];
                RL.src(R) = 3 * slot + d;
                RL.b(R) = ((d == 0) ? bounce : 0.f) - jv;
                RL.lo(R) = 0.f;
                RL.hi(R) = kBig;
                ++R;
            }
        }
#pragma unroll
        for (int i = 0; i < N; ++i) {
#pragma unroll
            for (int t = 0; t < 3; ++t) {
                if (!((on >> (3 * i + t)) & 1u)) continue;
                const BodyF& b = P->b[i];
                float lo, hi;
                if (t == 0) {
                    const bool up = (at_upper >> i) & 1u;
                    lo = up ? -kBig : 0.f;
                    hi = up ? 0.f : kBig;
                } else {
                    hi = (t == 1 ? b.effort : b.friction) * dt;
                    lo = -hi;
                }
                RL.src(R) = kJointRow + 3 * i + t;
                RL.b(R) = bb[i][t] - nu[6 + i];
                RL.lo(R) = lo;
                RL.hi(R) = hi;
                ++R;
            }
        }
        // word offset of a row's M^-1 J^T in the workspace
        auto mj_off = [&](int src) -> int {
            if (src >= kJointRow) return F->n_slots * L::kSlotWords + ((src - kJointRow) / 3) * L::kColWords;
            return (src / 3) * L::kSlotWords + L::kSlotHead + (src % 3) * 2 * NV + NV;
        };
        // Delassus matrix (symmetric): A_rc = J_r . M^-1 J_c^T
        for (int c = 0; c < R; ++c) {
            const int sc = RL.src(c);
            const int mo = mj_off(sc);
            float Mc[NV];
#pragma unroll
            for (int e = 0; e < NV; ++e) Mc[e] = ws.at(mo + e);
            for (int r = 0; r <= c; ++r) {
                const int sr = RL.src(r);
                float a;
                if (sr >= kJointRow) {
                    a = ws.at(mo + 6 + (sr - kJointRow) / 3);  // J = e_dof
                } else {
                    const int jo = mj_off(sr) - NV;
                    a = 0.f;
#pragma unroll
                    for (int e = 0; e < NV; ++e) a += ws.at(jo + e) * Mc[e];
                }
                RL.A(r, c) = a;
                RL.A(c, r) = a;
            }
            RL.A(c, c) *= 1.f + ((sc >= kJointRow) ? kJointCfm : kContactCfm);
            RL.x(c) = 0.f;
        }
        for (int it = 0; it < pgs_iters; ++it) {
            for (int r = 0; r < R; ++r) {
                float acc = RL.b(r);
                for (int c = 0; c < R; ++c) acc -= RL.A(r, c) * RL.x(c);
                const float v = RL.x(r) + acc * rcp(RL.A(r, r));
                const int sr = RL.src(r);
                float lo = RL.lo(r), hi = RL.hi(r);
                if (sr < kJointRow && (sr % 3) != 0) {  // friction: |x| <= mu x_normal
                    hi = F->mu * RL.x(r - sr % 3);
                    lo = -hi;
                }
                RL.x(r) = fminf(fmaxf(v, lo), hi);
            }
        }
        for (int r = 0; r < R; ++r) {
            const float xr = RL.x(r);
            const int sr = RL.src(r);
            if (sr < kJointRow) ws.at((sr / 3) * L::kSlotWords + 16 + sr % 3) = xr;
            if (xr == 0.f) continue;
            const int mo = mj_off(sr);
#pragma unroll
            for (int e = 0; e < NV; ++e) nu[e] += xr * ws.at(mo + e);
        }
    } else if (active || on) {
        // more rows than the LDS table holds: sequential impulses on nu over
        // the workspace rows (mathematically the same iteration)
        float xj[N][3];
#pragma unroll
        for (int i = 0; i < N; ++i) xj[i][0] = xj[i][1] = xj[i][2] = 0.f;
        const float inv_dt = rcp(dt);
        for (int it = 0; it < pgs_iters; ++it) {
            for (uint32_t m = active; m; m &= m - 1u) {
                const int o = __builtin_ctz(m) * L::kSlotWords;
                const float bounce = fminf(kContactErp * ws.at(o + 6) * inv_dt, kContactMaxErv);
                float xs[3] = {ws.at(o + 16), ws.at(o + 17), ws.at(o + 18)};
#pragma unroll
                for (int d = 0; d < 3; ++d) {
                    const int ro = o + L::kSlotHead + d * 2 * NV;
                    float jv = 0.f;
#pragma unroll
                    for (int e = 0; e < NV; ++e) jv += ws.at(ro + e) * nu[e];
                    const float arr = ws.at(o + 19 + d);
                    const float xo = xs[d];
                    const float target = (d == 0) ? bounce : 0.f;
                    float xn = xo + (target - jv - kContactCfm * arr * xo) * rcp(arr * (1.f + kContactCfm));
                    if (d == 0) {
                        xn = fmaxf(xn, 0.f);
                    } else {
                        const float hi = F->mu * xs[0];
                        xn = fminf(fmaxf(xn, -hi), hi);
                    }
                    const float delta = xn - xo;
#pragma unroll
                    for (int e = 0; e < NV; ++e) nu[e] += delta * ws.at(ro + NV + e);
                    xs[d] = xn;
                }
                ws.at(o + 16) = xs[0]; ws.at(o + 17) = xs[1]; ws.at(o + 18) = xs[2];
            }
            if constexpr (CONS) {
#pragma unroll
                for (int i = 0; i < N; ++i) {
                    if (!((need >> i) & 1u)) continue;
                    const BodyF& b = P->b[i];
                    const int co = F->n_slots * L::kSlotWords + i * L::kColWords;
                    const float inv_diag = rcp(ws.at(co + 6 + i));
#pragma unroll
                    for (int t = 0; t < 3; ++t) {
                        if (!((on >> (3 * i + t)) & 1u)) continue;
                        float lo, hi;
                        if (t == 0) {
                            const bool up = (at_upper >> i) & 1u;
                            lo = up ? -kBig : 0.f;
                            hi = up ? 0.f : kBig;
                        } else {
                            hi = (t == 1 ? b.effort : b.friction) * dt;
                            lo = -hi;
                        }
                        const float xn = fminf(fmaxf(xj[i][t] + (bb[i][t] - nu[6 + i]) * inv_diag, lo), hi);
                        const float delta = xn - xj[i][t];
                        xj[i][t] = xn;
#pragma unroll
                        for (int e = 0; e < NV; ++e) nu[e] += delta * ws.at(co + e);
                    }
                }
            }
        }
    }

    // ---- integratePositions ------------------------------------------------
    const float inv_dt = rcp(dt);
#pragma unroll
    for (int i = 0; i < N; ++i) {
        qdd[i] = (nu[6 + i] - X.qd[i]) * inv_dt;
        X.qd[i] = nu[6 + i];
        X.q[i] += dt * nu[6 + i];
    }
    const SV V = {{nu[0], nu[1], nu[2]}, {nu[3], nu[4], nu[5]}};
    integrate_pose(R0, V, dt, X.base);
    X.base.V = V;
    return active;
}

}  // namespace dev
}  // namespace mw
