// chain_dyn.hpp -- one engine substep of a fixed-base kinematic tree (serial
// chains and branched models such as the Panda), float32, one world per lane.  This is the MI355X restatement of DART 6.x World::step as
// driven by the reference's Physics system (Physics.cpp:1824-1835) [EXT]:
//
//   ABA with implicit joint damping  (Featherstone; DART GenericJoint::
//       updateInvProjArtInertiaImplicit / updateTotalForceDynamic)
//   qd += dt * qdd                   (integrateVelocities)
//   joint-space boxed LCP            (limits / servo / Coulomb friction rows,
//       projected Gauss-Seidel over an incrementally maintained dqd = M^-1 x)
//   q  += dt * qd                    (integratePositions, semi-implicit Euler)
//
// Layout decisions for CDNA4:
//   - N (dofs) and the topology TOPO (parent of every body, chain_params.hpp)
//     are template parameters and every per-body loop is unrolled, so
//     all per-body state (transforms, articulated terms, Minv columns) lives
//     in VGPRs; no runtime-indexed private arrays (they would go to scratch).
//   - model parameters come from a uniform pointer with compile-time offsets:
//     hipcc turns them into scalar (s_load) reads shared by the wave.
//   - spatial inertias are kept in 3x3 blocks (A sym, B, C sym: 21 floats).
#pragma once

#ifdef MW_HOST_TEST
// test-only host build of this header (tests/host_dyn): same code, CPU float32
#include <cmath>
#define __device__
#define __forceinline__ inline
#else
#include <hip/hip_runtime.h>
#endif

#include "chain_params.hpp"

namespace mw {
namespace dev {

struct f3 { float x, y, z; };

__device__ __forceinline__ f3 mk(float x, float y, float z) { return {x, y, z}; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ f3 operator-(f3 a) { return {-a.x, -a.y, -a.z}; }
__device__ __forceinline__ f3 operator*(float s, f3 a) { return {s * a.x, s * a.y, s * a.z}; }
__device__ __forceinline__ float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}

struct M3 { float m[9]; };  // row-major
struct Sy { float xx, yy, zz, xy, xz, yz; };
struct SV { f3 w, v; };     // spatial vector [angular; linear]
struct SI { Sy A; M3 B; Sy C; };  // symmetric 6x6 [[A, B], [B^T, C]]

__device__ __forceinline__ f3 mul(const M3& R, f3 v) {
    return {R.m[0] * v.x + R.m[1] * v.y + R.m[2] * v.z, R.m[3] * v.x + R.m[4] * v.y + R.m[5] * v.z,
            R.m[6] * v.x + R.m[7] * v.y + R.m[8] * v.z};
}
__device__ __forceinline__ f3 mulT(const M3& R, f3 v) {
    return {R.m[0] * v.x + R.m[3] * v.y + R.m[6] * v.z, R.m[1] * v.x + R.m[4] * v.y + R.m[7] * v.z,
            R.m[2] * v.x + R.m[5] * v.y + R.m[8] * v.z};
}

// Ground-contact slots of a collision shape (Physics.cpp:687-1219 builds box,
// sphere and cylinder collisions; oracle.c: or_slot_point is the fp64 twin).
// Returns the shape-frame point of slot c: box (h = half extents) corner c
// (bits x y z); sphere its centre (the caller lowers it by the radius);
// cylinder (h = {radius, half length}, axis z): 4 rim points per cap (c & 4:
// the +z cap), 90 degrees apart starting at the rim point deepest along the
// plane normal, so a lying cylinder touches at the exact ends of its contact
// line and a standing one on a square of its rim.  nz = the plane normal (world
// +z) in the shape frame = the third row of the shape's world rotation.
__device__ __forceinline__ f3 shape_slot_point(int type, const float* h, f3 nz, int c) {
    const bool box = (type == 0), cyl = (type == 2);
    float ux = -nz.x, uy = -nz.y;
    const float n2 = ux * ux + uy * uy;
    const bool tilted = n2 > 1e-12f;
    const float inv = tilted ? 1.f / sqrtf(n2) : 0.f;
    ux = tilted ? ux * inv : 1.f;
    uy = tilted ? uy * inv : 0.f;
    const int j = c & 3;  // 0: u, 1: z x u, 2: -u, 3: -(z x u)
    const float dx = (j == 0) ? ux : ((j == 1) ? -uy : ((j == 2) ? -ux : uy));
    const float dy = (j == 0) ? uy : ((j == 1) ? ux : ((j == 2) ? -uy : -ux));
    const float zc = (c & 4) ? h[1] : -h[1];
    return {box ? ((c & 4) ? h[0] : -h[0]) : (cyl ? h[0] * dx : 0.f),
            box ? ((c & 2) ? h[1] : -h[1]) : (cyl ? h[0] * dy : 0.f),
            box ? ((c & 1) ? h[2] : -h[2]) : (cyl ? zc : 0.f)};
}
// third row of Rb SR (the world +z axis in the shape frame)
__device__ __forceinline__ f3 shape_plane_normal(const M3& Rb, const float* SR) {
    return {Rb.m[6] * SR[0] + Rb.m[7] * SR[3] + Rb.m[8] * SR[6], Rb.m[6] * SR[1] + Rb.m[7] * SR[4] + Rb.m[8] * SR[7],
            Rb.m[6] * SR[2] + Rb.m[7] * SR[5] + Rb.m[8] * SR[8]};
}
__device__ __forceinline__ f3 mul(const Sy& S, f3 v) {
    return {S.xx * v.x + S.xy * v.y + S.xz * v.z, S.xy * v.x + S.yy * v.y + S.yz * v.z,
            S.xz * v.x + S.yz * v.y + S.zz * v.z};
}
__device__ __forceinline__ SV operator+(const SV& a, const SV& b) { return {a.w + b.w, a.v + b.v}; }
__device__ __forceinline__ SV operator*(float s, const SV& a) { return {s * a.w, s * a.v}; }
__device__ __forceinline__ float dot(const SV& a, const SV& b) { return dot(a.w, b.w) + dot(a.v, b.v); }

// X = Ad_{T^-1}: parent motion -> child coordinates
__device__ __forceinline__ SV ad_inv(const M3& R, f3 p, const SV& a) {
    return {mulT(R, a.w), mulT(R, a.v - cross(p, a.w))};
}
// X^T: child force -> parent coordinates
__device__ __forceinline__ SV dad_inv(const M3& R, f3 p, const SV& f) {
    const f3 fv = mul(R, f.v);
    return {mul(R, f.w) + cross(p, fv), fv};
}
__device__ __forceinline__ SV mul(const SI& I, const SV& x) {
    // B^T w = (w^T B)^T
    const f3 btw = {I.B.m[0] * x.w.x + I.B.m[3] * x.w.y + I.B.m[6] * x.w.z,
                    I.B.m[1] * x.w.x + I.B.m[4] * x.w.y + I.B.m[7] * x.w.z,
                    I.B.m[2] * x.w.x + I.B.m[5] * x.w.y + I.B.m[8] * x.w.z};
    return {mul(I.A, x.w) + mul(I.B, x.v), btw + mul(I.C, x.v)};
}

// R S R^T for symmetric S
__device__ __forceinline__ Sy rot_sym(const M3& R, const Sy& S) {
    float T[9];  // T = R S
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const f3 row = {R.m[r * 3], R.m[r * 3 + 1], R.m[r * 3 + 2]};
        const f3 c = mul(S, row);  // (R S)_r = S row (S symmetric)
        T[r * 3] = c.x; T[r * 3 + 1] = c.y; T[r * 3 + 2] = c.z;
    }
    auto e = [&](int r, int c) {
        return T[r * 3] * R.m[c * 3] + T[r * 3 + 1] * R.m[c * 3 + 1] + T[r * 3 + 2] * R.m[c * 3 + 2];
    };
    return {e(0, 0), e(1, 1), e(2, 2), e(0, 1), e(0, 2), e(1, 2)};
}
// R B R^T for general B
__device__ __forceinline__ M3 rot_gen(const M3& R, const M3& B) {
    M3 T, O;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c)
            T.m[r * 3 + c] = R.m[r * 3] * B.m[c] + R.m[r * 3 + 1] * B.m[3 + c] + R.m[r * 3 + 2] * B.m[6 + c];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c)
            O.m[r * 3 + c] = T.m[r * 3] * R.m[c * 3] + T.m[r * 3 + 1] * R.m[c * 3 + 1] + T.m[r * 3 + 2] * R.m[c * 3 + 2];
    return O;
}

// X^T I X with X = Ad_{T^-1}, T = (R, p): child articulated inertia -> parent.
//   A' = R A R^T, B' = R B R^T, C' = R C R^T, P = [p]x
//   A_p = A' + P B'^T - B' P - P C' P,  B_p = B' + P C',  C_p = C'
__device__ __forceinline__ SI to_parent(const M3& R, f3 p, const SI& I) {
    const Sy A = rot_sym(R, I.A);
    const M3 B = rot_gen(R, I.B);
    const Sy C = rot_sym(R, I.C);
    // PC = P C'  (column k of C' crossed: P x = p x x)
    const f3 c0 = {C.xx, C.xy, C.xz}, c1 = {C.xy, C.yy, C.yz}, c2 = {C.xz, C.yz, C.zz};
    const f3 pc0 = cross(p, c0), pc1 = cross(p, c1), pc2 = cross(p, c2);  // columns of P C'
    // B_p = B' + P C'
    M3 Bp;
    Bp.m[0] = B.m[0] + pc0.x; Bp.m[1] = B.m[1] + pc1.x; Bp.m[2] = B.m[2] + pc2.x;
    Bp.m[3] = B.m[3] + pc0.y; Bp.m[4] = B.m[4] + pc1.y; Bp.m[5] = B.m[5] + pc2.y;
    Bp.m[6] = B.m[6] + pc0.z; Bp.m[7] = B.m[7] + pc1.z; Bp.m[8] = B.m[8] + pc2.z;
    // Y = P B'^T : column k of B'^T is row k of B'
    const f3 b0 = {B.m[0], B.m[1], B.m[2]}, b1 = {B.m[3], B.m[4], B.m[5]}, b2 = {B.m[6], B.m[7], B.m[8]};
    const f3 y0 = cross(p, b0), y1 = cross(p, b1), y2 = cross(p, b2);  // columns of P B'^T
    // Z = P C' P = (P C') P ; (M P)_{rc} = row_r(M) . column_c(P); P columns: P e_c = p x e_c
    // row r of PC: (pc0.r, pc1.r, pc2.r);  M P = - (P^T M^T)^T ... use M P = -(P M^T)^T
    const f3 r0 = {pc0.x, pc1.x, pc2.x}, r1 = {pc0.y, pc1.y, pc2.y}, r2 = {pc0.z, pc1.z, pc2.z};
    // (PC P)_{rc} = - (p x row_r)_c
    const f3 z0 = -cross(p, r0), z1 = -cross(p, r1), z2 = -cross(p, r2);  // rows of PC'P
    // A_p = A' + Y + Y^T - Z  (since -B'P = (P B'^T)^T = Y^T)
    Sy Ap;
    Ap.xx = A.xx + 2.f * y0.x - z0.x;
    Ap.yy = A.yy + 2.f * y1.y - z1.y;
    Ap.zz = A.zz + 2.f * y2.z - z2.z;
    Ap.xy = A.xy + y1.x + y0.y - z0.y;
    Ap.xz = A.xz + y2.x + y0.z - z0.z;
    Ap.yz = A.yz + y2.y + y1.z - z1.z;
    return {Ap, Bp, C};
}

__device__ __forceinline__ SI& operator+=(SI& a, const SI& b) {
    a.A.xx += b.A.xx; a.A.yy += b.A.yy; a.A.zz += b.A.zz; a.A.xy += b.A.xy; a.A.xz += b.A.xz; a.A.yz += b.A.yz;
#pragma unroll
    for (int k = 0; k < 9; ++k) a.B.m[k] += b.B.m[k];
    a.C.xx += b.C.xx; a.C.yy += b.C.yy; a.C.zz += b.C.zz; a.C.xy += b.C.xy; a.C.xz += b.C.xz; a.C.yz += b.C.yz;
    return a;
}

// AI - psi * U U^T
__device__ __forceinline__ SI downdate(const SI& I, const SV& U, float psi) {
    SI o = I;
    const f3 a = U.w, b = U.v;
    o.A.xx -= psi * a.x * a.x; o.A.yy -= psi * a.y * a.y; o.A.zz -= psi * a.z * a.z;
    o.A.xy -= psi * a.x * a.y; o.A.xz -= psi * a.x * a.z; o.A.yz -= psi * a.y * a.z;
    const float ax[3] = {a.x, a.y, a.z}, bx[3] = {b.x, b.y, b.z};
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) o.B.m[r * 3 + c] -= psi * ax[r] * bx[c];
    o.C.xx -= psi * b.x * b.x; o.C.yy -= psi * b.y * b.y; o.C.zz -= psi * b.z * b.z;
    o.C.xy -= psi * b.x * b.y; o.C.xz -= psi * b.x * b.z; o.C.yz -= psi * b.y * b.z;
    return o;
}

// Per-world dynamic parameters: body masses and gravity in the base frame.
// Nominal values come from the shared block; per-world randomisation
// (kernels.hip: vecenv kernels with RAND) overrides them.  A mass change keeps
// the COM and the rotational inertia about the COM (an SDF <mass> edit).
template <int N>
struct Dyn {
    float m[N];
    f3 g;
};
template <int N>
__device__ __forceinline__ Dyn<N> nominal_dyn(const ChainF* __restrict__ P) {
    Dyn<N> D;
#pragma unroll
    for (int i = 0; i < N; ++i) D.m[i] = P->b[i].mass;
    D.g = {P->g[0], P->g[1], P->g[2]};
    return D;
}

// rotational inertia about the body origin for mass m: the stored Io (for
// b.mass) + (m - b.mass)(|c|^2 1 - c c^T); the correction folds away when
// m is the nominal mass of a constant-folded model
__device__ __forceinline__ Sy inertia_origin(const BodyF& b, float m) {
    const float dm = m - b.mass, cx = b.com[0], cy = b.com[1], cz = b.com[2];
    return {b.Io[0] + dm * (cy * cy + cz * cz), b.Io[1] + dm * (cx * cx + cz * cz),
            b.Io[2] + dm * (cx * cx + cy * cy), b.Io[3] - dm * cx * cy, b.Io[4] - dm * cx * cz,
            b.Io[5] - dm * cy * cz};
}

// rigid-body spatial inertia about the body origin
__device__ __forceinline__ SI rigid(const BodyF& b, float m) {
    SI I;
    I.A = inertia_origin(b, m);
    const float cx = b.com[0], cy = b.com[1], cz = b.com[2];
    // B = m [c]x
    I.B.m[0] = 0.f;     I.B.m[1] = -m * cz; I.B.m[2] = m * cy;
    I.B.m[3] = m * cz;  I.B.m[4] = 0.f;     I.B.m[5] = -m * cx;
    I.B.m[6] = -m * cy; I.B.m[7] = m * cx;  I.B.m[8] = 0.f;
    I.C = {m, m, m, 0.f, 0.f, 0.f};
    return I;
}

// NOTE: select components, never whole structs: `cond ? SV{..} : SV{..}` on
// the runtime joint type becomes a select between two stack objects, i.e.
// scratch stores + loads (seen as 2x WRITE_SIZE in the r01 PMC pass).
__device__ __forceinline__ SV motion(const BodyF& b, float s) {
    const bool rev = ((b.jtype & 1) == 0);
    const float sw = rev ? s : 0.f, sv = rev ? 0.f : s;
    return {{b.axis[0] * sw, b.axis[1] * sw, b.axis[2] * sw}, {b.axis[0] * sv, b.axis[1] * sv, b.axis[2] * sv}};
}
// S^T x.  Both dots are computed and the VALUES selected: written as
// `rev ? dot(a, x.w) : dot(a, x.v)`, SimplifyCFG sinks the common dot into a
// load through a selected address when x is stored, which pins the whole
// stage in scratch memory.  (dot(motion(b, 1), x) avoids that too but cannot
// fold its 0 * x terms for the constant-folded models.)
__device__ __forceinline__ float proj(const BodyF& b, const SV& x) {
    const f3 a = {b.axis[0], b.axis[1], b.axis[2]};
    const float dw = dot(a, x.w);
    const float dv = dot(a, x.v);
    return ((b.jtype & 1) == 0) ? dw : dv;
}

// AI S for the body's joint: revolute S = [a; 0] -> [A a; B^T a],
// prismatic S = [0; a] -> [B a; C a]  (component selects, see motion())
__device__ __forceinline__ SV ais(const SI& AI, const BodyF& b) {
    const bool rev = ((b.jtype & 1) == 0);
    const f3 a = {b.axis[0], b.axis[1], b.axis[2]};
    const f3 Aa = mul(AI.A, a), Bta = mulT(AI.B, a), Ba = mul(AI.B, a), Ca = mul(AI.C, a);
    return {{rev ? Aa.x : Ba.x, rev ? Aa.y : Ba.y, rev ? Aa.z : Ba.z},
            {rev ? Bta.x : Ca.x, rev ? Bta.y : Ca.y, rev ? Bta.z : Ca.z}};
}

// per-body factorization kept for the forward and impulse passes
struct BodyState {
    M3 R;
    f3 p;
    SV U;      // AI S (implicit)
    float psi; // (S^T AI S + dt d)^-1
    float tt;  // total joint force
    SV eta;    // velocity-product acceleration
    float pad_;  // 27 words: an odd record stride keeps LDS lanes conflict-free
};
struct ImpulseFactor {  // non-implicit (only when the model has damping)
    SV U;
    float psi;
};
struct SV7 {  // padded spatial vector (LDS record)
    SV v;
    float pad_;
};

// Per-body storage of one substep ("stage").  RegStage keeps it in VGPRs
// (small models: every index folds after unrolling); LdsStage keeps one
// padded record per (body, lane) in LDS, record stride = 64 lanes, so a
// wave's accesses to one field hit 64 distinct banks.  The generic 7..9-dof
// kernels use LdsStage: in VGPRs their per-body state exceeds the
// 512-register file and spills to scratch (global memory); the constant-folded
// ones fit (kernels.hip: lds_staged).
template <int N, bool DUAL>
struct RegStage {
    BodyState bs_[N];
    ImpulseFactor nf_[DUAL ? N : 1];
    SV own_[N];
    float mv_[N][N];  // M^-1 columns of the active constraint rows
    static constexpr bool kRuntimeColumns = false;
    __device__ __forceinline__ float& mv(int k, int j) { return mv_[k][j]; }
    __device__ __forceinline__ void fence() const {}
    __device__ __forceinline__ BodyState& bs(int i) { return bs_[i]; }
    __device__ __forceinline__ const BodyState& bs(int i) const { return bs_[i]; }
    __device__ __forceinline__ ImpulseFactor& nf(int i) { return nf_[i]; }
    __device__ __forceinline__ const ImpulseFactor& nf(int i) const { return nf_[i]; }
    __device__ __forceinline__ SV& own(int i) { return own_[i]; }
};

constexpr int kLdsLanes = 64;  // LdsStage kernels run one wave per workgroup

template <int N, bool DUAL>
struct LdsStage {
    BodyState* b;       // &records[0][lane]
    ImpulseFactor* f;
    SV7* o;
    float* m;           // M^-1, [N * N][lanes]
    // unrolled columns measured faster than one runtime-J column body
    // (scripts/ab_panda.py, 1024 Panda worlds: 27.7 vs 30.3 us per step)
#ifdef MW_RUNTIME_COLUMNS
    static constexpr bool kRuntimeColumns = true;
#else
    static constexpr bool kRuntimeColumns = false;
#endif
    __device__ __forceinline__ float& mv(int k, int j) const { return m[(k * N + j) * kLdsLanes]; }
    // compiler-only barrier: LDS values are re-read after it instead of being
    // kept live in VGPRs across the unrolled columns / PGS sweeps
    __device__ __forceinline__ void fence() const {
#ifndef MW_HOST_TEST
        asm volatile("" ::: "memory");
#endif
    }
    __device__ __forceinline__ BodyState& bs(int i) const { return b[i * kLdsLanes]; }
    __device__ __forceinline__ ImpulseFactor& nf(int i) const { return f[i * kLdsLanes]; }
    __device__ __forceinline__ SV& own(int i) const { return o[i * kLdsLanes].v; }
};

// LDS words per lane of an LdsStage<N, DUAL>
template <int N, bool DUAL>
constexpr int lds_stage_words() {
    return N * (27 + 7 + (DUAL ? 7 : 0)) + N * N;
}

// 1/x: the hardware reciprocal (1 ulp) on the device, IEEE division on the host
__device__ __forceinline__ float rcp(float x) {
#if defined(MW_HOST_TEST) || !defined(MW_FAST_MATH)
    return 1.f / x;
#else
    return __builtin_amdgcn_rcpf(x);
#endif
}

// sin and cos of a joint angle.  Cody-Waite reduction by pi/2 with a 3-part
// constant and minimax polynomials on [-pi/4, pi/4] (~1 ulp for |q| < 2^16 rad,
// i.e. > 10^4 turns); avoids libm's Payne-Hanek slow path (scratch + branches).
__device__ __forceinline__ void sincos_joint(float x, float* s_out, float* c_out) {
#if defined(MW_FAST_MATH)
    const float k = rintf(x * 0.636619772367581343f);
    float r = fmaf(-k, 1.57079625129699707031f, x);
    r = fmaf(-k, 7.54978941586159635335e-8f, r);
    r = fmaf(-k, 5.39030252995776476554e-15f, r);
    const float r2 = r * r;
    // sin(r) ~ r + r^3 P(r^2), cos(r) ~ 1 - r^2/2 + r^4 Q(r^2)  (Cephes sinf/cosf coefficients)
    const float ps = fmaf(fmaf(-1.9515295891e-4f, r2, 8.3321608736e-3f), r2, -1.6666654611e-1f);
    const float sn = fmaf(ps * r2, r, r);
    const float pc = fmaf(fmaf(2.443315711809948e-5f, r2, -1.388731625493765e-3f), r2, 4.166664568298827e-2f);
    const float cs = fmaf(pc * r2, r2, fmaf(-0.5f, r2, 1.0f));
    const int quad = static_cast<int>(k) & 3;
    const float s1 = (quad & 1) ? cs : sn;
    const float c1 = (quad & 1) ? sn : cs;
    *s_out = (quad & 2) ? -s1 : s1;
    *c_out = ((quad + 1) & 2) ? -c1 : c1;
#else
    sincosf(x, s_out, c_out);
#endif
}

__device__ __forceinline__ void joint_pose(const BodyF& b, float q, M3& R, f3& p) {
    if ((b.jtype & 1) == 0) {
        float s, c;
        sincos_joint(q, &s, &c);
        const float ax = b.axis[0], ay = b.axis[1], az = b.axis[2], v = 1.f - c;
        const float J[9] = {c + ax * ax * v,      ax * ay * v - az * s, ax * az * v + ay * s,
                            ay * ax * v + az * s, c + ay * ay * v,      ay * az * v - ax * s,
                            az * ax * v - ay * s, az * ay * v + ax * s, c + az * az * v};
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int k = 0; k < 3; ++k)
                R.m[r * 3 + k] = b.E[r * 3] * J[k] + b.E[r * 3 + 1] * J[3 + k] + b.E[r * 3 + 2] * J[6 + k];
        p = {b.r[0], b.r[1], b.r[2]};
    } else {
#pragma unroll
        for (int k = 0; k < 9; ++k) R.m[k] = b.E[k];
        p = {b.r[0] + q * b.Ea[0], b.r[1] + q * b.Ea[1], b.r[2] + q * b.Ea[2]};
    }
}

// DART's BallJoint (oracle.c ball_part; Joint.cpp:267-331 exposes it as
// core::JointType::Ball): positions = the rotation vector theta, velocities =
// the child's angular velocity in its own frame (relative Jacobian [I; 0],
// constant), positions integrated on SO(3) as R <- R exp(dt w).  The model
// lists it as three bodies at one point, BodyF::jtype bits 4-5 = part 1, 2, 3
// (unit axes x, y, z; the first two massless): part 1 carries the whole
// rotation E exp(theta), theta = (q_i, q_i+1, q_i+2); parts 2 and 3 have
// identity transforms.  Only the world-per-wavefront and scene kernels step
// such models (sim.cpp routes them there).
__device__ __forceinline__ int ball_part(const BodyF& b) { return (b.jtype >> 4) & 3; }

// E exp(theta) (Rodrigues; 1 - cos t written 2 sin^2(t/2): no cancellation)
__device__ __forceinline__ void ball_rot(const BodyF& b, float tx, float ty, float tz, M3& R) {
    const float t2 = tx * tx + ty * ty + tz * tz;
    const float t = sqrtf(t2);
    float sh, ch;
    sincos_joint(0.5f * t, &sh, &ch);
    const bool tiny = t < 1e-12f;
    const float it = tiny ? 0.f : rcp(t);
    const float A = tiny ? 1.f : 2.f * sh * ch * it;  // sin t / t
    const float hs = tiny ? 0.5f : sh * it;           // sin(t/2) / t
    const float B = 2.f * hs * hs;                    // (1 - cos t) / t^2
    const float K[9] = {0.f, -tz, ty, tz, 0.f, -tx, -ty, tx, 0.f};
    float X[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c)
            X[r * 3 + c] = ((r == c) ? 1.f : 0.f) + A * K[r * 3 + c] +
                           B * (K[r * 3] * K[c] + K[r * 3 + 1] * K[3 + c] + K[r * 3 + 2] * K[6 + c]);
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c)
            R.m[r * 3 + c] = b.E[r * 3] * X[c] + b.E[r * 3 + 1] * X[3 + c] + b.E[r * 3 + 2] * X[6 + c];
}

// joint transform of body i from the tree's coordinates q (a ball joint's
// part 1 reads q[i .. i + 2]; its parts 2 and 3 do not move)
__device__ __forceinline__ void joint_pose_tree(const BodyF& b, const float* q, int i, M3& R, f3& p) {
    const int bp = ball_part(b);
    if (bp == 0) {
        joint_pose(b, q[i], R, p);
        return;
    }
    if (bp == 1) {
        ball_rot(b, q[i], q[i + 1], q[i + 2], R);
    } else {
#pragma unroll
        for (int k = 0; k < 9; ++k) R.m[k] = b.E[k];
    }
    p = {b.r[0], b.r[1], b.r[2]};
}

// the velocity a joint's velocity-product term ad(V, S qd) sees: a ball
// joint's parts 2 and 3 without the ball's earlier parts (one joint of
// constant S; oracle.c joint_bias)
__device__ __forceinline__ SV ball_bias_velocity(const BodyF& b, const float* qd, int i, SV V) {
    const int bp = ball_part(b);
    if (bp >= 2) V.w.x -= qd[i - bp + 1];
    if (bp == 3) V.w.y -= qd[i - 1];
    return V;
}

// f64 constants of the ball-joint integrator: 1/n! for n = 0..23 (Taylor
// coefficients, correctly rounded), then 2 pi as hi + lo and 1 / (2 pi).
// Read through ball_coeffs()'s opaque pointer so that every use loads them
// (off the hot path) instead of the compiler keeping them in registers.
constexpr int kBall2PiHi = 24, kBall2PiLo = 25, kBallInv2Pi = 26;
#ifdef MW_HOST_TEST
static const double kBallConst[27] = {
#else
static __device__ const double kBallConst[27] = {
#endif
    1.0, 1.0, 0.5, 0.16666666666666666, 0.041666666666666664, 0.008333333333333333, 0.001388888888888889,
    0.0001984126984126984, 2.48015873015873e-05, 2.7557319223985893e-06, 2.755731922398589e-07,
    2.505210838544172e-08, 2.08767569878681e-09, 1.6059043836821613e-10, 1.1470745597729725e-11,
    7.647163731819816e-13, 4.779477332387385e-14, 2.8114572543455206e-15, 1.5619206968586225e-16,
    8.22063524662433e-18, 4.110317623312165e-19, 1.9572941063391263e-20, 8.896791392450574e-22,
    3.868170170630684e-23, 6.283185307179586, 2.4492935982947064e-16, 0.15915494309189535};

__device__ __forceinline__ const double* ball_coeffs() {
#ifdef MW_HOST_TEST
    return kBallConst;
#else
    int z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    return kBallConst + z;
#endif
}

// sin and cos of x, |x| <= pi/2: Taylor polynomials to x^23 / x^22 in Horner
// form (truncation below 1e-19 at pi/2)
__device__ __forceinline__ void ball_sincos(double x, const double* C, double& s, double& c) {
    const double x2 = x * x;
    double ps = C[23], pc = C[22];
#pragma unroll
    for (int j = 21; j >= 1; j -= 2) {
        ps = fma(-x2, ps, C[j]);
        pc = fma(-x2, pc, C[j - 1]);
    }
    s = x * ps;
    c = pc;
}

// component k of a ball joint's new position log(exp(theta) exp(dt w)),
// theta = th[0..2], w = w[0..2] (quaternion product; angle in [0, pi])
__device__ __forceinline__ float ball_integrate(float t0, float t1, float t2, float w0, float w1, float w2, float dt,
                                                int k) {
    // fp64: the stored rotation vector is rounded to fp32 once per step
    // (unbiased), but an fp32 composition carries ~1 ulp of systematic error
    // at a slowly moving angle, which drifts (r04r: 5e-5 rad after 500 steps
    // at |theta| = pi/2 against DART's fp64 scheme); one joint part per lane,
    // off the hot path
    // sin / cos / atan2 are this file's own (ball_sincos, below): the
    // library's f64 versions put ~28 f64 polynomial constants in registers
    // for the whole wave kernel (hoisted out of the step loop), 6 of them
    // spilled to scratch (r05)
    const double* C = ball_coeffs();
    auto quat = [C](double x, double y, double z, double (&qt)[4]) {
        const double t = sqrt(x * x + y * y + z * z);
        // t reduced by a multiple of 2 pi: the half-angle's sin and cos
        // change sign together, which negates the quaternion (the product's
        // sign is normalised below)
        const double kk = rint(t * C[kBallInv2Pi]);
        const double tr = fma(-kk, C[kBall2PiLo], fma(-kk, C[kBall2PiHi], t));
        double sn, cs;
        ball_sincos(0.5 * tr, C, sn, cs);
        const double s = (t == 0.0) ? 0.5 : sn / t;
        qt[0] = cs; qt[1] = s * x; qt[2] = s * y; qt[3] = s * z;
    };
    double a[4], b[4];
    const double h = dt;
    quat(t0, t1, t2, a);
    quat(h * w0, h * w1, h * w2, b);
    double c0 = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
    double c1 = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
    double c2 = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
    double c3 = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
    if (c0 < 0.0) { c0 = -c0; c1 = -c1; c2 = -c2; c3 = -c3; }
    const double v = sqrt(c1 * c1 + c2 * c2 + c3 * c3);
    // phi = atan2(v, c0) in [0, pi/2]: the fp32 angle, then one correction
    // phi0 + tan(phi - phi0) (exact up to (phi - phi0)^3 / 3 ~ 1e-22)
    const double p0 = static_cast<double>(atan2f(static_cast<float>(v), static_cast<float>(c0)));
    double sp, cp;
    ball_sincos(p0, C, sp, cp);
    const double phi = p0 + (v * cp - c0 * sp) / (c0 * cp + v * sp);
    const double f = (v == 0.0) ? 2.0 / c0 : 2.0 * phi / v;
    return static_cast<float>(f * ((k == 0) ? c1 : ((k == 1) ? c2 : c3)));
}

// ABA with implicit damping over the kinematic tree TOPO: fills W, returns qdd.
// Per-body temporaries are arrays indexed by compile-time body numbers (every
// loop is unrolled and parent_of() folds), so they stay in VGPRs; for a
// serial chain only one carried articulated inertia is live at a time.
template <int N, bool DUAL, Topo TOPO, class WK>
__device__ __forceinline__ void aba(const ChainF* __restrict__ P, const float (&q)[N],
                                    const float (&qd)[N], const float (&tau)[N], float dt,
                                    float (&qdd)[N], WK& W, const Dyn<N>& D) {
    SV V[N];
    f3 g[N];
    // outward pass: kinematics, velocities, bias forces
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const BodyF& b = P->b[i];
        BodyState& s = W.bs(i);
        const int pa = parent_of(TOPO, i);
        joint_pose(b, q[i], s.R, s.p);
        const SV Sq = motion(b, qd[i]);
        if (pa >= 0) {
            V[i] = ad_inv(s.R, s.p, V[pa]) + Sq;
            g[i] = mulT(s.R, g[pa]);
        } else {
            V[i] = Sq;
            g[i] = mulT(s.R, D.g);
        }
        const SV& Vi = V[i];
        // eta = ad(V, S qd)
        s.eta = {cross(Vi.w, Sq.w), cross(Vi.w, Sq.v) + cross(Vi.v, Sq.w)};
        // h = I V (rigid)
        const f3 c = {b.com[0], b.com[1], b.com[2]};
        const float m = D.m[i];
        const Sy Io = inertia_origin(b, m);
        const f3 hw = mul(Io, Vi.w) + m * cross(c, Vi.v);
        const f3 hv = m * (Vi.v - cross(c, Vi.w));
        // B = -dad(V, IV) - I [0; g]
        W.own(i) = {cross(Vi.w, hw) + cross(Vi.v, hv) - m * cross(c, g[i]),
                    cross(Vi.w, hv) - m * g[i]};
    }
    // inward pass: articulated inertias / biases accumulate into the parent
    SI carry[N];
    SI carryN[DUAL ? N : 1];
    SV carryB[N];
#pragma unroll
    for (int i = N - 1; i >= 0; --i) {
        const BodyF& b = P->b[i];
        BodyState& s = W.bs(i);
        const int pa = parent_of(TOPO, i);
        const bool kids = has_child(TOPO, N, i);
        SI AI = rigid(b, D.m[i]);
        SV Bi = W.own(i);
        if (kids) {
            AI += carry[i];
            Bi = Bi + carryB[i];
        }
        // U = AI S
        s.U = ais(AI, b);
        const float Dss = proj(b, s.U);
        s.psi = rcp(Dss + dt * b.damping);
        const SV AIeta = mul(AI, s.eta);
        s.tt = tau[i] - b.damping * qd[i] - proj(b, AIeta + Bi);
        if constexpr (DUAL) {
            SI AIn = rigid(b, D.m[i]);
            if (kids) AIn += carryN[i];
            const SV Un = ais(AIn, b);
            const float psin = rcp(proj(b, Un));
            W.nf(i).U = Un;
            W.nf(i).psi = psin;
            if (pa >= 0) {
                const SI c = to_parent(s.R, s.p, downdate(AIn, Un, psin));
                if (first_inward(TOPO, N, i)) carryN[pa] = c;
                else carryN[pa] += c;
            }
        }
        if (pa >= 0) {
            const SI c = to_parent(s.R, s.p, downdate(AI, s.U, s.psi));
            const SV beta = Bi + AIeta + (s.psi * s.tt) * s.U;
            const SV cb = dad_inv(s.R, s.p, beta);
            if (first_inward(TOPO, N, i)) { carry[pa] = c; carryB[pa] = cb; }
            else { carry[pa] += c; carryB[pa] = carryB[pa] + cb; }
        }
    }
    // outward pass: accelerations
    SV a[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const BodyF& b = P->b[i];
        const BodyState& s = W.bs(i);
        const int pa = parent_of(TOPO, i);
        if (pa >= 0) {
            const SV ap = ad_inv(s.R, s.p, a[pa]);
            qdd[i] = s.psi * (s.tt - dot(s.U, ap));
            a[i] = ap + s.eta + motion(b, qdd[i]);
        } else {
            qdd[i] = s.psi * s.tt;
            a[i] = s.eta + motion(b, qdd[i]);
        }
    }
}

// column j of M^-1 (velocity change of every dof for a unit impulse on dof j):
// the bias impulse climbs from J to the root (only J's ancestors are
// touched), then the outward pass reaches every body.
template <int N, bool DUAL, Topo TOPO, int J, class WK>
__device__ __forceinline__ void minv_column(const ChainF* __restrict__ P, const WK& W, float (&col)[N]) {
    float u[N];
    SV Bimp[N];
#pragma unroll
    for (int i = N - 1; i >= 0; --i) {
        if (!on_path(TOPO, i, J)) { u[i] = 0.f; continue; }
        u[i] = (i == J) ? 1.f : -proj(P->b[i], Bimp[i]);
        const int pa = parent_of(TOPO, i);
        if (pa >= 0) {
            SV U;
            float psi;
            if constexpr (DUAL) { U = W.nf(i).U; psi = W.nf(i).psi; }
            else { U = W.bs(i).U; psi = W.bs(i).psi; }
            if (i == J) Bimp[pa] = dad_inv(W.bs(i).R, W.bs(i).p, (psi * u[i]) * U);
            else Bimp[pa] = dad_inv(W.bs(i).R, W.bs(i).p, Bimp[i] + (psi * u[i]) * U);
        }
    }
    SV dv[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        SV U;
        float psi;
        if constexpr (DUAL) { U = W.nf(i).U; psi = W.nf(i).psi; }
        else { U = W.bs(i).U; psi = W.bs(i).psi; }
        const int pa = parent_of(TOPO, i);
        if (pa >= 0) {
            const SV dvp = ad_inv(W.bs(i).R, W.bs(i).p, dv[pa]);
            col[i] = psi * (u[i] - dot(U, dvp));
            dv[i] = dvp + motion(P->b[i], col[i]);
        } else {
            col[i] = psi * u[i];
            dv[i] = motion(P->b[i], col[i]);
        }
    }
}

// bit i set: body i is J or an ancestor of J
template <int N>
struct PathMasks {
    uint32_t m[N];
};
template <int N, Topo TOPO>
constexpr PathMasks<N> path_masks() {
    PathMasks<N> p{};
    for (int j = 0; j < N; ++j) {
        uint32_t bits = 0;
        for (int k = j; k >= 0; k = parent_of(TOPO, k)) bits |= 1u << k;
        p.m[j] = bits;
    }
    return p;
}

// column J (uniform, runtime) of M^-1: one copy of the column code for every
// J (LdsStage models), branches on the path mask are scalar
template <int N, bool DUAL, Topo TOPO, class WK>
__device__ __forceinline__ void minv_column_rt(const ChainF* __restrict__ P, const WK& W, int J, uint32_t path,
                                               float (&col)[N]) {
    float u[N];
    SV Bimp[N];
#pragma unroll
    for (int i = N - 1; i >= 0; --i) {
        u[i] = 0.f;
        if (!((path >> i) & 1u)) continue;
        const bool self = (i == J);
        u[i] = self ? 1.f : -proj(P->b[i], Bimp[i]);
        const int pa = parent_of(TOPO, i);
        if (pa >= 0) {
            SV U;
            float psi;
            if constexpr (DUAL) { U = W.nf(i).U; psi = W.nf(i).psi; }
            else { U = W.bs(i).U; psi = W.bs(i).psi; }
            if (self) Bimp[pa] = dad_inv(W.bs(i).R, W.bs(i).p, (psi * u[i]) * U);
            else Bimp[pa] = dad_inv(W.bs(i).R, W.bs(i).p, Bimp[i] + (psi * u[i]) * U);
        }
    }
    SV dv[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        SV U;
        float psi;
        if constexpr (DUAL) { U = W.nf(i).U; psi = W.nf(i).psi; }
        else { U = W.bs(i).U; psi = W.bs(i).psi; }
        const int pa = parent_of(TOPO, i);
        if (pa >= 0) {
            const SV dvp = ad_inv(W.bs(i).R, W.bs(i).p, dv[pa]);
            col[i] = psi * (u[i] - dot(U, dvp));
            dv[i] = dvp + motion(P->b[i], col[i]);
        } else {
            col[i] = psi * u[i];
            dv[i] = motion(P->b[i], col[i]);
        }
    }
}

// the M^-1 columns of the dofs with an active row (bit d of `need`)
template <int N, bool DUAL, Topo TOPO, class WK, int J = 0>
__device__ __forceinline__ void minv_columns(const ChainF* __restrict__ P, WK& W, uint32_t need) {
    if constexpr (WK::kRuntimeColumns) {
        constexpr PathMasks<N> paths = path_masks<N, TOPO>();
        for (int j = 0; j < N; ++j) {
            if ((need >> j) & 1u) {
                float col[N];
                W.fence();
                minv_column_rt<N, DUAL, TOPO>(P, W, j, paths.m[j], col);
#pragma unroll
                for (int k = 0; k < N; ++k) W.mv(k, j) = col[k];
            }
        }
    } else if constexpr (J < N) {
        if ((need >> J) & 1u) {
            float col[N];
            W.fence();
            minv_column<N, DUAL, TOPO, J>(P, W, col);
#pragma unroll
            for (int k = 0; k < N; ++k) W.mv(k, J) = col[k];
        }
        minv_columns<N, DUAL, TOPO, WK, J + 1>(P, W, need);
    }
}

constexpr float kBig = 3.402823466e38f;  // FLT_MAX: "no bound" on the device

// DART constants [EXT]: ERP 0.01, max error-reduction velocity 10
constexpr float kErp = 0.01f;
constexpr float kMaxErv = 10.f;

// One engine substep.  act[i]: kActForce (tau[i] is the clipped command) or
// kActServo (vcmd[i] is the velocity command).  CONS enables the LCP rows.
template <int N, bool DUAL, bool CONS, Topo TOPO, class WK>
__device__ __forceinline__ void substep(const ChainF* __restrict__ P, float (&q)[N], float (&qd)[N],
                                        const float (&tau)[N], const uint8_t (&act)[N],
                                        const float (&vcmd)[N], float dt, int pgs_iters,
                                        float (&qdd)[N], WK& W, const Dyn<N>& D,
                                        float* __restrict__ qlo = nullptr) {
    aba<N, DUAL, TOPO>(P, q, qd, tau, dt, qdd, W, D);
#pragma unroll
    for (int i = 0; i < N; ++i) qd[i] += dt * qdd[i];

    if constexpr (CONS) {
        // rows per dof: 0 limit, 1 servo, 2 Coulomb friction.  Only the
        // right-hand sides are kept; the boxes are recomputed from the uniform
        // parameters (limit: [0, inf) at the lower bound, (-inf, 0] at the
        // upper one; servo +-effort dt; friction +-friction dt).
        uint32_t on = 0u, at_upper = 0u, need = 0u;
        float bb[N][3];
#pragma unroll
        for (int i = 0; i < N; ++i) {
            const BodyF& b = P->b[i];
            bb[i][0] = bb[i][1] = bb[i][2] = 0.f;
            if (b.limited) {
                float viol = q[i] - b.lower;
                bool act_lim = false;
                if (viol <= 0.f) {
                    act_lim = true;
                } else {
                    viol = q[i] - b.upper;
                    if (viol >= 0.f) { act_lim = true; at_upper |= 1u << i; }
                }
                if (act_lim) {
                    on |= 1u << (3 * i);
                    const float bounce = fminf(fmaxf(-viol * kErp * rcp(dt), -kMaxErv), kMaxErv);
                    bb[i][0] = -qd[i] + bounce;
                }
            }
            if (act[i] == kActServo) {
                const float vc = fminf(fmaxf(vcmd[i], -b.vel_limit), b.vel_limit);
                const float err = vc - qd[i];
                if (err != 0.f) { on |= 1u << (3 * i + 1); bb[i][1] = err; }
            }
            if (b.friction != 0.f && qd[i] != 0.f) { on |= 1u << (3 * i + 2); bb[i][2] = -qd[i]; }
            if ((on >> (3 * i)) & 7u) need |= 1u << i;
        }
        if (on) {
            minv_columns<N, DUAL, TOPO, WK>(P, W, need);
            float x[N][3], dq[N];
#pragma unroll
            for (int i = 0; i < N; ++i) { x[i][0] = x[i][1] = x[i][2] = 0.f; dq[i] = 0.f; }
            for (int it = 0; it < pgs_iters; ++it) {
                W.fence();
                // a sweep that moves no impulse is a fixed point: every later
                // sweep would repeat it exactly, so stopping there returns the
                // same bits as running all pgs_iters sweeps
                bool moved = false;
#pragma unroll
                for (int d = 0; d < N; ++d) {
                    if (!((need >> d) & 1u)) continue;
                    const BodyF& b = P->b[d];
                    const float inv_diag = rcp(W.mv(d, d));
#pragma unroll
                    for (int t = 0; t < 3; ++t) {
                        if ((on >> (3 * d + t)) & 1u) {
                            float lo, hi;
                            if (t == 0) {
                                const bool up = (at_upper >> d) & 1u;
                                // unbounded side: FLT_MAX (the kernels are built
                                // finite-math-only, see the Makefile)
                                lo = up ? -kBig : 0.f;
                                hi = up ? 0.f : kBig;
                            } else {
                                hi = (t == 1 ? b.effort : b.friction) * dt;
                                lo = -hi;
                            }
                            const float xn = fminf(fmaxf(x[d][t] + (bb[d][t] - dq[d]) * inv_diag, lo), hi);
                            const float delta = xn - x[d][t];
                            moved |= delta != 0.f;
                            x[d][t] = xn;
#pragma unroll
                            for (int k = 0; k < N; ++k) dq[k] += delta * W.mv(k, d);
                        }
                    }
                }
                if (!moved) break;
            }
            const float inv_dt = rcp(dt);
#pragma unroll
            for (int i = 0; i < N; ++i) {
                qd[i] += dq[i];
                qdd[i] += dq[i] * inv_dt;
            }
        }
    }
    if (qlo) {
        // compensated q += dt qd: (q, qlo) is an unevaluated sum; TwoSum
        // keeps the rounding error of every step in qlo, Fast2Sum renormalises
#pragma unroll
        for (int i = 0; i < N; ++i) {
            const float h = dt * qd[i];
            const float s = q[i] + h;
            const float bv = s - q[i];
            const float err = (q[i] - (s - bv)) + (h - bv);
            const float lo = qlo[i] + err;
            const float hi = s + lo;
            qlo[i] = lo - (hi - s);
            q[i] = hi;
        }
    } else {
#pragma unroll
        for (int i = 0; i < N; ++i) q[i] += dt * qd[i];
    }
}

// register-staged substep (small models)
template <int N, bool DUAL, bool CONS, Topo TOPO = chain_topo(N)>
__device__ __forceinline__ void substep(const ChainF* __restrict__ P, float (&q)[N], float (&qd)[N],
                                        const float (&tau)[N], const uint8_t (&act)[N],
                                        const float (&vcmd)[N], float dt, int pgs_iters,
                                        float (&qdd)[N]) {
    RegStage<N, DUAL> W;
    substep<N, DUAL, CONS, TOPO>(P, q, qd, tau, act, vcmd, dt, pgs_iters, qdd, W, nominal_dyn<N>(P));
}

// register-staged substep with per-world dynamic parameters
template <int N, bool DUAL, bool CONS, Topo TOPO = chain_topo(N)>
__device__ __forceinline__ void substep_dyn(const ChainF* __restrict__ P, float (&q)[N], float (&qd)[N],
                                            const float (&tau)[N], const uint8_t (&act)[N],
                                            const float (&vcmd)[N], float dt, int pgs_iters,
                                            float (&qdd)[N], const Dyn<N>& D) {
    RegStage<N, DUAL> W;
    substep<N, DUAL, CONS, TOPO>(P, q, qd, tau, act, vcmd, dt, pgs_iters, qdd, W, D);
}

}  // namespace dev
}  // namespace mw
