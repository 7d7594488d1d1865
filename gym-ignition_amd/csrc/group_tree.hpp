// group_tree.hpp -- one engine substep of a fixed-base kinematic tree with a
// world spread over a 16-lane row of the wavefront (lane i = body / dof i,
// four worlds per wave64).  Same physics as chain_dyn.hpp (DART 6 World::step
// as driven by Physics.cpp:1824-1835 [EXT]: forward dynamics with implicit
// joint damping, v-integrate, joint-space boxed LCP by projected Gauss-Seidel,
// semi-implicit p-integrate), restated for parallel depth instead of the
// serial Featherstone passes:
//
//   poses      joint transforms per lane, absolute poses by pointer jumping
//              over the parent links (ceil(log2(depth + 1)) rounds)
//   M          composite-rigid-body inertias = subtree sums of the bodies'
//              inertias in a common frame (row suffix scan by DPP), then
//              M[i][j] = S_j . (Ic_i S_i) for every ancestor j of i (CRBA)
//   h          RNEA with qdd = 0 in the common frame: tree prefix sums of
//              S qd (velocities) and of the velocity-product terms
//              (accelerations), per-body forces, subtree sums of the forces
//   solve      (M + dt D) qdd = tau - D qd - h by a Cholesky factorisation
//              distributed over the row (lane i owns row i, DPP broadcasts)
//   LCP        the M^-1 columns of the dofs with an active row by triangular
//              solves; PGS rows as in chain_dyn.hpp (same order, same boxes,
//              same fixed-point exit), dqd distributed over the lanes
//
// (M + dt D) qdd = tau - D qd - h is the joint-space form of DART's implicit
// damping in the ABA (Psi = (S^T A S + dt d)^-1, joint force tau - d qd); the
// impulses use M without the dt D term, as DART's impulse ABA does.
//
// The common frame is the base frame translated to the origin of a body
// half-way down the deepest chain (`ref`): the quadratic forms S^T Ic S of
// distal joints cancel terms ~ m |p|^2 of the lever arm |p| to the frame
// origin, and a mid-chain origin halves |p| (scripts/proto_group_crba.py:
// float32 qdd error 1.7e-2 about the base origin, 3.9e-3 about the elbow's).
#pragma once

#include <hip/hip_runtime.h>

#include <utility>

#include "chain_dyn.hpp"
#include "pid.hpp"

namespace mw {
namespace dev {

constexpr int kGroupLanes = 16;  // lanes per world = one DPP row
constexpr int kGroupMaxBodies = kGroupLanes;

// Phase timing (debug builds only: EXTRA=-DMW_GROUP_PROF, scripts/group_prof.py):
// shader-clock cycles per phase, summed over the worlds of a launch.
constexpr int kGroupProfPhases = 10;   // [9]: PGS sweeps
#ifdef MW_GROUP_PROF
#define MW_GPROF_T(var) const long long var = clock64()
#define MW_GPROF_ACC(k, a, b) (prof[k] += static_cast<unsigned long long>((b) - (a)))
#else
#define MW_GPROF_T(var)
#define MW_GPROF_ACC(k, a, b)
#endif

// ------------------------------------------------ row (16-lane) exchanges
// lane i of every row reads lane K of the same row
template <int K>
__device__ __forceinline__ float row_bcast(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x150 + K, 0xf, 0xf, false));
}
template <int K>
__device__ __forceinline__ int row_bcast_i(int x) {
    return __builtin_amdgcn_update_dpp(0, x, 0x150 + K, 0xf, 0xf, false);
}
// lane i reads lane i + S of the same row, 0 past the row's end (row_shl)
template <int S>
__device__ __forceinline__ float row_down(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x100 + S, 0xf, 0xf, true));
}
// lane i reads lane i - S of the same row, 0 before the row's start (row_shr)
template <int S>
__device__ __forceinline__ float row_up(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x110 + S, 0xf, 0xf, true));
}
// lane i reads lane `src` (row-relative, runtime) of the same row
__device__ __forceinline__ float row_shfl(float x, int src) { return __shfl(x, src, kGroupLanes); }
__device__ __forceinline__ int row_shfl(int x, int src) { return __shfl(x, src, kGroupLanes); }

// compile-time loop: f(std::integral_constant<int, I>) for I = 0..N-1
template <class F, int... I>
__device__ __forceinline__ void sfor_(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
    sfor_(f, std::make_integer_sequence<int, N>{});
}

// sum over lanes i..15 of the row
__device__ __forceinline__ float row_suffix(float x) {
    x += row_down<1>(x);
    x += row_down<2>(x);
    x += row_down<4>(x);
    x += row_down<8>(x);
    return x;
}

// ------------------------------------------------------- per-lane model
// The lane's body (zeros for the padding lanes i >= n).  Topology of the
// row (host-computed, chain_params.hpp: group_topology_words): parent,
// ancestor bit mask, end of the subtree range [i, end) (bodies are numbered
// depth-first, so a subtree is contiguous), and the lane-order chain segment
// the lane belongs to: h = distance to the segment's head (lanes head..i have
// parent(k) = k - 1), hp = the head's parent, level = segments between the
// lane and the root.  Path (root -> i) reductions are a segmented DPP scan
// over the segment plus `level` fix-up rounds from hp.
//
// Lane predicates that the unrolled loops test over and over (i == k,
// i >= k, "k is an ancestor of i", "h >= s") are kept as 0 / 1 floats and
// applied by multiply-add instead of selects: a select needs a 64-bit lane
// mask in SGPRs, and dozens of live masks spill the scalar file.
template <int N>
struct GBody {
    M3 E;
    f3 r, axis, com, Ea;
    Sy Icm;          // rotational inertia about the COM
    float mass, damping, friction, lower, upper, effort;
    int prism, limited, parent;
    int end;         // subtree = bodies [i, end)
    int hp, level;   // lane-order chain segment (chain_params.hpp: group_topology_words)
    float bodyf;     // 1 for a body lane, 0 for padding
    float seg[4];    // h >= 1, 2, 4, 8
    float eq[N], ge[N], anc[N];  // i == k, i >= k, k is an ancestor of i
};

template <int N>
__device__ __forceinline__ GBody<N> load_gbody(const ChainF* __restrict__ P, int li, int n) {
    GBody<N> g{};
    const bool body = li < n;
    // padding lanes read body 0 and zero what they read (no branches: the
    // struct stays in registers)
    const BodyF& b = P->b[body ? li : 0];
    const float bf = body ? 1.f : 0.f;
#pragma unroll
    for (int k = 0; k < 9; ++k) g.E.m[k] = body ? b.E[k] : ((k % 4 == 0) ? 1.f : 0.f);
    g.r = bf * f3{b.r[0], b.r[1], b.r[2]};
    g.axis = bf * f3{b.axis[0], b.axis[1], b.axis[2]};
    g.com = bf * f3{b.com[0], b.com[1], b.com[2]};
    g.Ea = bf * f3{b.Ea[0], b.Ea[1], b.Ea[2]};
    const float m = bf * b.mass, cx = b.com[0], cy = b.com[1], cz = b.com[2];
    // Io (about the body origin) -> about the COM: Io - m (|c|^2 1 - c c^T)
    g.Icm = {bf * b.Io[0] - m * (cy * cy + cz * cz), bf * b.Io[1] - m * (cx * cx + cz * cz),
             bf * b.Io[2] - m * (cx * cx + cy * cy), bf * b.Io[3] + m * cx * cy, bf * b.Io[4] + m * cx * cz,
             bf * b.Io[5] + m * cy * cz};
    g.mass = m;
    g.damping = bf * b.damping;
    g.friction = bf * b.friction;
    g.lower = b.lower;
    g.upper = b.upper;
    g.effort = b.effort;
    g.prism = body ? (b.jtype & 1) : 0;
    g.limited = body ? b.limited : 0;
    g.parent = body ? b.parent : -1;
    const uint32_t anc = body ? b.anc : 0u;
    g.end = body ? b.end : li + 1;
    const int seg = body ? b.seg : 0;
    const int h = seg & 0xff;
    g.hp = ((seg >> 8) & 0xff) - 1;
    g.level = (seg >> 16) & 0xff;
    g.bodyf = bf;
    g.seg[0] = h >= 1 ? 1.f : 0.f;
    g.seg[1] = h >= 2 ? 1.f : 0.f;
    g.seg[2] = h >= 4 ? 1.f : 0.f;
    g.seg[3] = h >= 8 ? 1.f : 0.f;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        g.eq[k] = (li == k) ? 1.f : 0.f;
        g.ge[k] = (li >= k) ? 1.f : 0.f;
        g.anc[k] = ((anc >> k) & 1u) ? 1.f : 0.f;
    }
    return g;
}

// ----------------------------------------------------- tree prefix sums
// Row topology of the model (uniform): Hillis-Steele steps of the segmented
// scans, the number of segment levels, the common frame's body
struct GTopo {
    int steps, levels, ref;
    int fix;   // the one head parent of the level-1 segments, or -1
    int dend;  // the one subtree end before n, or -1
    bool diff; // some subtree ends before n
};
__device__ __forceinline__ GTopo load_gtopo(const ChainF* __restrict__ P) {
    const int a = P->gtopo, b = P->gtopo2;
    return {(a >> 16) & 0xff, (a >> 8) & 0xff, a & 0xff, (b & 0xff) - 1, ((b >> 8) & 0xff) - 1, ((b >> 16) & 1) != 0};
}

// f(std::integral_constant<int, K>) for the uniform runtime lane k: one
// uniform branch picks the instance, whose broadcasts are DPP row_newbcast:K
template <class F>
__device__ __forceinline__ void with_lane(int k, F&& f) {
    sfor<kGroupLanes>([&](auto K) {
        if (k == K) f(K);
    });
}

// x_i <- sum of x over i and its ancestors
template <int K, int N>
__device__ __forceinline__ void tree_prefix(float (&x)[K], const GBody<N>& B, const GTopo& T, int li) {
    auto step = [&](auto S) {
        constexpr int s = S;
        constexpr int e = (s == 1) ? 0 : (s == 2) ? 1 : (s == 4) ? 2 : 3;
#pragma unroll
        for (int k = 0; k < K; ++k) x[k] = fmaf(row_up<s>(x[k]), B.seg[e], x[k]);
    };
    if (T.steps > 0) step(std::integral_constant<int, 1>{});
    if (T.steps > 1) step(std::integral_constant<int, 2>{});
    if (T.steps > 2) step(std::integral_constant<int, 4>{});
    if (T.steps > 3) step(std::integral_constant<int, 8>{});
    if (T.fix >= 0) {
        // one level-1 segment head parent: DPP broadcasts
        const float fm = (B.level == 1) ? 1.f : 0.f;
        with_lane(T.fix, [&](auto L) {
#pragma unroll
            for (int k = 0; k < K; ++k) x[k] = fmaf(row_bcast<L>(x[k]), fm, x[k]);
        });
        return;
    }
    for (int r = 1; r <= T.levels; ++r) {
        const bool fix = B.level == r;
        const float fm = fix ? 1.f : 0.f;
        const int src = fix ? B.hp : li;
#pragma unroll
        for (int k = 0; k < K; ++k) x[k] = fmaf(row_shfl(x[k], src), fm, x[k]);
    }
}

// (R, p) <- X_root ... X_parent X_i: the same segmented scan with pose
// composition (X_a X_b = (R_a R_b, R_a p_b + p_a)) as the operator; a lane
// that does not take part composes with the identity (m = 0)
__device__ __forceinline__ void compose_masked(M3 Ra, f3 pa, float m, M3& R, f3& p) {
    const float m1 = 1.f - m;
#pragma unroll
    for (int k = 0; k < 9; ++k) Ra.m[k] *= m;
    Ra.m[0] += m1; Ra.m[4] += m1; Ra.m[8] += m1;
    pa = m * pa;
    p = mul(Ra, p) + pa;
    M3 Rn;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int k = 0; k < 3; ++k)
            Rn.m[r * 3 + k] = Ra.m[r * 3] * R.m[k] + Ra.m[r * 3 + 1] * R.m[3 + k] + Ra.m[r * 3 + 2] * R.m[6 + k];
    R = Rn;
}
template <int N>
__device__ __forceinline__ void tree_poses(M3& R, f3& p, const GBody<N>& B, const GTopo& T, int li) {
    auto step = [&](auto S) {
        constexpr int s = S;
        constexpr int e = (s == 1) ? 0 : (s == 2) ? 1 : (s == 4) ? 2 : 3;
        M3 Ra;
#pragma unroll
        for (int k = 0; k < 9; ++k) Ra.m[k] = row_up<s>(R.m[k]);
        const f3 pa = {row_up<s>(p.x), row_up<s>(p.y), row_up<s>(p.z)};
        compose_masked(Ra, pa, B.seg[e], R, p);
    };
    if (T.steps > 0) step(std::integral_constant<int, 1>{});
    if (T.steps > 1) step(std::integral_constant<int, 2>{});
    if (T.steps > 2) step(std::integral_constant<int, 4>{});
    if (T.steps > 3) step(std::integral_constant<int, 8>{});
    if (T.fix >= 0) {
        with_lane(T.fix, [&](auto L) {
            M3 Ra;
#pragma unroll
            for (int k = 0; k < 9; ++k) Ra.m[k] = row_bcast<L>(R.m[k]);
            const f3 pa = {row_bcast<L>(p.x), row_bcast<L>(p.y), row_bcast<L>(p.z)};
            compose_masked(Ra, pa, (B.level == 1) ? 1.f : 0.f, R, p);
        });
        return;
    }
    for (int r = 1; r <= T.levels; ++r) {
        const bool fix = B.level == r;
        const int src = fix ? B.hp : li;
        M3 Ra;
#pragma unroll
        for (int k = 0; k < 9; ++k) Ra.m[k] = row_shfl(R.m[k], src);
        const f3 pa = {row_shfl(p.x, src), row_shfl(p.y, src), row_shfl(p.z, src)};
        compose_masked(Ra, pa, fix ? 1.f : 0.f, R, p);
    }
}

// x_i <- sum of x over the subtree of i: suffix sums of the row minus the
// suffix past the subtree's end (exact when the subtree runs to the row's
// end or the rest is zero; diff: some body's subtree ends before n)
template <int K>
__device__ __forceinline__ void subtree_sum(float (&x)[K], int end, int li, const GTopo& T) {
#pragma unroll
    for (int k = 0; k < K; ++k) x[k] = row_suffix(x[k]);
    if (T.dend >= 0) {
        // one subtree end before n: DPP broadcasts
        const float sm = (end == T.dend) ? 1.f : 0.f;
        with_lane(T.dend, [&](auto L) {
#pragma unroll
            for (int k = 0; k < K; ++k) x[k] = fmaf(-row_bcast<L>(x[k]), sm, x[k]);
        });
    } else if (T.diff) {
        const bool sub = end < kGroupLanes;
        const float sm = sub ? 1.f : 0.f;
        const int src = sub ? end : li;
#pragma unroll
        for (int k = 0; k < K; ++k) x[k] = fmaf(-row_shfl(x[k], src), sm, x[k]);
    }
}

// ------------------------------------------------- Cholesky over the row
// Lane i holds row i of an N x N SPD matrix (r[j], j <= i; the diagonal at
// j = i).  After row_factor(): r[j] = L[i][j] (j < i), r[i] = L[i][i];
// ct[j] = L[j][i] (j > i: lane i's column of L, zero for j <= i); inv[k] =
// 1 / L[k][k] in every lane of the row.  The entries right of the diagonal
// (r[j], j > i) are updated like the others and never read: no lane masks
// in the elimination.
template <int N>
struct RowChol {
    float r[N], ct[N], inv[N];
};

template <int N, int M>
__device__ __forceinline__ void row_factor(RowChol<N>& C, const GBody<M>& B) {
    sfor<N>([&](auto K) {
        constexpr int k = K;
        const float dk = row_bcast<k>(C.r[k]);
        const float ik = __builtin_amdgcn_rsqf(dk);
        C.inv[k] = ik;
        const float lik = C.r[k] * ik;  // lane k: sqrt(dk); lanes i > k: L[i][k]
        C.r[k] = lik;
        sfor<N - k - 1>([&](auto J) {
            constexpr int j = k + 1 + J;
            const float ljk = row_bcast<j>(lik);
            C.r[j] = fmaf(-lik, ljk, C.r[j]);
            C.ct[j] = fmaf(B.eq[k], ljk, C.ct[j]);
        });
    });
}

// solve L L^T x = b (lane i holds b_i, returns x_i); the right-hand side is
// zero above row K0 (unit columns: K0 = the column's dof)
template <int N, int K0 = 0, int M>
__device__ __forceinline__ float row_solve(const RowChol<N>& C, float b, const GBody<M>& B) {
    float y = 0.f;
    sfor<N - K0>([&](auto KK) {
        constexpr int k = K0 + KK;
        const float yk = row_bcast<k>(b) * C.inv[k];
        y = fmaf(B.eq[k], yk, y);
        b = fmaf(-C.r[k], yk, b);  // rows i > k; i <= k are done
    });
    float x = 0.f;
    sfor<N>([&](auto KK) {
        constexpr int k = N - 1 - KK;
        const float xk = row_bcast<k>(y) * C.inv[k];
        x = fmaf(B.eq[k], xk, x);
        y = fmaf(-C.ct[k], xk, y);  // ct[k] = 0 in lanes i >= k
    });
    return x;
}

// spatial helpers in the common frame (inertia as mass, first moment h = m c
// and rotational inertia J about the frame origin)
struct GI {
    float m;
    f3 h;
    Sy J;
};
__device__ __forceinline__ SV gmul(const GI& I, const SV& V) {
    return {mul(I.J, V.w) + cross(I.h, V.v), I.m * V.v - cross(I.h, V.w)};
}

// ------------------------------------------------------------- substep
// Lane li (< n: body li) of a world.  q, qd, qlo: this lane's joint; tau its
// force.  Returns with q, qd (and qlo) advanced by one substep.
template <int N, bool DUAL, bool CONS>
__device__ __forceinline__ void group_substep(const GBody<N>& B, int li, int n, const GTopo& T,
                                              f3 grav, float& q, float& qd, float& qlo, float tau, float dt,
                                              float inv_dt, int pgs_iters,
                                              unsigned long long (&prof)[kGroupProfPhases]) {
    (void)prof;
    (void)n;
    MW_GPROF_T(t0);
    // joint pose in the parent frame
    M3 R;
    f3 p;
    if (!B.prism) {
        float s, c;
        sincos_joint(q, &s, &c);
        const float ax = B.axis.x, ay = B.axis.y, az = B.axis.z, v = 1.f - c;
        const float J[9] = {c + ax * ax * v,      ax * ay * v - az * s, ax * az * v + ay * s,
                            ay * ax * v + az * s, c + ay * ay * v,      ay * az * v - ax * s,
                            az * ax * v - ay * s, az * ay * v + ax * s, c + az * az * v};
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int k = 0; k < 3; ++k)
                R.m[r * 3 + k] = B.E.m[r * 3] * J[k] + B.E.m[r * 3 + 1] * J[3 + k] + B.E.m[r * 3 + 2] * J[6 + k];
        p = B.r;
    } else {
        R = B.E;
        p = B.r + q * B.Ea;
    }
    // absolute poses
    tree_poses(R, p, B, T, li);
    // common frame: origin at body T.ref's origin (uniform: one DPP broadcast)
    {
        f3 pr = {0.f, 0.f, 0.f};
        with_lane(T.ref, [&](auto K) { pr = {row_bcast<K>(p.x), row_bcast<K>(p.y), row_bcast<K>(p.z)}; });
        p = p - pr;
    }
    MW_GPROF_T(t1);
    MW_GPROF_ACC(1, t0, t1);
    // joint motion subspace, rigid inertia
    const f3 a0 = mul(R, B.axis);
    SV S;
    if (!B.prism) S = {a0, cross(p, a0)};
    else S = {{0.f, 0.f, 0.f}, a0};
    GI I;
    {
        const f3 c0 = mul(R, B.com) + p;
        const Sy Jr = rot_sym(R, B.Icm);
        const float m = B.mass, cc = dot(c0, c0);
        I.m = m;
        I.h = m * c0;
        I.J = {Jr.xx + m * (cc - c0.x * c0.x), Jr.yy + m * (cc - c0.y * c0.y), Jr.zz + m * (cc - c0.z * c0.z),
               Jr.xy - m * c0.x * c0.y,        Jr.xz - m * c0.x * c0.z,        Jr.yz - m * c0.y * c0.z};
    }
    // composite inertia of the subtree
    float ci[10] = {I.m, I.h.x, I.h.y, I.h.z, I.J.xx, I.J.yy, I.J.zz, I.J.xy, I.J.xz, I.J.yz};
    subtree_sum<10>(ci, B.end, li, T);
    const GI Ic = {ci[0], {ci[1], ci[2], ci[3]}, {ci[4], ci[5], ci[6], ci[7], ci[8], ci[9]}};
    const SV F = gmul(Ic, S);
    // rows of M (implicit: + dt d on the diagonal); padding lanes: unit rows
    RowChol<N> C;
    RowChol<(DUAL && CONS) ? N : 1> Cn;
    {
        const float diag = fmaf(B.bodyf, dot(S, F) - 1.f, 1.f);
        const float diag_i = diag + dt * B.damping;
        sfor<N>([&](auto J) {
            constexpr int j = J;
            float mij = 0.f;
            if constexpr (j < N - 1) {
                const SV Sj = {{row_bcast<j>(S.w.x), row_bcast<j>(S.w.y), row_bcast<j>(S.w.z)},
                               {row_bcast<j>(S.v.x), row_bcast<j>(S.v.y), row_bcast<j>(S.v.z)}};
                mij = B.anc[j] * dot(Sj, F);
            }
            C.r[j] = fmaf(B.eq[j], diag_i, mij);
            if constexpr (DUAL && CONS) Cn.r[j] = fmaf(B.eq[j], diag, mij);
            C.ct[j] = 0.f;
            C.inv[j] = 0.f;
            if constexpr (DUAL && CONS) { Cn.ct[j] = 0.f; Cn.inv[j] = 0.f; }
        });
    }
    MW_GPROF_T(t2);
    MW_GPROF_ACC(2, t1, t2);
    // bias forces (RNEA, qdd = 0, base acceleration -g)
    float hb;
    {
        const SV Sq = qd * S;
        float v6[6] = {Sq.w.x, Sq.w.y, Sq.w.z, Sq.v.x, Sq.v.y, Sq.v.z};
        tree_prefix<6>(v6, B, T, li);
        const SV V = {{v6[0], v6[1], v6[2]}, {v6[3], v6[4], v6[5]}};
        // velocity-product acceleration V x S qd (= V_parent x S qd)
        const SV cv = {cross(V.w, Sq.w), cross(V.w, Sq.v) + cross(V.v, Sq.w)};
        float a6[6] = {cv.w.x, cv.w.y, cv.w.z, cv.v.x, cv.v.y, cv.v.z};
        tree_prefix<6>(a6, B, T, li);
        const SV A = {{a6[0], a6[1], a6[2]}, {a6[3] - grav.x, a6[4] - grav.y, a6[5] - grav.z}};
        const SV IV = gmul(I, V);
        const SV IA = gmul(I, A);
        float f6[6];
        {
            const f3 fw = IA.w + cross(V.w, IV.w) + cross(V.v, IV.v);
            const f3 fv = IA.v + cross(V.w, IV.v);
            f6[0] = fw.x; f6[1] = fw.y; f6[2] = fw.z; f6[3] = fv.x; f6[4] = fv.y; f6[5] = fv.z;
        }
        subtree_sum<6>(f6, B.end, li, T);
        hb = dot(S, SV{{f6[0], f6[1], f6[2]}, {f6[3], f6[4], f6[5]}});
    }
    MW_GPROF_T(t3);
    MW_GPROF_ACC(3, t2, t3);
    row_factor<N>(C, B);
    const float rhs = B.bodyf * (tau - B.damping * qd - hb);
    float qdd = row_solve<N>(C, rhs, B);
    qd += dt * qdd;
    MW_GPROF_T(t4);
    MW_GPROF_ACC(4, t3, t4);

    if constexpr (CONS) {
        // rows of this lane's dof: 0 limit, 2 Coulomb friction (no servo rows:
        // the JointController drives Position / Velocity joints by force)
        uint32_t on = 0u;
        bool up = false;
        float b0 = 0.f, b2 = 0.f;
        if (B.limited) {
            float viol = q - B.lower;
            bool act = false;
            if (viol <= 0.f) {
                act = true;
            } else {
                viol = q - B.upper;
                if (viol >= 0.f) { act = true; up = true; }
            }
            if (act) {
                on |= 1u;
                const float bounce = fminf(fmaxf(-viol * kErp * inv_dt, -kMaxErv), kMaxErv);
                b0 = -qd + bounce;
            }
        }
        if (B.friction != 0.f && qd != 0.f) { on |= 4u; b2 = -qd; }
        // the wave skips the LCP when no world of it has a row
        if (__any(on != 0u)) {
            if constexpr (DUAL) row_factor<N>(Cn, B);
            float mc[N], invd[N], rb0[N], rb2[N], lo0[N], hi0[N], a0m[N], a2m[N], x0[N], x2[N];
            // dofs with a limit / friction row in some world of the wave: the
            // union of the four 16-lane slices of the ballots (scalar ops)
            auto rows_of = [](uint64_t m) {
                return static_cast<uint32_t>((m | (m >> 16) | (m >> 32) | (m >> 48)) & 0xffffu);
            };
            const uint32_t rows0 = rows_of(__ballot((on & 1u) != 0u));
            const uint32_t rows2 = rows_of(__ballot((on & 4u) != 0u));
            const float onf0 = (on & 1u) ? 1.f : 0.f, onf2 = (on & 4u) ? 1.f : 0.f, upf = up ? 1.f : 0.f;
            sfor<N>([&](auto D) {
                constexpr int d = D;
                x0[d] = x2[d] = 0.f;
                mc[d] = invd[d] = rb0[d] = rb2[d] = a0m[d] = a2m[d] = lo0[d] = hi0[d] = 0.f;
                if (((rows0 | rows2) >> d) & 1u) {
                    // row constants of dof d, uniform over the world's lanes
                    rb0[d] = row_bcast<d>(b0);
                    rb2[d] = row_bcast<d>(b2);
                    a0m[d] = row_bcast<d>(onf0);
                    a2m[d] = row_bcast<d>(onf2);
                    const float u = row_bcast<d>(upf);
                    lo0[d] = u != 0.f ? -kBig : 0.f;
                    hi0[d] = u != 0.f ? 0.f : kBig;
                    // M^-1 column d
                    if constexpr (DUAL) mc[d] = row_solve<N, d>(Cn, B.eq[d], B);
                    else mc[d] = row_solve<N, d>(C, B.eq[d], B);
                    invd[d] = rcp(row_bcast<d>(mc[d]));
                }
            });
            MW_GPROF_T(t5);
            MW_GPROF_ACC(5, t4, t5);
            float dq = 0.f;
            for (int it = 0; it < pgs_iters; ++it) {
                float moved = 0.f;
                sfor<N>([&](auto D) {
                    constexpr int d = D;
                    if ((rows0 >> d) & 1u) {
                        const float xn = fminf(fmaxf(x0[d] + (rb0[d] - row_bcast<d>(dq)) * invd[d], lo0[d]), hi0[d]);
                        const float delta = (xn - x0[d]) * a0m[d];
                        moved = fmaxf(moved, fabsf(delta));
                        x0[d] += delta;
                        dq = fmaf(delta, mc[d], dq);
                    }
                    if ((rows2 >> d) & 1u) {
                        // friction bound of dof d (uniform: the model is shared)
                        const float fr = row_bcast<d>(B.friction) * dt;
                        const float xn = fminf(fmaxf(x2[d] + (rb2[d] - row_bcast<d>(dq)) * invd[d], -fr), fr);
                        const float delta = (xn - x2[d]) * a2m[d];
                        moved = fmaxf(moved, fabsf(delta));
                        x2[d] += delta;
                        dq = fmaf(delta, mc[d], dq);
                    }
                });
#ifdef MW_GROUP_PROF
                prof[9] += 1;
#endif
                // a sweep that moves no impulse in any world of the wave is a
                // fixed point of every one of them (chain_dyn.hpp: substep)
                if (!__any(moved != 0.f)) break;
            }
            qd += dq;
            qdd += dq * inv_dt;
            MW_GPROF_T(t6);
            MW_GPROF_ACC(6, t5, t6);
        }
    }
    // compensated q += dt qd (chain_dyn.hpp: substep)
    const float h = dt * qd;
    const float s = q + h;
    const float bv = s - q;
    const float err = (q - (s - bv)) + (h - bv);
    const float lo = qlo + err;
    const float hi = s + lo;
    qlo = lo - (hi - s);
    q = hi;
    (void)qdd;
}

}  // namespace dev
}  // namespace mw
