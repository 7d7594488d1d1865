// wave_crba.hpp -- the world-per-wavefront step (wave_tree.hpp) in joint
// space: the same physics as wave_step (DART 6 World::step restated [EXT],
// reached from /root/reference/cpp/scenario/plugins/Physics/Physics.cpp:1824-1835;
// oracle.c or_float_step), with the tree phases restated as dense linear
// algebra on the matrix cores instead of the articulated-body recursions:
//
//   forward     level-parallel (lane = body): joint transforms, velocities,
//               world poses, the velocity-product terms and the RNEA
//               accelerations with qdd = 0 (gravity enters through the bias
//               forces, as in the ABA)
//   backward    level-parallel: composite rigid-body inertias Ic and composite
//               bias forces fc (no articulated downdate)
//   CRBA        lane = body i: M[i][i] = S_i^T Ic_i S_i, then up its ancestor
//               path M[j][i] = S_j^T X^T ... Ic_i S_i, the base block Ic_0; the
//               bias h_i = S_i^T fc_i.  M is stored in REVERSED dof order (the
//               deepest dofs first, the base's six last): the elimination
//               order of the ABA, no fill-in
//   solve       (M + dt D) [a0; qdd] = [0; tau - D qd] - h by the block LDL^T
//               of wave_lcp.hpp (one v_mfma_f32_32x32x2_f32 per tile and per
//               pair of dofs) -- DART's implicit joint damping; a damped model
//               factors M once more without D for the impulses (DART's impulse
//               dynamics use the non-implicit inertias)
//   rows        J (lane = row) by the inward walk of wave_response without its
//               impulse recursion, then Y = D^-1/2 L^-1 J^T by a forward
//               substitution over the dof pairs (L columns uniform from LDS)
//   Delassus    A = Y^T Y on the matrix cores (positive semidefinite by
//               construction), the CFM on its diagonal
//   impulses    dnu = M^-1 J^T x = L^-T D^-1/2 (Y x): one back substitution
//
// Capacities as wave_step.  LDS: M in the responses' stack (dead: no response
// pass), L in the MJ rows, Y in the J rows.
#pragma once

namespace mw {
namespace dev {

// M row stride in the stack region (row-major; lane c reads row rr at column c)
constexpr int kCrbaMStride = 64;

// A composite rigid-body inertia in 10 numbers (a subtree is a rigid body
// while its joints are held): mass, first moment h = m c and the rotational
// inertia about the body ORIGIN.  Moving it to the parent frame is ~75 FMAs
// against ~200 for the 6x6 congruence of an articulated inertia (to_parent).
struct Rigid10 {
    float m;
    f3 h;
    Sy I;
};
// the accumulator of a body's children (the wave kernel's WaveAcc slot, reused)
struct CrbaAcc {
    Rigid10 I;
    SV B;
};

__device__ __forceinline__ Rigid10 rigid10(const BodyF& b) {
    return {b.mass, mk(b.mass * b.com[0], b.mass * b.com[1], b.mass * b.com[2]), inertia_origin(b, b.mass)};
}
__device__ __forceinline__ Rigid10 operator+(const Rigid10& a, const Rigid10& b) {
    return {a.m + b.m, a.h + b.h,
            {a.I.xx + b.I.xx, a.I.yy + b.I.yy, a.I.zz + b.I.zz, a.I.xy + b.I.xy, a.I.xz + b.I.xz, a.I.yz + b.I.yz}};
}
// child (R, p: the child's orientation and origin in the parent frame) ->
// parent: h' = R h + m p, I' = R I R^T - [p]x[Rh]x - [Rh]x[p]x - m [p]x^2
// ([a]x[b]x = b a^T - (a.b) 1)
__device__ __forceinline__ Rigid10 to_parent10(const M3& R, const f3& p, const Rigid10& X) {
    const f3 hr = mul(R, X.h);
    const Sy Ir = rot_sym(R, X.I);
    const float ph = dot(p, hr), pp = dot(p, p);
    const float dg = 2.f * ph + X.m * pp;
    Sy I;
    I.xx = Ir.xx - 2.f * hr.x * p.x - X.m * p.x * p.x + dg;
    I.yy = Ir.yy - 2.f * hr.y * p.y - X.m * p.y * p.y + dg;
    I.zz = Ir.zz - 2.f * hr.z * p.z - X.m * p.z * p.z + dg;
    I.xy = Ir.xy - hr.x * p.y - p.x * hr.y - X.m * p.x * p.y;
    I.xz = Ir.xz - hr.x * p.z - p.x * hr.z - X.m * p.x * p.z;
    I.yz = Ir.yz - hr.y * p.z - p.y * hr.z - X.m * p.y * p.z;
    return {X.m, hr + X.m * p, I};
}
// the 6 x 6 form [[I, [h]x], [[h]x^T, m 1]] (rigid() of chain_dyn.hpp)
__device__ __forceinline__ SI si_of(const Rigid10& X) {
    SI S;
    S.A = X.I;
    S.B.m[0] = 0.f;      S.B.m[1] = -X.h.z; S.B.m[2] = X.h.y;
    S.B.m[3] = X.h.z;    S.B.m[4] = 0.f;    S.B.m[5] = -X.h.x;
    S.B.m[6] = -X.h.y;   S.B.m[7] = X.h.x;  S.B.m[8] = 0.f;
    S.C = {X.m, X.m, X.m, 0.f, 0.f, 0.f};
    return S;
}

// the tile width of the joint-space factorisation
template <int MAXN>
struct CrbaDims {
    static constexpr int kNv = 6 + MAXN;
    static constexpr int kNvp = (kNv + 1) & ~1;               // dof pairs
    static constexpr int kLs = WaveWorld<MAXN>::kRowStride;   // L column stride (odd)
    static_assert(kLs >= kNvp, "L record fits the MJ rows");
};

// (M + diag) tiles from the LDS matrix Mm (row-major, stride kCrbaMStride,
// nv x nv): free x free entries, identity elsewhere; dd = this lane's diagonal
// addition for dof c (T00) and 32 + c (T01 / T11)
template <int RC>
__device__ __forceinline__ void crba_tiles(const float* __restrict__ Mm, uint64_t freeM, float dd0, float dd1,
                                           v16f& T00, v16f& T01, v16f& T11) {
    const int lane = lane_id();
    const int c = lane & 31;
    const bool hi = lane >= 32;
    const bool cf0 = mask_bit(freeM, c), cf1 = mask_bit(freeM, 32 + c);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int r0 = 8 * (i / 4) + (i % 4);
        const int rr = hi ? r0 + 4 : r0;
        const bool rf = mask_bit(freeM, rr);
        const float v = Mm[rr * kCrbaMStride + c] + ((rr == c) ? dd0 : 0.f);
        T00[i] = (rf && cf0) ? v : ((rr == c) ? 1.f : 0.f);
        if constexpr (RC == 64) {
            T01[i] = (rf && cf1) ? Mm[rr * kCrbaMStride + 32 + c] : 0.f;
            const bool rf1 = mask_bit(freeM, 32 + rr);
            const float w = Mm[(32 + rr) * kCrbaMStride + 32 + c] + ((rr == c) ? dd1 : 0.f);
            T11[i] = (rf1 && cf1) ? w : ((rr == c) ? 1.f : 0.f);
        }
    }
}

// Factor (M + diag) over the free dofs, L to Lw (stride LS, rows < LROWS),
// 1/sqrt(d) per dof to dsq (if given); returns the solution of the system
// with right-hand side rhs (lane = row; held rows 0).
template <int RC, int LS, int LROWS>
__device__ __forceinline__ float crba_ldl(const float* __restrict__ Mm, uint64_t freeM, float dd0, float dd1, float rhs,
                                          float* Lw, float* dsq) {
    MfmaLdl<RC, LS, LROWS> M;
    M.freeM = freeM;
    M.Lw = Lw;
    M.dsq = dsq;
    M.T01 = v16f{};
    M.T11 = v16f{};
    crba_tiles<RC>(Mm, freeM, dd0, dd1, M.T00, M.T01, M.T11);
    wave_lds_sync();  // Lw may alias nothing read above, but keep the tile reads before the L stores
    M.r = mask_bit(freeM, lane_id()) ? rhs : 0.f;
    M.y = 0.f;
    M.template forward<0>();
    wave_lds_sync();
    ldl_backward<RC - 2, LS>(M.y, freeM, Lw);
    return mask_bit(freeM, lane_id()) ? M.y : 0.f;
}

// forward / backward passes and the joint-space matrix: fills Mm (reversed
// dof order k' = nv - 1 - k, k = 6 + i for body i, k = e for base component
// e), the body records (R, p, Rw, pw, depth) and gen[k'] = the generalized
// force without the inertial part: tau - d qd - h (joints), -h (base)
template <int MAXN>
__device__ __forceinline__ void wave_crba_tree(const ChainF* __restrict__ P, const FloatF* __restrict__ F, int N,
                                               const M3& R0, const f3& p0, const SV& V0, WaveWorld<MAXN>& L,
                                               float* __restrict__ Mm, float* __restrict__ gen, bool ext) {
    const int lane = lane_id();
    const bool own = lane < N;
    const int i = own ? lane : 0;
    const BodyF b = P->b[i];
    const int pa = b.parent;
    const int depth = own ? F->body_depth[i] : -1;
    const int srank = F->body_srank[i];
    const int levels = F->levels, fanout = F->fanout;
    const int NV = 6 + N;
    const f3 gw = mk(F->g[0], F->g[1], F->g[2]);
    const int slot = (pa >= 0) ? pa : MAXN;
    static_assert(sizeof(CrbaAcc) <= sizeof(WaveAcc), "composite accumulator in the wave slot");
    if (lane <= MAXN) reinterpret_cast<CrbaAcc*>(&L.acc[0])[lane] = CrbaAcc{};
    // ---- forward: kinematics, velocities, RNEA accelerations (qdd = 0)
    M3 R, Rw;
    f3 p, pw;
    SV V, A, Bf;
    for (int d = 0; d < levels; ++d) {
        if (depth == d) {
            joint_pose_tree(b, L.q, i, R, p);
            const SV Sq = motion(b, L.qd[i]);
            const SV Vp = (pa >= 0) ? L.body[pa].V : V0;
            const SV Ap = (pa >= 0) ? L.body[pa].U : SV{{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
            const M3 Rwp = (pa >= 0) ? L.body[pa].Rw : R0;
            const f3 pwp = (pa >= 0) ? L.body[pa].pw : p0;
            V = ad_inv(R, p, Vp) + Sq;
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int c = 0; c < 3; ++c)
                    Rw.m[r * 3 + c] =
                        Rwp.m[r * 3] * R.m[c] + Rwp.m[r * 3 + 1] * R.m[3 + c] + Rwp.m[r * 3 + 2] * R.m[6 + c];
            pw = pwp + mul(Rwp, p);
            const SV Ve = ball_bias_velocity(b, L.qd, i, V);
            const SV eta = {cross(Ve.w, Sq.w), cross(Ve.w, Sq.v) + cross(Ve.v, Sq.w)};
            A = ad_inv(R, p, Ap) + eta;
            Bf = rigid_bias(b.mass, mk(b.com[0], b.com[1], b.com[2]), inertia_origin(b, b.mass), V, mulT(Rw, gw));
            L.body[i].V = V;
            L.body[i].U = A;  // the RNEA acceleration rides in the U slot (no ABA here)
            L.body[i].Rw = Rw;
            L.body[i].pw = pw;
            // the joint transform: the CRBA climbs below and the J rows read it
            L.body[i].R = R;
            L.body[i].p = p;
            L.body[i].depth = depth;
        }
    }
    // own bias force f_i = I_i a_i + B_i (- the world wrench, body frame)
    SV fb = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
    if (own) {
        fb = mul(rigid(b, b.mass), A) + Bf;
        if (ext) {
            const float* e = L.ext[1 + i];
            fb = fb + (-1.f) * SV{mulT(Rw, mk(e[3], e[4], e[5])), mulT(Rw, mk(e[0], e[1], e[2]))};
        }
    }
    // ---- backward: composite inertias and bias forces, deepest level first
    CrbaAcc* acc = reinterpret_cast<CrbaAcc*>(&L.acc[0]);  // 16 of the slot's 48 words
    for (int d = levels - 1; d >= 0; --d) {
        const bool mine = (depth == d);
        Rigid10 c, Ic;
        SV cb, fc;
        if (mine) {
            Ic = rigid10(b) + acc[i].I;
            fc = fb + acc[i].B;
            c = to_parent10(R, p, Ic);
            cb = dad_inv(R, p, fc);
        }
        for (int k = 0; k < fanout; ++k) {
            if (mine && srank == k) {
                CrbaAcc& a = acc[slot];
                a.I = a.I + c;
                a.B = a.B + cb;
            }
        }
        if (mine) {
            // the body's own composite replaces its children's sum (nobody
            // reads the sum again)
            acc[i].I = Ic;
            acc[i].B = fc;
        }
    }
    wave_lds_sync();
    // ---- the joint-space matrix, reversed order (zero first)
    const int nz = NV * kCrbaMStride;
    for (int e = lane; e < nz; e += kWaveLanes) Mm[e] = 0.f;
    wave_lds_sync();
    if (own) {
        const SI Ic = si_of(acc[i].I);
        SV Fv = ais(Ic, b);
        const int kk = N - 1 - i;
        Mm[kk * kCrbaMStride + kk] = proj(b, Fv);
        gen[kk] = L.tau[i] - b.damping * L.qd[i] - proj(b, acc[i].B);
        Fv = dad_inv(R, p, Fv);
        const uint64_t path = F->body_path[i] & ~(uint64_t{1} << i);
        for (uint64_t m = path; m != 0;) {
            const int j = 63 - __builtin_clzll(m);
            m &= ~(uint64_t{1} << j);
            const float mji = proj(P->b[j], Fv);
            const int kj = N - 1 - j;
            Mm[kj * kCrbaMStride + kk] = mji;
            Mm[kk * kCrbaMStride + kj] = mji;
            Fv = dad_inv(L.body[j].R, L.body[j].p, Fv);
        }
        const float fe[6] = {Fv.w.x, Fv.w.y, Fv.w.z, Fv.v.x, Fv.v.y, Fv.v.z};
#pragma unroll
        for (int e = 0; e < 6; ++e) {
            const int ke = NV - 1 - e;
            Mm[ke * kCrbaMStride + kk] = fe[e];
            Mm[kk * kCrbaMStride + ke] = fe[e];
        }
    }
    // the base: its composite inertia (6 x 6) and bias
    {
        const Rigid10 base10 = {F->mass, mk(F->mass * F->com[0], F->mass * F->com[1], F->mass * F->com[2]),
                                Sy{F->Io[0], F->Io[1], F->Io[2], F->Io[3], F->Io[4], F->Io[5]}};
        const SI Ic0 = si_of(base10 + acc[MAXN].I);
        SV fc0 = rigid_bias(F->mass, mk(F->com[0], F->com[1], F->com[2]),
                            Sy{F->Io[0], F->Io[1], F->Io[2], F->Io[3], F->Io[4], F->Io[5]}, V0, mulT(R0, gw)) +
                 acc[MAXN].B;
        if (ext) {
            const float* e = L.ext[0];
            fc0 = fc0 + (-1.f) * SV{mulT(R0, mk(e[3], e[4], e[5])), mulT(R0, mk(e[0], e[1], e[2]))};
        }
        if (lane < 6) {
            // row e of Ic0: [A B; B^T C]
            const float A9[9] = {Ic0.A.xx, Ic0.A.xy, Ic0.A.xz, Ic0.A.xy, Ic0.A.yy, Ic0.A.yz,
                                 Ic0.A.xz, Ic0.A.yz, Ic0.A.zz};
            const float C9[9] = {Ic0.C.xx, Ic0.C.xy, Ic0.C.xz, Ic0.C.xy, Ic0.C.yy, Ic0.C.yz,
                                 Ic0.C.xz, Ic0.C.yz, Ic0.C.zz};
            const float f6[6] = {fc0.w.x, fc0.w.y, fc0.w.z, fc0.v.x, fc0.v.y, fc0.v.z};
            const int e = lane;
            const int ke = NV - 1 - e;
            float fe = 0.f;
#pragma unroll
            for (int r = 0; r < 6; ++r) fe = (r == e) ? f6[r] : fe;
            gen[ke] = -fe;
#pragma unroll
            for (int f = 0; f < 6; ++f) {
                float v = 0.f;
#pragma unroll
                for (int r = 0; r < 3; ++r)
#pragma unroll
                    for (int cc = 0; cc < 3; ++cc) {
                        if (r == e && cc == f) v = A9[r * 3 + cc];
                        if (r == e && cc + 3 == f) v = Ic0.B.m[r * 3 + cc];
                        if (r + 3 == e && cc == f) v = Ic0.B.m[cc * 3 + r];
                        if (r + 3 == e && cc + 3 == f) v = C9[r * 3 + cc];
                    }
                Mm[ke * kCrbaMStride + (NV - 1 - f)] = v;
            }
        }
    }
    wave_lds_sync();
}

// Y = D^-1/2 L^-1 J^T for this lane's row (Y[k] = J[k] in, reversed order),
// L from Lw (stride LS), pairs of freeM
template <int NVP, int LS, int J>
__device__ __forceinline__ void crba_trsm(float (&Y)[NVP], uint64_t freeM, const float* __restrict__ Lw) {
    if (((freeM >> J) & 3ull) != 0ull) {
        const float z0 = Y[J];
        Y[J + 1] = fmaf(-Lw[J * LS + J + 1], z0, Y[J + 1]);
        const float z1 = Y[J + 1];
#pragma unroll
        for (int k = J + 2; k < NVP; ++k) Y[k] = fmaf(-Lw[J * LS + k], z0, fmaf(-Lw[(J + 1) * LS + k], z1, Y[k]));
    }
    if constexpr (J + 2 < NVP) crba_trsm<NVP, LS, J + 2>(Y, freeM, Lw);
}

// One engine step in joint space (header); the interface and the phases
// after the tree are wave_step's.
template <int MAXN, bool CONS>
__device__ __forceinline__ uint32_t wave_step_crba(const ChainF* __restrict__ P, const FloatF* __restrict__ F, int N,
                                                   FreeState& base, WaveWorld<MAXN>& L, float dt, int pgs_iters,
                                                   float pgs_tol, bool warm, int lcp_solves, float* qdd_out,
                                                   int* overflow, int* unconverged, unsigned long long* prof, bool ext) {
    using Dm = CrbaDims<MAXN>;
    constexpr int NVP = Dm::kNvp, LS = Dm::kLs;
    const int lane = lane_id();
    const int NV = 6 + N;
    MW_PROF_T(t0);
    const M3 R0 = quat_to_R(base.qw, base.qx, base.qy, base.qz);
    float* Mm = &L.stack[0][0][0];
    float* Lw = &L.MJ[0][0];
    static_assert(sizeof(L.stack) >= 64 * kCrbaMStride * sizeof(float), "M in the stack region");
    wave_crba_tree<MAXN>(P, F, N, R0, base.p, base.V, L, Mm, L.gen, ext);
    MW_PROF_T(t0b);
    MW_PROF_ACC(18, t0, t0b);
    const uint64_t allM = (1ull << NV) - 1ull;  // NV <= 54
    const uint64_t freeM = F->fixed ? ((1ull << N) - 1ull) : allM;
    const bool dual = F->dual != 0;
    // DART's implicit damping on the joint dofs (reversed: lane c is body N - 1 - c)
    float dd0 = 0.f, dd1 = 0.f;
    {
        const int b0 = N - 1 - (lane & 31), b1 = N - 33 - (lane & 31);
        if (b0 >= 0) dd0 = dt * P->b[b0].damping;
        if (b1 >= 0) dd1 = dt * P->b[b1].damping;
    }
    if (lane < 64) L.dsq[lane] = 0.f;
    const float rhs = (lane < NV) ? L.gen[lane] : 0.f;
    float y;
    if constexpr (Dm::kNv <= 32) {
        y = crba_ldl<32, LS, NVP>(Mm, freeM, dd0, dd1, rhs, Lw, dual ? nullptr : L.dsq);
        if (dual) (void)crba_ldl<32, LS, NVP>(Mm, freeM, 0.f, 0.f, 0.f, Lw, L.dsq);
    } else {
        if (NV <= 32) {
            y = crba_ldl<32, LS, NVP>(Mm, freeM, dd0, dd1, rhs, Lw, dual ? nullptr : L.dsq);
            if (dual) (void)crba_ldl<32, LS, NVP>(Mm, freeM, 0.f, 0.f, 0.f, Lw, L.dsq);
        } else {
            y = crba_ldl<64, LS, NVP>(Mm, freeM, dd0, dd1, rhs, Lw, dual ? nullptr : L.dsq);
            if (dual) (void)crba_ldl<64, LS, NVP>(Mm, freeM, 0.f, 0.f, 0.f, Lw, L.dsq);
        }
    }
    // accelerations: lane k' holds joint N - 1 - k' (k' < N) or base component NV - 1 - k'
    if (lane < N) qdd_out[N - 1 - lane] = y;
    float a0v[6];
#pragma unroll
    for (int e = 0; e < 6; ++e) a0v[e] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, y), NV - 1 - e));
    wave_lds_sync();
    MW_PROF_T(t1);
    MW_PROF_ACC(1, t0, t1);
    MW_PROF_ACC(19, t0b, t1);
    // integrateVelocities (lane e: nu component e)
    if (lane < NV) {
        float v;
        if (lane < 6) {
            const float V0[6] = {base.V.w.x, base.V.w.y, base.V.w.z, base.V.v.x, base.V.v.y, base.V.v.z};
            float ae = 0.f, ve = 0.f;
#pragma unroll
            for (int e = 0; e < 6; ++e) {
                ae = (lane == e) ? a0v[e] : ae;
                ve = (lane == e) ? V0[e] : ve;
            }
            v = F->fixed ? 0.f : ve + dt * ae;
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
    const int my_j = __builtin_popcount(jbits);
    int before = 0, total_j = 0;
    for (int d = 0; d < N; ++d) {
        const int cnt = __builtin_amdgcn_readlane(my_j, d);
        before += (d < lane) ? cnt : 0;
        total_j += cnt;
    }
    int R = n_contact_rows + total_j;
    if (R > kWaveMaxRows) {
        if (lane == 0) *overflow += R - kWaveMaxRows;
        R = kWaveMaxRows;
    }
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
    wave_lds_sync();

    MW_PROF_T(t2);
    MW_PROF_ACC(2, t1, t2);
    if (R > 0) {
        // ---- J rows (lane = row), reversed dof order, to L.J -----------------
        if (lane < R) {
            float* Jr = L.J[lane];
#pragma unroll
            for (int e = 0; e < WaveWorld<MAXN>::kJStride; ++e) Jr[e] = 0.f;
            const int src = L.src[lane];
            if (src < kJointRow) {
                const int slot = src / 3, d = src % 3;
                int sh = 0;
                while (sh + 1 < F->n_shapes && F->shape_slot0[sh + 1] <= slot) ++sh;
                const int k = F->shape_body[sh];
                const f3 bpt = {L.s_b[slot][0], L.s_b[slot][1], L.s_b[slot][2]};
                // body-frame direction R_k^T d: n -> row 2, t1 -> -row 1, t2 -> row 0
                const int row = (d == 0) ? 2 : ((d == 1) ? 1 : 0);
                const float sg = (d == 1) ? -1.f : 1.f;
                const f3 dir = {sg * L.s_R[slot][row * 3], sg * L.s_R[slot][row * 3 + 1],
                                sg * L.s_R[slot][row * 3 + 2]};
                SV Fi = {cross(bpt, dir), dir};
                float jv = 0.f;
                const uint64_t path = (k >= 0) ? F->body_path[k] : uint64_t{0};
                for (uint64_t m = path; m != 0;) {
                    const int i = 63 - __builtin_clzll(m);
                    m &= ~(uint64_t{1} << i);
                    const float ji = proj(P->b[i], Fi);
                    Jr[N - 1 - i] = ji;
                    jv += ji * L.nu[6 + i];
                    Fi = dad_inv(L.body[i].R, L.body[i].p, Fi);
                }
                if (!F->fixed) {
                    const float fe[6] = {Fi.w.x, Fi.w.y, Fi.w.z, Fi.v.x, Fi.v.y, Fi.v.z};
#pragma unroll
                    for (int e = 0; e < 6; ++e) {
                        Jr[NV - 1 - e] = fe[e];
                        jv += fe[e] * L.nu[e];
                    }
                }
                const float bounce = (d == 0) ? fminf(kContactErp * L.s_depth[slot] * rcp(dt), kContactMaxErv) : 0.f;
                L.b[lane] = bounce - jv;
            } else {
                const int j = (src - kJointRow) / 3;
                Jr[N - 1 - j] = 1.f;
            }
        }
        // ---- Y = D^-1/2 L^-1 J^T (lane = row) --------------------------------
        float Y[NVP];
#pragma unroll
        for (int k = 0; k < NVP; ++k) Y[k] = (lane < R) ? L.J[lane][k] : 0.f;
        crba_trsm<NVP, LS, 0>(Y, freeM, Lw);
        if (lane < R) {
#pragma unroll
            for (int k = 0; k < NVP; ++k) L.J[lane][k] = Y[k] * L.dsq[k];
        }
        wave_lds_sync();
        MW_PROF_T(t3);
        MW_PROF_ACC(3, t2, t3);
        // ---- Delassus A = Y Y^T on the matrix cores (wave_step's tile layout)
        const int ncr = (n_contact_rows < R) ? n_contact_rows : R;
        const int lr = lane & 31, lh = lane >> 5;
        const bool two = R > 32;
        v16f t00 = {}, t01 = {}, t10 = {}, t11 = {};
#pragma unroll
        for (int k = 0; k < NVP / 2; ++k) {
            const int e = 2 * k + lh;
            const float y0 = L.J[lr][e];
            t00 = __builtin_amdgcn_mfma_f32_32x32x2f32(y0, y0, t00, 0, 0, 0);
            if (two) {
                const float y1 = L.J[32 + lr][e];
                t01 = __builtin_amdgcn_mfma_f32_32x32x2f32(y0, y1, t01, 0, 0, 0);
                t10 = __builtin_amdgcn_mfma_f32_32x32x2f32(y1, y0, t10, 0, 0, 0);
                t11 = __builtin_amdgcn_mfma_f32_32x32x2f32(y1, y1, t11, 0, 0, 0);
            }
        }
        float a[kWaveMaxRows];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int r0 = 8 * (i / 4) + (i % 4);
            const float g0 = __shfl_xor(lh ? t00[i] : t01[i], 32);
            a[r0] = lh ? g0 : t00[i];
            a[r0 + 4] = lh ? t01[i] : g0;
            const float g1 = __shfl_xor(lh ? t10[i] : t11[i], 32);
            a[32 + r0] = lh ? g1 : t10[i];
            a[32 + r0 + 4] = lh ? t11[i] : g1;
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
        float x0 = 0.f, x1w = 0.f;
        const int wid = (lane < R) ? ((L.src[lane] < kJointRow) ? L.src[lane]
                                                                 : kWaveWarmJoint0 + (L.src[lane] - kJointRow))
                                   : 0;
        if (warm && lane < R) {
            x0 = L.xw[wid];
            x1w = L.xw[kWaveWarmWords + wid];
        }
        float x1s = 0.f;
        if (lcp_solves > 0) {
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
            // the LCP's workspace: the stack region (M is dead once factored)
            float* U = &L.stack[0][0][0];
            int nsolve = 0, nround = 0, nsolve1 = 0;
            long long cyc[3] = {0, 0, 0};
            constexpr int kWaveLcpMfma = (!MW_LCP_MFMA || MAXN <= 16) ? kLcpMfmaNone : kLcpMfma32;
            bool ok;
            if (R <= 16)
                ok = wave_lcp_exact<16, false, kLcpStageSweeps, kWaveLcpMfma>(a, Rw, mu, R, lcp_solves, pgs_iters,
                                                                             pgs_tol, L.rc, U, x1s, xe, nsolve,
                                                                             nround, nsolve1, cyc);
            else if (R <= 32)
                ok = wave_lcp_exact<32, false, kLcpStageSweeps, kWaveLcpMfma>(a, Rw, mu, R, lcp_solves, pgs_iters,
                                                                             pgs_tol, L.rc, U, x1s, xe, nsolve,
                                                                             nround, nsolve1, cyc);
            else
                ok = wave_lcp_exact<kWaveMaxRows, false, kLcpStageSweeps, kWaveLcpMfma>(
                    a, Rw, mu, R, lcp_solves, pgs_iters, pgs_tol, L.rc, U, x1s, xe, nsolve, nround, nsolve1, cyc);
#ifdef MW_WAVE_PROF
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
            if (!ok && lane == 0) *unconverged += 1;
        } else {
#pragma unroll
            for (int r = 0; r < kWaveMaxRows; ++r) x[r] = warm ? read_lane(x0, r) : 0.f;
            if (pgs_tol > 0.f)
                wave_pgs<MAXN, true>(L, a, x, Rpad, ncr, mu, pgs_iters, pgs_tol);
            else
                wave_pgs<MAXN, false>(L, a, x, Rpad, ncr, mu, pgs_iters, 0.f);
        }
        MW_PROF_T(t5);
        MW_PROF_ACC(5, t4, t5);
        // ---- dnu = M^-1 J^T x = L^-T D^-1/2 (Y^T x), lane = dof (reversed) ----
        float xl = 0.f, u = 0.f;
#pragma unroll
        for (int rb = 0; rb < kWaveMaxRows; rb += 8) {
            if (rb >= Rpad) break;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int r = rb + k;
                xl = (lane == r) ? x[r] : xl;
                if (r < R && lane < NVP) u += x[r] * L.J[r][lane];
            }
        }
        u *= (lane < NVP) ? L.dsq[lane] : 0.f;
        if constexpr (Dm::kNv <= 32) {
            ldl_backward<30, LS>(u, freeM, Lw);
        } else {
            if (NV <= 32) ldl_backward<30, LS>(u, freeM, Lw);
            else ldl_backward<62, LS>(u, freeM, Lw);
        }
        const float dnu = mask_bit(freeM, lane) ? u : 0.f;
        if (lane < R) {
            const int src = L.src[lane];
            if (src < kJointRow) L.s_x[src / 3][src % 3] = xl;
        }
        wave_lds_sync();
        if (lane < NV) L.nu[NV - 1 - lane] += dnu;
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
    wave_lds_sync();

    // ---- integratePositions ---------------------------------------------------
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

}  // namespace dev
}  // namespace mw
