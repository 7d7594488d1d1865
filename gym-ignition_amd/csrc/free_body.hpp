// free_body.hpp -- one engine step of a floating rigid body with ground-plane
// contacts, float32, one world per lane.  Restates, like oracle.c
// or_free_step (fp64), DART 6.x as driven by the reference's Physics system
// [EXT]:
//
//   FreeJoint forward dynamics   I a = -(V x* I V) + I [0; g_b]   (body frame)
//   integrateVelocities          V += dt a
//   ContactConstraint rows       per contact point: normal (x_n >= 0, error
//                                reduction 0.01 capped at 1e-3 m/s) and two
//                                ODE plane-space tangents (|x_t| <= mu x_n),
//                                CFM 1e-5, projected Gauss-Seidel
//   integratePositions           T <- T exp(dt V)   (DART FreeJoint, SE(3) exp)
//
// Layout for CDNA4: the contact points live in fixed slots (8 corners per
// box, slot 0 of a sphere) with an active bitmask, so every per-slot array is
// indexed by an unrolled constant -- no compaction, no dynamically indexed
// private arrays.  The PGS runs in "sequential impulse" form on the 6-vector
// body twist: a row needs J = [b x d; d] (recomputed) and M^-1 J (the inverse
// spatial inertia is a per-model constant, precomputed on the host), never
// the Delassus matrix.
#pragma once

#include "chain_dyn.hpp"

namespace mw {

constexpr int kMaxFreeShapes = 2;
constexpr int kMaxFreeSlots = 8 * kMaxFreeShapes;

struct FreeF {
    float mass;
    float com[3];
    float Io[6];          // rotational inertia about the body origin: xx yy zz xy xz yz
    float Minv[36];       // inverse spatial inertia [angular; linear], row-major
    float g[3];           // world gravity
    float mu;             // Coulomb friction with the ground
    int32_t n_shapes;
    int32_t ground;       // ground plane z = 0 present
    int32_t shape_type[kMaxFreeShapes];  // 0 box, 1 sphere, 2 cylinder, 3 mesh points
    float shape_size[kMaxFreeShapes][3]; // box half extents / sphere radius
    float shape_R[kMaxFreeShapes][9];
    float shape_p[kMaxFreeShapes][3];
    int32_t mesh_npts[kMaxFreeShapes];   // type 3: support points (<= 8, one per slot)
    float mesh_pt[kMaxFreeShapes][8][3]; // in the shape frame
};

namespace dev {

// DART ContactConstraint defaults [EXT]
constexpr float kContactErp = 0.01f;
constexpr float kContactMaxErv = 1e-3f;
constexpr float kContactCfm = 1e-5f;

struct FreeState {
    f3 p;          // body origin, world
    float qw, qx, qy, qz;  // orientation (unit quaternion)
    SV V;          // twist, body frame [w; v]
};

__device__ __forceinline__ M3 quat_to_R(float w, float x, float y, float z) {
    M3 R;
    R.m[0] = 1.f - 2.f * (y * y + z * z); R.m[1] = 2.f * (x * y - w * z);       R.m[2] = 2.f * (x * z + w * y);
    R.m[3] = 2.f * (x * y + w * z);       R.m[4] = 1.f - 2.f * (x * x + z * z); R.m[5] = 2.f * (y * z - w * x);
    R.m[6] = 2.f * (x * z - w * y);       R.m[7] = 2.f * (y * z + w * x);       R.m[8] = 1.f - 2.f * (x * x + y * y);
    return R;
}

// DART FreeJoint::integratePositions: T <- T exp(dt V) (SE(3) exponential,
// V = [w; v] in the body frame); R is the rotation of S's quaternion.
__device__ __forceinline__ void integrate_pose(const M3& R, const SV& V, float dt, FreeState& S) {
    const f3 phi = dt * V.w, u = dt * V.v;
    const float th2 = dot(phi, phi);
    float b, cc;  // V(phi) = 1 + b K + cc K^2
    if (th2 < 1e-8f) {
        b = 0.5f - th2 * (1.f / 24.f);
        cc = (1.f / 6.f) - th2 * (1.f / 120.f);
    } else {
        const float th = sqrtf(th2);
        float sn, cs;
        sincos_joint(th, &sn, &cs);
        b = (1.f - cs) / th2;
        cc = (th - sn) / (th2 * th);
    }
    const f3 Ku = cross(phi, u);
    const f3 dp = u + b * Ku + cc * cross(phi, Ku);
    S.p = S.p + mul(R, dp);
    // q <- q (x) [cos(th/2), sin(th/2) phi/th]
    float hs, hc;
    const float th = sqrtf(th2);
    sincos_joint(0.5f * th, &hs, &hc);
    const float k = (th2 < 1e-12f) ? 0.5f : hs / th;
    const float dw = hc, dx = k * phi.x, dy = k * phi.y, dz = k * phi.z;
    const float nw = S.qw * dw - S.qx * dx - S.qy * dy - S.qz * dz;
    const float nx = S.qw * dx + S.qx * dw + S.qy * dz - S.qz * dy;
    const float ny = S.qw * dy - S.qx * dz + S.qy * dw + S.qz * dx;
    const float nz = S.qw * dz + S.qx * dy - S.qy * dx + S.qz * dw;
    const float inv = 1.f / sqrtf(nw * nw + nx * nx + ny * ny + nz * nz);
    S.qw = nw * inv; S.qx = nx * inv; S.qy = ny * inv; S.qz = nz * inv;
}

__device__ __forceinline__ SV minv_mul(const FreeF& __restrict__ F, const SV& x) {
    const float in[6] = {x.w.x, x.w.y, x.w.z, x.v.x, x.v.y, x.v.z};
    float o[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < 6; ++k) acc += F.Minv[r * 6 + k] * in[k];
        o[r] = acc;
    }
    return {{o[0], o[1], o[2]}, {o[3], o[4], o[5]}};
}

// body-frame point of slot k of shape s (box corner k; sphere: centre;
// cylinder: rim point k, chain_dyn.hpp shape_slot_point) for body rotation Rb
template <bool MESH>
__device__ __forceinline__ f3 slot_point(const FreeF& F, int s, int k, const M3& Rb) {
    const float* R = F.shape_R[s];
    const f3 l = (MESH && F.shape_type[s] == 3)
                     ? mk(F.mesh_pt[s][k][0], F.mesh_pt[s][k][1], F.mesh_pt[s][k][2])
                     : shape_slot_point(F.shape_type[s], F.shape_size[s], shape_plane_normal(Rb, R), k);
    return {F.shape_p[s][0] + R[0] * l.x + R[1] * l.y + R[2] * l.z,
            F.shape_p[s][1] + R[3] * l.x + R[4] * l.y + R[5] * l.z,
            F.shape_p[s][2] + R[6] * l.x + R[7] * l.y + R[8] * l.z};
}

// Contact slot record in LDS (31 words: odd, so a wave's accesses to one
// field hit distinct banks); slot records of a lane are kFreeLanes apart.
// Per row the step caches M^-1 J and the diagonal, so a PGS sweep is two
// 6-dots and a 6-axpy per row.
constexpr int kFreeLanes = 64;
struct SlotRec {
    f3 b;          // contact point, body frame
    f3 xw;         // contact point, world frame (start of the step)
    float depth;
    float x[3];    // impulses: normal, t1, t2
    float mj[3][6];  // M^-1 J per row
    float arr[3];    // J M^-1 J^T per row (without CFM)
};
static_assert(sizeof(SlotRec) == 31 * 4, "SlotRec layout: an odd word count");

struct Contacts {
    uint32_t active;   // bit per slot
    SlotRec* rec;      // &records[0][lane]
    __device__ __forceinline__ SlotRec& at(int slot) const { return rec[slot * kFreeLanes]; }
};

// One engine step; the contacts of the step stay in C (positions, impulses).
// MESH: some shape entry holds mesh support points (a separate instance, so
// the box / sphere / cylinder bodies keep the unrolled slot loop).
template <bool MESH>
__device__ __forceinline__ void free_step(const FreeF* __restrict__ Fp, float dt, int pgs_iters, FreeState& S,
                                          Contacts& C) {
    const FreeF& F = *Fp;
    const M3 R = quat_to_R(S.qw, S.qx, S.qy, S.qz);
    // forward dynamics: I a = dad(V, I V) + I [0; g_b]
    const f3 gb = mulT(R, mk(F.g[0], F.g[1], F.g[2]));
    const f3 c = {F.com[0], F.com[1], F.com[2]};
    const Sy Io = {F.Io[0], F.Io[1], F.Io[2], F.Io[3], F.Io[4], F.Io[5]};
    const SV& V0 = S.V;
    const f3 hw = mul(Io, V0.w) + F.mass * cross(c, V0.v);
    const f3 hv = F.mass * (V0.v - cross(c, V0.w));
    // dad(V, h) = ad(V)^T h = [hw x w + hv x v; hv x w];  I [0; g] = [m c x g; m g]
    const SV f = {cross(hw, V0.w) + cross(hv, V0.v) + F.mass * cross(c, gb), cross(hv, V0.w) + F.mass * gb};
    const SV a = minv_mul(F, f);
    SV V = V0 + dt * a;

    // contacts at the positions of the start of the step
    C.active = 0u;
    if (F.ground) {
#pragma unroll
        for (int s = 0; s < kMaxFreeShapes; ++s) {
            if (s >= F.n_shapes) break;
            const bool sphere = (F.shape_type[s] == 1);
            const int nk = sphere ? 1 : (MESH && F.shape_type[s] == 3) ? F.mesh_npts[s] : 8;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if (k >= nk) break;
                f3 b = slot_point<MESH>(F, s, k, R);
                f3 xw = S.p + mul(R, b);
                float depth = -xw.z;
                if (sphere) {  // its lowest point
                    const float r = F.shape_size[s][0];
                    depth = r - xw.z;
                    xw.z -= r;
                    b = mulT(R, xw - S.p);
                }
                if (depth > 0.f) {
                    const int slot = 8 * s + k;
                    C.active |= 1u << slot;
                    SlotRec& r = C.at(slot);
                    r.b = b;
                    r.xw = xw;
                    r.depth = depth;
                    r.x[0] = r.x[1] = r.x[2] = 0.f;
                }
            }
        }
    }

    if (C.active) {
        // directions in the body frame: n = +z, t1, t2 = ODE dPlaneSpace(n)
        const f3 db[3] = {mulT(R, mk(0.f, 0.f, 1.f)), mulT(R, mk(0.f, -1.f, 0.f)), mulT(R, mk(1.f, 0.f, 0.f))};
        const float inv_dt = rcp(dt);
        // rows of this step: M^-1 J and the diagonal, once
        for (uint32_t m = C.active; m; m &= m - 1u) {
            SlotRec& r = C.at(__builtin_ctz(m));
            const f3 b = r.b;
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                const SV J = {cross(b, db[d]), db[d]};
                const SV MJ = minv_mul(F, J);
                r.mj[d][0] = MJ.w.x; r.mj[d][1] = MJ.w.y; r.mj[d][2] = MJ.w.z;
                r.mj[d][3] = MJ.v.x; r.mj[d][4] = MJ.v.y; r.mj[d][5] = MJ.v.z;
                r.arr[d] = dot(J, MJ);
            }
        }
        for (int it = 0; it < pgs_iters; ++it) {
            for (uint32_t m = C.active; m; m &= m - 1u) {
                SlotRec& r = C.at(__builtin_ctz(m));
                const f3 b = r.b;
                const float bounce = fminf(kContactErp * r.depth * inv_dt, kContactMaxErv);
                float xs[3] = {r.x[0], r.x[1], r.x[2]};
#pragma unroll
                for (int d = 0; d < 3; ++d) {
                    const SV J = {cross(b, db[d]), db[d]};
                    const SV MJ = {{r.mj[d][0], r.mj[d][1], r.mj[d][2]}, {r.mj[d][3], r.mj[d][4], r.mj[d][5]}};
                    const float Arr = r.arr[d];
                    // x += (b - sum_c A_rc x_c) / A_rr  with  sum_c A_rc x_c = J (V - V1) + cfm A_rr x
                    const float target = (d == 0) ? bounce : 0.f;
                    const float xo = xs[d];
                    float xn = xo + (target - dot(J, V) - kContactCfm * Arr * xo) * rcp(Arr * (1.f + kContactCfm));
                    if (d == 0) {
                        xn = fmaxf(xn, 0.f);
                    } else {
                        const float hi = F.mu * xs[0];
                        xn = fminf(fmaxf(xn, -hi), hi);
                    }
                    V = V + (xn - xo) * MJ;
                    xs[d] = xn;
                }
                r.x[0] = xs[0]; r.x[1] = xs[1]; r.x[2] = xs[2];
            }
        }
    }

    // integratePositions: T <- T exp(dt V)
    integrate_pose(R, V, dt, S);
    S.V = V;
}

}  // namespace dev
}  // namespace mw
