// scene_kernel.hip -- one engine step of a SCENE (several models in one world:
// World::insertModel, cpp/scenario/gazebo/src/World.cpp:394-420), ONE WORLD
// PER WAVEFRONT.  Same physics as oracle.c or_scene_step (DART 6 World::step
// restated [EXT]: ABA with implicit damping, v-integration, one boxed LCP over
// every contact and joint row, impulse velocities, p-integration), the
// mapping of wave_tree.hpp generalised from one floating tree to a forest:
//
//   nodes            lane = node: the model bases (fixed or floating) and
//                    every body; the level-parallel ABA walks the forest by
//                    depth (bases are level 0), child -> parent sums through
//                    per-node LDS accumulators one sibling rank at a time
//                    (deterministic); a floating base solves its 6x6
//                    articulated inertia on its own lane (Cholesky, kept in
//                    LDS for the impulse responses); a welded base does not
//                    move.
//   wrenches         Link::applyWorldWrench (Link.cpp:484-560) records with an
//                    expiry iteration (Physics.cpp:1446-1525): the active
//                    ones enter the node's bias force, body frame.
//   contacts         lane = ground slot (box corners, sphere bottoms under
//                    z = 0), then lane = shape pair of two models (box-box
//                    SAT + face clipping / edge-edge, box-sphere,
//                    sphere-sphere: the restatement of oracle.c or_collide);
//                    points compacted in (slot, pair, point) order.
//   rows             contact rows (normal + 2 friction directions, ODE
//                    dPlaneSpace) then joint rows (limit / servo / Coulomb);
//                    lane = row responses M^-1 J^T: the two bodies of a
//                    contact each walk their path to their base, floating
//                    bases solve through the stored factor, then the outward
//                    pass over that model's bodies.
//   Delassus / PGS   A = J (M^-1 J^T)^T in LDS (lane = column); projected
//                    Gauss-Seidel in row order (the oracle's), lane c owning
//                    rows c and c + 64: residual w_c, impulse x_c; one row
//                    update = two lane reads, a clamp and one FMA per lane.
#include <hip/hip_runtime.h>

#include "xcd.hpp"
#include "free_body.hpp"
#include "kernels.hpp"
#include "pid.hpp"
#include "scene_params.hpp"
#include "wave_tree.hpp"

namespace mw {
namespace dev {

// per-node record (39 words, odd: lane-strided parent gathers are conflict-free)
struct ScNode {
    M3 R;        // joint transform parent -> node (bases: unused)
    f3 p;
    SV U;        // AI S (impulse inertia)
    float psi;
    float tt;
    SV V;        // velocity, then acceleration
    M3 Rw;       // world pose
    f3 pw;
    int32_t depth;
};
static_assert(sizeof(ScNode) == 39 * 4, "ScNode layout");

// narrow-phase workspace words per lane (ScWorld::clip): two clipping
// polygons of <= 8 vertices x {u, v, x, y, z}, then 8 point slots (a pair's
// output: the first np); columns for 32 lanes, so shape pairs run 32 per pass
// (half the workspace of one column per lane)
constexpr int kScWsPoly = 0, kScWsOut = 80, kScWsWords = 112;
constexpr int kScClipLanes = 32;

template <int MAXNV>
struct ScWorld {
    static constexpr int kStride = MAXNV + 1;     // odd: lane-strided rows are conflict-free
    ScNode node[kScMaxNodes];
    // phase-disjoint storage (one wave runs the phases in program order):
    // the ABA's child -> parent accumulators, the narrow phase's workspace,
    // the response passes' per-lane stacks, then the exact LCP's pivot rows
    // (the Delassus matrix of <= 64 rows sits in registers; more rows take the
    // large-contact path) or that path's LCP scratch -- 21 KiB.  The world's
    // record is 53,024 B (MAXNV 32): three worlds per CU.  At 54,240 B it
    // still ran two (the CU's LDS is handed out in blocks: 3 x 54,240 B did
    // not fit), at 53,024 B three: the three-cube leg 0.739 -> 0.561 ms
    // 
    union {
        WaveAcc acc[kScMaxNodes];
        float clip[kScWsWords][kScClipLanes];        // the narrow phase's per-lane workspace
        float stack[kScMaxDepth][7][kWaveLanes];
        alignas(16) float lcp[kLcpWorkFloats];       // the exact LCP's pivot rows (16-byte reads)
        float big[kScBigRows + 64 * 64];             // the large-contact LCP: vs, T0 (xs in the row arrays)
    };
    float l0[kScMaxModels][28];   // Chol6 (l[21], id[6]) of every floating base
    float q[kScMaxBodies], qd[kScMaxBodies], qdd[kScMaxBodies], tau[kScMaxBodies], vc[kScMaxBodies];
    uint32_t act[kScMaxBodies];
    float nu[MAXNV];
    float J[kScMaxRows][kStride];     // (J then MJ: also the large-contact LCP's T1 tile)
    float MJ[kScMaxRows][kStride];
    F4 rc[kScMaxRows];            // {b, 1/A_rr, lo, hi} (rc .. rhi: also the large-contact LCP's impulses)
    int32_t src[kScMaxRows];      // contact rows 3 c + d; joint rows kJointRow + 3 body + type
    float rb[kScMaxRows], rlo[kScMaxRows], rhi[kScMaxRows];
    float c_p[kScMaxContacts][3], c_n[kScMaxContacts][3];   // (tangents: plane_space_f of the normal where used)
    float c_d[kScMaxContacts];
    int32_t c_na[kScMaxContacts], c_nb[kScMaxContacts];
    int32_t c_key[kScMaxContacts];  // warm-start identity: ground slot, or n_slots + 4 pair + point
    float c_x[kScMaxContacts][3];
};

#ifdef MW_WAVE_PROF
constexpr int kScDumpFloats = 8 + 64 * 64 + 8 * 64;
__device__ float g_sc_dump[kDumpSlots * kScDumpFloats];
__device__ unsigned int g_sc_dump_claim;
#endif

// the world's exact-LCP warm-start record (SceneDev::warm); rec == nullptr: cold
struct ScWarm {
    int32_t* rec;
    int W, w;
    __device__ int32_t& n() const { return rec[w]; }
    __device__ int32_t& key(int c) const { return rec[static_cast<size_t>(1 + c) * W + w]; }
    __device__ float& x(int r) const {
        return reinterpret_cast<float*>(rec)[static_cast<size_t>(1 + kScMaxContacts + r) * W + w];
    }
    // the exact solve's stage-1 impulse of row r
    __device__ float& x1(int r) const {
        return reinterpret_cast<float*>(rec)[static_cast<size_t>(1 + kScMaxContacts + kScWarmRows + r) * W + w];
    }
};

// PGS sweeps of exact mode end once a sweep moves no constraint velocity by
// more than this (sim.cpp kExactPgsTol): the exact solve takes over
constexpr float kScExactPgsTol = 1e-6f;
// PGS sweeps per stage of the exact solve (wave_lcp.hpp STAGE_SWEEPS; the
// wave kernels keep 4)
#ifndef MW_SC_STAGE_SWEEPS
#define MW_SC_STAGE_SWEEPS 6
#endif
constexpr int kScStageSweeps = MW_SC_STAGE_SWEEPS;

// ODE dPlaneSpace (oracle.c plane_space), float32
__device__ __forceinline__ void plane_space_f(f3 n, f3& p, f3& q) {
    if (fabsf(n.z) > 0.70710678f) {
        const float a = n.y * n.y + n.z * n.z, k = rsqrtf(a);
        p = {0.f, -n.z * k, n.y * k};
        q = {a * k, -n.x * p.z, n.x * p.y};
    } else {
        const float a = n.x * n.x + n.y * n.y, k = rsqrtf(a);
        p = {-n.y * k, n.x * k, 0.f};
        q = {-n.z * p.y, n.z * p.x, a * k};
    }
}

__device__ __forceinline__ f3 col(const M3& R, int k) { return {R.m[k], R.m[3 + k], R.m[6 + k]}; }
__device__ __forceinline__ M3 mul3(const M3& A, const M3& B) {
    M3 C;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) C.m[r * 3 + c] = A.m[r * 3] * B.m[c] + A.m[r * 3 + 1] * B.m[3 + c] + A.m[r * 3 + 2] * B.m[6 + c];
    return C;
}

// ---------------------------------------------------------------- narrow phase
// Restatement of oracle.c box_box / box_sphere / or_collide in float32 (same
// axis order, tie rules, clipping order and point reduction).

// Point sets of the narrow phase.  ScWsPts: a lane's column of the contact
// workspace in LDS (ScWorld::clip, slot i = 4 words {x, y, z, depth} at a
// stride of one wavefront) -- the clipping polygons and the kept points of a
// pair live there, not in per-lane arrays indexed at run time (those went to
// scratch: 45.6k of the three-cube scene's 165k cycles per world-step were
// its three box pairs, r06 profile).  ScArrPts: plain arrays (the hull pair's
// own clipping buffer).
struct ScWsPts {
    float* w;
    __device__ __forceinline__ f3 pt(int i) const {
        return {w[(4 * i) * kScClipLanes], w[(4 * i + 1) * kScClipLanes], w[(4 * i + 2) * kScClipLanes]};
    }
    __device__ __forceinline__ float dep(int i) const { return w[(4 * i + 3) * kScClipLanes]; }
    __device__ __forceinline__ void set(int i, f3 x, float d) const {
        w[(4 * i) * kScClipLanes] = x.x;
        w[(4 * i + 1) * kScClipLanes] = x.y;
        w[(4 * i + 2) * kScClipLanes] = x.z;
        w[(4 * i + 3) * kScClipLanes] = d;
    }
    __device__ __forceinline__ void move(int m, int i) const { set(m, pt(i), dep(i)); }
};
struct ScArrPts {
    f3* p;
    float* d;
    __device__ __forceinline__ f3 pt(int i) const { return p[i]; }
    __device__ __forceinline__ float dep(int i) const { return d[i]; }
    __device__ __forceinline__ void move(int m, int i) const { p[m] = p[i]; d[m] = d[i]; }
};

// the oracle's reduction to 4 points (deepest, farthest, largest triangle,
// farthest from its centroid), compacted in place in the original order
template <class S>
__device__ __forceinline__ int sc_reduce(int n, const S& s) {
    if (n <= 4) return n;
    int a = 0;
    for (int i = 1; i < n; ++i) if (s.dep(i) > s.dep(a)) a = i;
    const f3 pa = s.pt(a);
    uint32_t used = 1u << a;
    int b = -1;
    float best = -1.f;
    for (int i = 0; i < n; ++i) {
        if ((used >> i) & 1u) continue;
        const f3 e = s.pt(i) - pa;
        const float v = dot(e, e);
        if (v > best) { best = v; b = i; }
    }
    used |= 1u << b;
    int c = -1;
    best = -1.f;
    const f3 pb = s.pt(b);
    const f3 ab = pb - pa;
    for (int i = 0; i < n; ++i) {
        if ((used >> i) & 1u) continue;
        const f3 x = cross(ab, s.pt(i) - pa);
        const float v = dot(x, x);
        if (v > best) { best = v; c = i; }
    }
    used |= 1u << c;
    const f3 g = (1.f / 3.f) * (pa + pb + s.pt(c));
    int e4 = -1;
    best = -1.f;
    for (int i = 0; i < n; ++i) {
        if ((used >> i) & 1u) continue;
        const f3 e = s.pt(i) - g;
        const float v = dot(e, e);
        if (v > best) { best = v; e4 = i; }
    }
    used |= 1u << e4;
    int m = 0;
    for (int i = 0; i < n; ++i)
        if ((used >> i) & 1u) { s.move(m, i); ++m; }
    return 4;
}

__device__ __forceinline__ f3 sel3(f3 x0, f3 x1, f3 x2, int k) { return k == 0 ? x0 : (k == 1 ? x1 : x2); }
__device__ __forceinline__ float self3(float x0, float x1, float x2, int k) { return k == 0 ? x0 : (k == 1 ? x1 : x2); }

// (the axis / half-extent triples are selected, never indexed at run time:
// a run-time index into a local array puts the array in scratch)
__device__ __forceinline__ int sc_box_box(f3 hA, f3 cA, const M3& RA, f3 hB, f3 cB, const M3& RB, f3& n,
                                          const ScWsPts& out, float* ws) {
    const f3 a[3] = {col(RA, 0), col(RA, 1), col(RA, 2)};
    const f3 b[3] = {col(RB, 0), col(RB, 1), col(RB, 2)};
    const float ha[3] = {hA.x, hA.y, hA.z}, hb[3] = {hB.x, hB.y, hB.z};
    const f3 T = cB - cA;
    float best_face = 3.0e38f, best_edge = 3.0e38f;
    int face = -1, ei = -1, ej = -1;
    f3 eaxis = {0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const f3 L = k < 3 ? a[k] : b[k - 3];
        float rA = 0.f, rB = 0.f;
#pragma unroll
        for (int i = 0; i < 3; ++i) { rA += ha[i] * fabsf(dot(a[i], L)); rB += hb[i] * fabsf(dot(b[i], L)); }
        const float pen = rA + rB - fabsf(dot(T, L));
        if (pen < 0.f) return 0;
        if (pen < best_face) { best_face = pen; face = k; }
    }
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            f3 L = cross(a[i], b[j]);
            const float len = sqrtf(dot(L, L));
            if (len < 1e-6f) continue;
            L = (1.f / len) * L;
            float rA = 0.f, rB = 0.f;
#pragma unroll
            for (int k = 0; k < 3; ++k) { rA += ha[k] * fabsf(dot(a[k], L)); rB += hb[k] * fabsf(dot(b[k], L)); }
            const float pen = rA + rB - fabsf(dot(T, L));
            if (pen < 0.f) return 0;
            if (pen < best_edge) { best_edge = pen; ei = i; ej = j; eaxis = L; }
        }
    if (ei >= 0 && best_edge < 0.95f * best_face - 1e-5f) {
        f3 L = eaxis;
        if (dot(L, T) > 0.f) L = -L;
        n = L;
        f3 pa = cA, pb = cB;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if (k != ei) pa = pa + ((dot(a[k], n) > 0.f ? -1.f : 1.f) * ha[k]) * a[k];
            if (k != ej) pb = pb + ((dot(b[k], n) > 0.f ? 1.f : -1.f) * hb[k]) * b[k];
        }
        const f3 u = sel3(a[0], a[1], a[2], ei), v = sel3(b[0], b[1], b[2], ej);
        const float hae = self3(ha[0], ha[1], ha[2], ei), hbe = self3(hb[0], hb[1], hb[2], ej);
        const f3 w0 = pa - pb;
        const float uv = dot(u, v), uw = dot(u, w0), vw = dot(v, w0);
        const float den = 1.f - uv * uv;
        float s = den > 1e-12f ? (uv * vw - uw) / den : 0.f;
        float t = den > 1e-12f ? (vw - uv * uw) / den : 0.f;
        s = fminf(fmaxf(s, -hae), hae);
        t = fminf(fmaxf(t, -hbe), hbe);
        out.set(0, 0.5f * ((pa + s * u) + (pb + t * v)), best_edge);
        return 1;
    }
    const bool refA = face < 3;
    const int fk = refA ? face : face - 3;
    const f3 cR = refA ? cA : cB, cI = refA ? cB : cA;
    const f3 R0 = refA ? a[0] : b[0], R1 = refA ? a[1] : b[1], R2 = refA ? a[2] : b[2];
    const f3 I0 = refA ? b[0] : a[0], I1 = refA ? b[1] : a[1], I2 = refA ? b[2] : a[2];
    const float hR0 = refA ? ha[0] : hb[0], hR1 = refA ? ha[1] : hb[1], hR2 = refA ? ha[2] : hb[2];
    const float hI0 = refA ? hb[0] : ha[0], hI1 = refA ? hb[1] : ha[1], hI2 = refA ? hb[2] : ha[2];
    f3 nr = sel3(R0, R1, R2, fk);
    if (dot(nr, cI - cR) < 0.f) nr = -nr;
    n = refA ? -nr : nr;
    int ik = 0;
    float bd = 0.f;
    {
        const float d0 = fabsf(dot(I0, nr)), d1 = fabsf(dot(I1, nr)), d2 = fabsf(dot(I2, nr));
        if (d0 > bd) { bd = d0; ik = 0; }
        if (d1 > bd) { bd = d1; ik = 1; }
        if (d2 > bd) { bd = d2; ik = 2; }
    }
    const f3 Iik = sel3(I0, I1, I2, ik);
    const float sg = dot(Iik, nr) > 0.f ? -1.f : 1.f;
    const int k1 = (ik + 1) % 3, k2 = (ik + 2) % 3;
    const int u1 = (fk + 1) % 3, u2 = (fk + 2) % 3;
    const f3 Ik1 = sel3(I0, I1, I2, k1), Ik2 = sel3(I0, I1, I2, k2);
    const float hIik = self3(hI0, hI1, hI2, ik), hIk1 = self3(hI0, hI1, hI2, k1), hIk2 = self3(hI0, hI1, hI2, k2);
    const f3 Ru1 = sel3(R0, R1, R2, u1), Ru2 = sel3(R0, R1, R2, u2);
    const float hRu1 = self3(hR0, hR1, hR2, u1), hRu2 = self3(hR0, hR1, hR2, u2);
    const f3 fc = cR + self3(hR0, hR1, hR2, fk) * nr;
    // polygon: (u, v, x, y, z) per vertex, clipped between the workspace's two
    // polygons (at most 8 vertices): word (8 c + i) 5 + k of the lane's column
    auto poly = [ws](int c, int i, int k) -> float& { return ws[((8 * c + i) * 5 + k) * kScClipLanes]; };
    const float sx[4] = {1.f, -1.f, -1.f, 1.f}, sy[4] = {1.f, 1.f, -1.f, -1.f};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const f3 x = cI + (sg * hIik) * Iik + (sx[q] * hIk1) * Ik1 + (sy[q] * hIk2) * Ik2;
        const f3 rel = x - fc;
        poly(0, q, 0) = dot(rel, Ru1);
        poly(0, q, 1) = dot(rel, Ru2);
        poly(0, q, 2) = x.x; poly(0, q, 3) = x.y; poly(0, q, 4) = x.z;
    }
    int cnt = 4, cur = 0;
    for (int plane = 0; plane < 4 && cnt > 0; ++plane) {
        const int axis = plane >> 1;
        const float s2 = (plane & 1) ? -1.f : 1.f;
        const float h = axis ? hRu2 : hRu1;
        int m = 0;
        for (int i = 0; i < cnt; ++i) {
            const int j = (i + 1 < cnt) ? i + 1 : 0;
            const float dp = s2 * poly(cur, i, axis) - h, dq = s2 * poly(cur, j, axis) - h;
            if (dp <= 0.f && m < 8) {
#pragma unroll
                for (int k = 0; k < 5; ++k) poly(cur ^ 1, m, k) = poly(cur, i, k);
                ++m;
            }
            if (((dp < 0.f && dq > 0.f) || (dp > 0.f && dq < 0.f)) && m < 8) {
                const float t = dp / (dp - dq);
#pragma unroll
                for (int k = 0; k < 5; ++k) {
                    const float P = poly(cur, i, k);
                    poly(cur ^ 1, m, k) = P + t * (poly(cur, j, k) - P);
                }
                ++m;
            }
        }
        cnt = m;
        cur ^= 1;
    }
    int np = 0;
    for (int i = 0; i < cnt; ++i) {
        const f3 x = {poly(cur, i, 2), poly(cur, i, 3), poly(cur, i, 4)};
        const float dep = dot(fc - x, nr);
        if (dep > 0.f && np < 8) { out.set(np, x, dep); ++np; }
    }
    return sc_reduce(np, out);
}

__device__ __forceinline__ int sc_box_sphere(f3 h, f3 c, const M3& R, float rad, f3 s, f3& nbs, f3& pt, float& dep) {
    const f3 l = mulT(R, s - c);
    const f3 q = {fminf(fmaxf(l.x, -h.x), h.x), fminf(fmaxf(l.y, -h.y), h.y), fminf(fmaxf(l.z, -h.z), h.z)};
    const bool inside = q.x == l.x && q.y == l.y && q.z == l.z;
    if (!inside) {
        f3 e = l - q;
        const float dist = sqrtf(dot(e, e));
        if (dist > rad || dist <= 0.f) return 0;  // dist 0: the centre on the face (no direction)
        e = (1.f / dist) * e;
        nbs = mul(R, e);
        pt = c + mul(R, q);
        dep = rad - dist;
        return 1;
    }
    const float g[3] = {h.x - fabsf(l.x), h.y - fabsf(l.y), h.z - fabsf(l.z)};
    int kk = 0;
    if (g[1] < g[kk]) kk = 1;
    if (g[2] < g[kk]) kk = 2;
    const float lk = kk == 0 ? l.x : (kk == 1 ? l.y : l.z);
    const float sg = lk >= 0.f ? 1.f : -1.f;
    f3 lq = l;
    if (kk == 0) lq.x = sg * h.x; else if (kk == 1) lq.y = sg * h.y; else lq.z = sg * h.z;
    nbs = sg * col(R, kk);
    pt = c + mul(R, lq);
    dep = rad + g[kk];
    return 1;
}

// cylinder (h = {radius, half length}, axis z) against a sphere: oracle.c
// cylinder_sphere in float32 (nbs from the cylinder into the sphere, the point
// on the cylinder surface)
__device__ __forceinline__ int sc_cylinder_sphere(f3 h, f3 c, const M3& R, float rad, f3 s, f3& nbs, f3& pt,
                                                  float& dep) {
    const f3 l = mulT(R, s - c);
    const float rho = sqrtf(l.x * l.x + l.y * l.y);
    const bool inside = rho <= h.x && fabsf(l.z) <= h.y;
    if (!inside) {
        const float k = rho > h.x ? h.x / rho : 1.f;
        const f3 q = {l.x * k, l.y * k, fminf(fmaxf(l.z, -h.y), h.y)};
        f3 e = l - q;
        const float dist = sqrtf(dot(e, e));
        if (dist > rad || dist == 0.f) return 0;
        e = (1.f / dist) * e;
        nbs = mul(R, e);
        pt = c + mul(R, q);
        dep = rad - dist;
        return 1;
    }
    const float gs = h.x - rho, gc = h.y - fabsf(l.z);
    const bool side = gs < gc && rho > 0.f;
    const float sg = l.z >= 0.f ? 1.f : -1.f;
    const float ir = side ? 1.f / rho : 0.f;
    const f3 e = {side ? l.x * ir : 0.f, side ? l.y * ir : 0.f, side ? 0.f : sg};
    const f3 q = {side ? h.x * e.x : l.x, side ? h.x * e.y : l.y, side ? l.z : sg * h.y};
    nbs = mul(R, e);
    pt = c + mul(R, q);
    dep = rad + (side ? gs : gc);
    return 1;
}

// cylinder pairs (cylinder-box, cylinder-cylinder): oracle.c cylinder_pair in
// float32 -- least-overlap axis among the shapes' candidate axes (box faces;
// cylinder axis and radial direction), sampled features (box corners; 4 rim
// points per cap at 0.999 r facing the other centre) inside the other shape
// and past its extreme plane, <= 8 kept, reduced to 4
__device__ __forceinline__ float sc_support(int type, f3 h, const M3& R, f3 n) {
    if (type == 0)
        return h.x * fabsf(dot(n, col(R, 0))) + h.y * fabsf(dot(n, col(R, 1))) + h.z * fabsf(dot(n, col(R, 2)));
    const float c = dot(n, col(R, 2));
    return h.x * sqrtf(fmaxf(1.f - c * c, 0.f)) + h.y * fabsf(c);
}

__device__ __forceinline__ int sc_axes(int type, f3 c, const M3& R, f3 other, f3* ax) {
    if (type == 0) {
        ax[0] = col(R, 0);
        ax[1] = col(R, 1);
        ax[2] = col(R, 2);
        return 3;
    }
    ax[0] = col(R, 2);
    const f3 d = other - c;
    const f3 q = d - dot(d, ax[0]) * ax[0];
    const float nq = sqrtf(dot(q, q));
    if (nq <= 1e-9f) return 1;
    ax[1] = (1.f / nq) * q;
    return 2;
}

__device__ __forceinline__ f3 sc_pair_sample(int type, f3 h, f3 c, const M3& R, f3 other, int k) {
    f3 l;
    if (type == 0) {
        l = {(k & 4) ? h.x : -h.x, (k & 2) ? h.y : -h.y, (k & 1) ? h.z : -h.z};
    } else {
        const f3 d = mulT(R, other - c);
        float ux = d.x, uy = d.y;
        const float n2 = ux * ux + uy * uy;
        if (n2 > 1e-12f) {
            const float inv = 1.f / sqrtf(n2);
            ux *= inv;
            uy *= inv;
        } else {
            ux = 1.f;
            uy = 0.f;
        }
        const int j = k & 3;
        const float dx = (j == 0) ? ux : ((j == 1) ? -uy : ((j == 2) ? -ux : uy));
        const float dy = (j == 0) ? uy : ((j == 1) ? ux : ((j == 2) ? -uy : -ux));
        l = {0.999f * h.x * dx, 0.999f * h.x * dy, (k & 4) ? h.y : -h.y};
    }
    return c + mul(R, l);
}

__device__ __forceinline__ bool sc_inside(int type, f3 h, f3 c, const M3& R, f3 p) {
    const f3 l = mulT(R, p - c);
    if (type == 0) return h.x - fabsf(l.x) > 0.f && h.y - fabsf(l.y) > 0.f && h.z - fabsf(l.z) > 0.f;
    return h.x - sqrtf(l.x * l.x + l.y * l.y) > 0.f && h.y - fabsf(l.z) > 0.f;
}

// Inlined (r03).  Round 2 kept it out of line after an inlined build showed
// NaN poses in box / sphere piles that never reach it; re-tested in r03 with
// it inlined and the MW_SC_NANCHECK build (every phase of every step checked
// for a non-finite pose, coordinate or contact): no non-finite value in any
// scene test, and the inlined kernel spills less (scratch 1040 -> 944 B per
// lane, SGPR spills 547 -> 84).  The one division that could see a zero
// under -ffinite-math-only (sc_box_sphere's 1 / dist) is guarded.
__device__ __forceinline__ int sc_cylinder_pair(int ta, f3 ha, f3 ca, const M3& Ra, int tb, f3 hb, f3 cb,
                                                const M3& Rb, f3& n, const ScWsPts& out) {
    f3 ax[6];
    int na = sc_axes(ta, ca, Ra, cb, ax);
    na += sc_axes(tb, cb, Rb, ca, ax + na);
    const f3 dab = ca - cb;
    int best = -1;
    float ov_min = 0.f;
    for (int k = 0; k < na; ++k) {
        const float ov = sc_support(ta, ha, Ra, ax[k]) + sc_support(tb, hb, Rb, ax[k]) - fabsf(dot(ax[k], dab));
        if (ov <= 0.f) return 0;
        if (best < 0 || ov < ov_min) { ov_min = ov; best = k; }
    }
    n = dot(ax[best], dab) >= 0.f ? ax[best] : -ax[best];
    const float plane_b = dot(n, cb) + sc_support(tb, hb, Rb, n);
    const float plane_a = dot(n, ca) - sc_support(ta, ha, Ra, n);
    int m = 0;
    for (int side = 0; side < 2; ++side)
        for (int k = 0; k < 8 && m < 8; ++k) {
            const f3 q = side ? sc_pair_sample(tb, hb, cb, Rb, ca, k) : sc_pair_sample(ta, ha, ca, Ra, cb, k);
            const bool in = side ? sc_inside(ta, ha, ca, Ra, q) : sc_inside(tb, hb, cb, Rb, q);
            const float dep = side ? dot(n, q) - plane_a : plane_b - dot(n, q);
            if (!in || dep <= 0.f) continue;
            out.set(m, q, dep);
            ++m;
        }
    return sc_reduce(m, out);
}

// ---- the hull narrow phase of mesh shapes (round 6; oracle.c hull_pair) ----
// A mesh collides with boxes and other meshes as the convex hull of its
// support points (scene_params.hpp ScHull, built by hull.hpp on the host);
// a box as the unit box hull scaled by its half extents.
struct ScPoly {
    const ScHull* H;
    f3 s;      // vertex scale: the half extents of a box, 1 for a mesh
    bool box;
    __device__ __forceinline__ f3 v(int i) const { return {H->v[i][0] * s.x, H->v[i][1] * s.y, H->v[i][2] * s.z}; }
    __device__ __forceinline__ f3 n(int f) const { return {H->plane[f][0], H->plane[f][1], H->plane[f][2]}; }
    __device__ __forceinline__ float d(int f) const {
        return box ? fabsf(H->plane[f][0]) * s.x + fabsf(H->plane[f][1]) * s.y + fabsf(H->plane[f][2]) * s.z
                   : H->plane[f][3];
    }
    __device__ __forceinline__ f3 ctr() const { return {H->ctr[0] * s.x, H->ctr[1] * s.y, H->ctr[2] * s.z}; }
};

// closest points of segments p0 + s u, q0 + t v (s, t in [0, 1]): their midpoint
__device__ __forceinline__ f3 sc_segment_mid(f3 p0, f3 p1, f3 q0, f3 q1) {
    const f3 u = p1 - p0, v = q1 - q0, w = p0 - q0;
    const float a = dot(u, u), b = dot(u, v), c = dot(v, v), d = dot(u, w), e = dot(v, w);
    const float den = a * c - b * b;
    float s = den > 1e-18f * a * c ? (b * e - c * d) / den : 0.f;
    s = fminf(fmaxf(s, 0.f), 1.f);
    float t = c > 0.f ? (b * s + e) / c : 0.f;
    if (t < 0.f || t > 1.f) {
        t = fminf(fmaxf(t, 0.f), 1.f);
        s = a > 0.f ? (b * t - d) / a : 0.f;
        s = fminf(fmaxf(s, 0.f), 1.f);
    }
    return 0.5f * ((p0 + s * u) + (q0 + t * v));
}

constexpr int kScClipMax = 24;   // clipped polygon (a hull face has <= 16 vertices; the oracle keeps 40)

// Polytope A vs polytope B (shape frames (cA, RA), (cB, RB)): the separating-
// axis test over both face-normal sets and the edge pairs whose Gauss-map
// arcs cross (the faces of the Minkowski difference), reference-face clipping
// of the incident face; the float32 restatement of oracle.c hull_pair (same
// loops, tie rules and reduction).  Normal from B into A.  A call, not
// inlined: only mesh pairs reach it.
__device__ __noinline__ int sc_hull_pair(ScPoly A, f3 cA, M3 RA, ScPoly B, f3 cB, M3 RB, f3& n, ScWsPts out) {
    float pen[2] = {3.0e38f, 3.0e38f};
    int face[2] = {-1, -1};
    for (int side = 0; side < 2; ++side) {
        const ScPoly& H = side ? B : A;
        const ScPoly& O = side ? A : B;
        const M3& R = side ? RB : RA;
        const M3& Ro = side ? RA : RB;
        const f3 c = side ? cB : cA, co = side ? cA : cB;
        for (int f = 0; f < H.H->nf; ++f) {
            const f3 nw = mul(R, H.n(f));
            const float dw = H.d(f) + dot(nw, c);
            const f3 nl = mulT(Ro, nw);   // the normal in the other shape's frame
            float mn = 3.0e38f;
            for (int j = 0; j < O.H->nv; ++j) mn = fminf(mn, dot(nl, O.v(j)));
            const float ov = dw - (mn + dot(nw, co));
            if (ov < 0.f) return 0;
            if (ov < pen[side]) { pen[side] = ov; face[side] = f; }
        }
    }
    const f3 ca = cA + mul(RA, A.ctr()), cb = cB + mul(RB, B.ctr());
    float pen_e = 3.0e38f;
    f3 eaxis = {0.f, 0.f, 0.f};
    int ea = -1, eb = -1;
    for (int i = 0; i < A.H->ne; ++i) {
        const f3 a = mul(RA, A.n(A.H->ef[i][0])), b = mul(RA, A.n(A.H->ef[i][1]));
        const f3 bxa = cross(b, a);
        const f3 pa0 = cA + mul(RA, A.v(A.H->e[i][0])), pa1 = cA + mul(RA, A.v(A.H->e[i][1]));
        const f3 da = pa1 - pa0;
        for (int j = 0; j < B.H->ne; ++j) {
            const f3 c = -mul(RB, B.n(B.H->ef[j][0])), d = -mul(RB, B.n(B.H->ef[j][1]));
            const f3 dxc = cross(d, c);
            const float cba = dot(c, bxa), dba = dot(d, bxa), adc = dot(a, dxc), bdc = dot(b, dxc);
            if (!(cba * dba < 0.f && adc * bdc < 0.f && cba * bdc > 0.f)) continue;
            const f3 pb0 = cB + mul(RB, B.v(B.H->e[j][0])), pb1 = cB + mul(RB, B.v(B.H->e[j][1]));
            const f3 db = pb1 - pb0;
            f3 u = cross(da, db);
            const float len = sqrtf(dot(u, u));
            if (len <= 1e-6f * sqrtf(dot(da, da) * dot(db, db))) continue;
            u = (1.f / len) * u;
            if (dot(u, cb - ca) < 0.f) u = -u;   // A -> B
            const f3 ul = mulT(RA, u), vl = mulT(RB, u);
            float amax = -3.0e38f, bmin = 3.0e38f;
            for (int p = 0; p < A.H->nv; ++p) amax = fmaxf(amax, dot(ul, A.v(p)));
            for (int p = 0; p < B.H->nv; ++p) bmin = fminf(bmin, dot(vl, B.v(p)));
            const float ov = (amax + dot(u, cA)) - (bmin + dot(u, cB));
            if (ov < 0.f) return 0;
            if (ov < pen_e) { pen_e = ov; ea = i; eb = j; eaxis = u; }
        }
    }
    const bool refB = pen[1] < 0.95f * pen[0] - 1e-5f;
    const float pen_f = refB ? pen[1] : pen[0];
    if (ea >= 0 && pen_e < 0.95f * pen_f - 1e-5f) {
        n = -eaxis;
        out.set(0, sc_segment_mid(cA + mul(RA, A.v(A.H->e[ea][0])), cA + mul(RA, A.v(A.H->e[ea][1])),
                                  cB + mul(RB, B.v(B.H->e[eb][0])), cB + mul(RB, B.v(B.H->e[eb][1]))),
                pen_e);
        return 1;
    }
    const ScPoly& Rp = refB ? B : A;
    const ScPoly& Ip = refB ? A : B;
    const M3& Rr = refB ? RB : RA;
    const M3& Ri = refB ? RA : RB;
    const f3 cr = refB ? cB : cA, ci = refB ? cA : cB;
    const int fr = face[refB ? 1 : 0];
    const f3 nr = mul(Rr, Rp.n(fr));   // pointing to the incident polytope
    const float dr = Rp.d(fr) + dot(nr, cr);
    int fi = 0;
    float best = 3.0e38f;
    for (int f = 0; f < Ip.H->nf; ++f) {
        const float sdot = dot(mul(Ri, Ip.n(f)), nr);
        if (sdot < best) { best = sdot; fi = f; }
    }
    f3 buf[2][kScClipMax];
    int cnt = Ip.H->fnv[fi], cur = 0;
    for (int k = 0; k < cnt; ++k) buf[0][k] = ci + mul(Ri, Ip.v(Ip.H->fv[fi][k]));
    const int nrv = Rp.H->fnv[fr];
    for (int k = 0; k < nrv && cnt > 0; ++k) {
        const f3 r0 = cr + mul(Rr, Rp.v(Rp.H->fv[fr][k]));
        const f3 r1 = cr + mul(Rr, Rp.v(Rp.H->fv[fr][(k + 1) % nrv]));
        const f3 sn = cross(r1 - r0, nr);   // outward side-plane normal
        const float s0 = dot(sn, r0);
        int m = 0;
        for (int i = 0; i < cnt; ++i) {
            const f3 P = buf[cur][i], Q = buf[cur][(i + 1) % cnt];
            const float dp = dot(sn, P) - s0, dq = dot(sn, Q) - s0;
            if (dp <= 0.f && m < kScClipMax) buf[cur ^ 1][m++] = P;
            if (((dp < 0.f && dq > 0.f) || (dp > 0.f && dq < 0.f)) && m < kScClipMax) {
                const float t = dp / (dp - dq);
                buf[cur ^ 1][m++] = P + t * (Q - P);
            }
        }
        cnt = m;
        cur ^= 1;
    }
    // the points below the reference face, compacted in place
    float D8[kScClipMax];
    int np = 0;
    for (int i = 0; i < cnt; ++i) {
        const float dep = dr - dot(nr, buf[cur][i]);
        if (dep > 0.f) { buf[cur][np] = buf[cur][i]; D8[np] = dep; ++np; }
    }
    np = sc_reduce(np, ScArrPts{buf[cur], D8});
    n = refB ? nr : -nr;
    for (int i = 0; i < np; ++i) out.set(i, buf[cur][i], D8[i]);
    return np;
}

// shapes a, b (type 0 box: size = half extents, 1 sphere: size.x = radius,
// 2 cylinder: size = {radius, half length}): normal from B into A, up to 4
// points / depths
// shapes a, b (type 0 box: size = half extents, 1 sphere: size.x = radius,
// 2 cylinder: size = {radius, half length}): normal from B into A, up to 4
// points / depths into the lane's workspace slots (ws: its column of
// ScWorld::clip)
__device__ __forceinline__ int sc_collide(int ta, f3 sa, f3 ca, const M3& Ra, int tb, f3 sb, f3 cb, const M3& Rb,
                                          f3& n, float* ws) {
    const ScWsPts out{ws + kScWsOut * kScClipLanes};
    f3 pt, nbs;
    float dep;
    if ((ta == 2 && tb == 1) || (ta == 1 && tb == 2)) {
        if (ta == 2) {  // cylinder A, sphere B: n from B into A
            if (!sc_cylinder_sphere(sa, ca, Ra, sb.x, cb, nbs, pt, dep)) return 0;
            n = -nbs;
        } else {
            if (!sc_cylinder_sphere(sb, cb, Rb, sa.x, ca, nbs, pt, dep)) return 0;
            n = nbs;
        }
        out.set(0, pt, dep);
        return 1;
    }
    if (ta == 2 || tb == 2) return sc_cylinder_pair(ta, sa, ca, Ra, tb, sb, cb, Rb, n, out);
    if (ta == 0 && tb == 0) return sc_box_box(sa, ca, Ra, sb, cb, Rb, n, out, ws + kScWsPoly * kScClipLanes);
    if (ta == 1 && tb == 1) {
        const f3 d = ca - cb;
        const float dist = sqrtf(dot(d, d));
        const float pen = sa.x + sb.x - dist;
        if (pen < 0.f || dist < 1e-12f) return 0;
        n = (1.f / dist) * d;
        out.set(0, cb + (sb.x - 0.5f * pen) * n, pen);
        return 1;
    }
    if (ta == 0) {
        if (!sc_box_sphere(sa, ca, Ra, sb.x, cb, nbs, pt, dep)) return 0;
        n = -nbs;
    } else {
        if (!sc_box_sphere(sb, cb, Rb, sa.x, ca, nbs, pt, dep)) return 0;
        n = nbs;
    }
    out.set(0, pt, dep);
    return 1;
}

// exclusive prefix over the wave of per-lane counts in [0, 7]
__device__ __forceinline__ int wave_prefix7(int v, int& total) {
    const uint64_t lt = (uint64_t{1} << lane_id()) - 1u;
    int pre = 0;
    total = 0;
#pragma unroll
    for (int bit = 0; bit < 3; ++bit) {
        const uint64_t m = __ballot((v >> bit) & 1);
        pre += (1 << bit) * __popcll(m & lt);
        total += (1 << bit) * __popcll(m);
    }
    return pre;
}

// ------------------------------------------------------------------ responses
// Response of the row in MJ / J (accumulated) to a spatial impulse f on node k
// (k < K: a base) or, with k = -1, to a unit impulse on body j's joint; returns
// J nu.  Same passes as wave_response, restricted to k's model.
template <int MAXNV>
__device__ __forceinline__ float sc_response(const SceneF* __restrict__ P, ScWorld<MAXNV>& L, int k, int j, SV f,
                                             float* __restrict__ Jrow, float* __restrict__ MJrow) {
    const int lane = lane_id();
    const int m = (k >= 0) ? P->node_model[k] : P->body_model[j];
    const SceneModelF& md = P->model[m];
    const int start = (k >= 0) ? P->node_body[k] : j;
    const uint64_t path = (start >= 0) ? P->body_path[start] : uint64_t{0};
    SV Bi = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}}, Fi = Bi;
    if (k >= 0) { Bi = -1.f * f; Fi = f; }
    float jv = 0.f;
    for (uint64_t mm = path; mm != 0;) {
        const int i = 63 - __builtin_clzll(mm);
        mm &= ~(uint64_t{1} << i);
        const BodyF& b = P->b[i];
        const ScNode& s = L.node[P->body_node[i]];
        const int c = P->body_coord[i];
        const float ji = proj(b, Fi);
        Jrow[c] += ji;
        jv += ji * L.nu[c];
        const float u = ((i == j) ? 1.f : 0.f) - proj(b, Bi);
        L.stack[s.depth - 1][6][lane] = u;
        Bi = dad_inv(s.R, s.p, Bi + (s.psi * u) * s.U);
        Fi = dad_inv(s.R, s.p, Fi);
    }
    SV dV0 = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
    if (md.floating) {
        const int o = md.coff;
        const float fb[6] = {Fi.w.x, Fi.w.y, Fi.w.z, Fi.v.x, Fi.v.y, Fi.v.z};
#pragma unroll
        for (int e = 0; e < 6; ++e) {
            Jrow[o + e] += fb[e];
            jv += fb[e] * L.nu[o + e];
        }
        Chol6 L0;
#pragma unroll
        for (int e = 0; e < 21; ++e) L0.l[e] = L.l0[m][e];
#pragma unroll
        for (int e = 0; e < 6; ++e) L0.id[e] = L.l0[m][21 + e];
        dV0 = L0.solve(-1.f * Bi);
        const float dv[6] = {dV0.w.x, dV0.w.y, dV0.w.z, dV0.v.x, dV0.v.y, dV0.v.z};
#pragma unroll
        for (int e = 0; e < 6; ++e) MJrow[o + e] += dv[e];
    }
    SV dv_prev = dV0;
    const int i0 = md.body0, i1 = md.body0 + md.n_bodies;
    for (int i = i0; i < i1; ++i) {
        const BodyF& b = P->b[i];
        const ScNode& s = L.node[P->body_node[i]];
        const int pa = b.parent;
        SV dvp_in;
        if (pa == i - 1 && i > i0) {
            dvp_in = dv_prev;
        } else if (pa >= 0) {
            const int dp = L.node[P->body_node[pa]].depth - 1;
            dvp_in = {{L.stack[dp][0][lane], L.stack[dp][1][lane], L.stack[dp][2][lane]},
                      {L.stack[dp][3][lane], L.stack[dp][4][lane], L.stack[dp][5][lane]}};
        } else {
            dvp_in = dV0;
        }
        const SV dvp = ad_inv(s.R, s.p, dvp_in);
        const float u = ((path >> i) & 1u) ? L.stack[s.depth - 1][6][lane] : 0.f;
        const float mmv = s.psi * (u - dot(s.U, dvp));
        MJrow[P->body_coord[i]] += mmv;
        const SV dv = dvp + motion(b, mmv);
        dv_prev = dv;
        float* st = &L.stack[s.depth - 1][0][lane];
        st[0 * kWaveLanes] = dv.w.x; st[1 * kWaveLanes] = dv.w.y; st[2 * kWaveLanes] = dv.w.z;
        st[3 * kWaveLanes] = dv.v.x; st[4 * kWaveLanes] = dv.v.y; st[5 * kWaveLanes] = dv.v.z;
    }
    return jv;
}

// joint force of body d on substep s (dof_force with the model's PID gate)
__device__ __forceinline__ float sc_dof_force(const SceneF* __restrict__ P, const SceneDev& S,
                                              const PidF* __restrict__ pid, const SceneGates& G, int W, int w,
                                              const SceneArgs& A, int s, int d, uint32_t act, float cmd, float vc,
                                              float q, float qd) {
    const float e = P->b[d].effort;
    float tau = (act == kActForce && s == 0) ? fminf(fmaxf(cmd, -e), e) : 0.f;
    if (act >= kActPidPos) {
        const size_t k = static_cast<size_t>(d) * W + w;
        float u = S.pid_u[k];
        if ((G.gate[P->body_model[d]] >> s) & 1u) {
            const float err = (act == kActPidPos) ? (q - S.ptgt[k]) : (qd - vc);
            float el = S.pid_e[k], ie = S.pid_i[k];
            if (pid_update(pid[d], err, A.inv_dt, A.dt, el, ie, u)) {
                S.pid_e[k] = el; S.pid_i[k] = ie; S.pid_u[k] = u;
            } else {
                u = 0.f;
            }
        }
        tau = fminf(fmaxf(u, -e), e);
    }
    return tau;
}

// Debug builds (EXTRA=-DMW_SC_NANCHECK): after each phase of a step, the
// first non-finite value of the node records, coordinates and contacts of a
// world is printed (bit test of the exponent: -ffinite-math-only folds isfinite)
#ifdef MW_SC_NANCHECK
__device__ __forceinline__ bool sc_bad(float v) { return nonfinite_bits(v); }
template <int MAXNV>
__device__ void sc_nancheck(const SceneF* __restrict__ P, const ScWorld<MAXNV>& L, int phase, int nc, bool& reported) {
    const int lane = lane_id();
    int what = -1;
    float val = 0.f;
    if (lane < P->n_nodes) {
        const ScNode& nd = L.node[lane];
        const float* f = reinterpret_cast<const float*>(&nd);
        for (int k = 0; k < 38; ++k)
            if (sc_bad(f[k])) { what = k; val = f[k]; break; }
    }
    if (what < 0 && lane < P->nv && sc_bad(L.nu[lane])) { what = 100; val = L.nu[lane]; }
    if (what < 0 && lane < nc) {
        for (int k = 0; k < 3; ++k)
            if (sc_bad(L.c_p[lane][k]) || sc_bad(L.c_n[lane][k])) { what = 200 + k; val = L.c_p[lane][k]; }
        if (sc_bad(L.c_d[lane])) { what = 210; val = L.c_d[lane]; }
    }
    const uint64_t m = __ballot(what >= 0);
    if (m && !reported) {
        const int l = __builtin_ctzll(m);
        if (lane == l)
            printf("MW_SC_NANCHECK world %d phase %d lane %d field %d value %08x nc %d\n", (int)blockIdx.x, phase,
                   lane, what, __float_as_uint(val), nc);
        reported = true;
    }
}
#define MW_SC_CHECK(ph, ncv) sc_nancheck<MAXNV>(P, L, ph, ncv, nan_reported)
#else
#define MW_SC_CHECK(ph, ncv)
#endif

// ---------------------------------------------------------- large-contact steps
// DART's step has no contact cap (Physics.cpp:1824-1835; World.cpp:70-180
// inserts any number of models).  A world-step with more contact points than
// the LDS record holds (kScMaxContacts) or more rows than the 64-lane
// register LCP runs its constraint phase in the world's workspace in HBM
// (SceneDev::big, sized by the host from the scene's worst case up to
// kScBigContacts points / kScBigRows rows): the same rows, responses and
// Delassus arithmetic as the compact path, in 64-row batches through the LDS
// rows, and DART's two-stage boxed LCP (wave_lcp.hpp header) by the same
// primal active-set method as wave_boxqp over the whole system, each linear
// solve a dense LDL^T of the free rows in 64x64 tiles in the workspace.
// (Block Gauss-Seidel over 64-row exact blocks was tried first: on a row of
// eight cubes in face contact, cond(A) ~ 1e6, its fp64 emulation needed 48
// sweeps for stage 1 and stalled at 100x the tolerance in stage 2.)  Cold
// start from PGS sweeps (the warm record keys kScMaxContacts points).
constexpr int kScBigFields = 11;   // per-row fields of the workspace (below)
struct ScBigWs {
    float* base;   // this world's workspace, nullptr: none
    int cmax, R;   // contact and row capacity (R: a multiple of 64)
    int nvmax;     // the instance's MAXNV (leading dimension of J^T / MJ^T)
    __device__ float* ct(int c) const { return base + static_cast<size_t>(c) * kScBigContactWords; }
    // row fields: 0 joint-row source (3 body + type, int bits), 1 b, 2 lo, 3
    // hi (the rows' own boxes), 4 stage-1 impulse, 5 / 6 the stage's box, 7
    // active-set state (int bits: 0-1 held at none / lo / hi, 2 frozen, 3
    // released), 8 gradient A x - b, 9 residual tolerance, 10 LDL^T pivot
    __device__ float* row(int f) const {
        return base + static_cast<size_t>(cmax) * kScBigContactWords + static_cast<size_t>(f) * R;
    }
    __device__ float* JT() const { return row(kScBigFields); }
    __device__ float* MJT() const { return row(kScBigFields) + static_cast<size_t>(nvmax) * R; }
    __device__ float* A() const { return row(kScBigFields) + 2 * static_cast<size_t>(nvmax) * R; }
    __device__ float* Lf() const { return A() + static_cast<size_t>(R) * R; }
};

// LDS scratch of the large-contact LCP (inside ScWorld's union), as LDS
// pointers: generic ones made the compiler form (and hoist, and spill) a
// flat -> LDS conversion per address of the unrolled tile loops
using lds_float = __attribute__((address_space(3))) float;
struct ScBigLds {
    lds_float* xs;   // [kScBigRows] impulses
    lds_float* vs;   // [kScBigRows] the solve's right-hand side / result
    lds_float* T0;   // [64][64] the current diagonal tile: l_rc below, d_c on the diagonal
    lds_float* T1;   // [64][64] a panel tile
};
constexpr int kScBigLdsFloats = 2 * kScBigRows + 2 * 64 * 64;
constexpr int kScBigSweeps = 24;   // PGS sweeps before each stage's active-set solve

// contact c of the narrow phase into the workspace
__device__ __forceinline__ void sc_big_put(const ScBigWs& G, int c, f3 x, f3 n, float dep, int na, int nb, int key) {
    float* o = G.ct(c);
    o[0] = x.x; o[1] = x.y; o[2] = x.z;
    o[3] = n.x; o[4] = n.y; o[5] = n.z;
    o[12] = dep;
    o[13] = __int_as_float(na);
    o[14] = __int_as_float(nb);
    o[15] = __int_as_float(key);
}

// one 64x64 Delassus block on the matrix cores (the compact path's tiles):
// rows from the LDS rows L.J (block i), columns from L.MJ (block j); lane c
// ends with a[r] = J_r . MJ_c.  Columns >= NV of both are zero.
template <int MAXNV>
__device__ __forceinline__ void sc_tile64(const ScWorld<MAXNV>& L, int NV, float (&a)[kWaveLanes]) {
    const int lane = lane_id();
    const int lr = lane & 31, lh = lane >> 5;
    v16f t00 = {}, t01 = {}, t10 = {}, t11 = {};
    constexpr int kKs = MAXNV / 2;
#pragma unroll
    for (int k0 = 0; k0 < kKs; k0 += 4) {
        if (2 * k0 >= NV) break;
        float jv0[4], mv0[4], jv1[4], mv1[4];
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const int e = 2 * (k0 + kk) + lh;
            jv0[kk] = L.J[lr][e];
            mv0[kk] = L.MJ[lr][e];
            jv1[kk] = L.J[32 + lr][e];
            mv1[kk] = L.MJ[32 + lr][e];
        }
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            t00 = __builtin_amdgcn_mfma_f32_32x32x2f32(jv0[kk], mv0[kk], t00, 0, 0, 0);
            t01 = __builtin_amdgcn_mfma_f32_32x32x2f32(jv0[kk], mv1[kk], t01, 0, 0, 0);
            t10 = __builtin_amdgcn_mfma_f32_32x32x2f32(jv1[kk], mv0[kk], t10, 0, 0, 0);
            t11 = __builtin_amdgcn_mfma_f32_32x32x2f32(jv1[kk], mv1[kk], t11, 0, 0, 0);
        }
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
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
}

// (A x)_r for the lane's row r over the first n columns (A symmetric: column
// r, coalesced over the lanes), compensated as lcp_matvec (Dot2); mag = sum
// |A_rc x_c|.  Rows are padded to 64, so every read is inside A.
__device__ __forceinline__ float sc_big_dot(const float* __restrict__ A, int R, const lds_float* __restrict__ xs, int r,
                                            int n, float& mag) {
#pragma clang fp contract(off)
    float w = 0.f, cc = 0.f, m = 0.f;
    for (int c0 = 0; c0 < n; c0 += 8) {
        float av[8], xv[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            av[k] = A[static_cast<size_t>(c0 + k) * R + r];
            xv[k] = (c0 + k < n) ? xs[c0 + k] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const float p = av[k] * xv[k];
            const float pe = fmaf(av[k], xv[k], -p);
            const float t = w + p;
            const float z = t - w;
            cc += ((w - (t - z)) + (p - z)) + pe;
            w = t;
            m += fabsf(p);
        }
    }
    mag = m;
    return w + cc;
}

__device__ __forceinline__ int sc_st(const float* st, int r) { return __float_as_int(st[r]); }
__device__ __forceinline__ bool sc_free(int st) { return (st & 3) == 0; }

// Dense LDL^T of the free rows (row state 0; NR.. and held rows: identity)
// in 64x64 tiles, right-looking, lane = column of a tile: Lf's lower
// triangle ends with l_rc d_c (r > c), the pivots d_c in row field 10.
__device__ __noinline__ void sc_big_factor(ScBigWs G, int NR, int nb, ScBigLds S) {
    const int lane = lane_id();
    const int R = G.R;
    const float* A = G.A();
    float* Lf = G.Lf();
    const float* st = G.row(7);
    float* dd = G.row(10);
    for (int bi = 0; bi < nb; ++bi)
        for (int bj = 0; bj <= bi; ++bj) {
            const int c = bj * kWaveLanes + lane;
            const bool fc = c < NR && sc_free(sc_st(st, c));
            for (int i = 0; i < kWaveLanes; ++i) {
                const int r = bi * kWaveLanes + i;
                const bool fr = r < NR && sc_free(sc_st(st, r));
                const float v = A[static_cast<size_t>(r) * R + c];
                Lf[static_cast<size_t>(r) * R + c] = (fr && fc) ? v : ((r == c) ? 1.f : 0.f);
            }
        }
    __threadfence_block();
    for (int k = 0; k < nb; ++k) {
        const size_t o = static_cast<size_t>(kWaveLanes * k) * R + kWaveLanes * k;   // tile (k, k)
        // lane c: column c (the upper entries from row c: symmetric)
        float t[kWaveLanes];
#pragma unroll
        for (int r = 0; r < kWaveLanes; ++r)
            t[r] = (r >= lane) ? Lf[o + static_cast<size_t>(r) * R + lane] : Lf[o + static_cast<size_t>(lane) * R + r];
#pragma unroll
        for (int j = 0; j < kWaveLanes; ++j) {
            float dj = read_lane(t[j], j);
            dj = (fabsf(dj) < 1e-30f) ? 1e-30f : dj;   // the elimination's zero-pivot guard
            const float lc = (lane > j) ? t[j] * rcp(dj) : 0.f;
#pragma unroll
            for (int r = j + 1; r < kWaveLanes; ++r) t[r] = fmaf(-read_lane(t[r], j), lc, t[r]);
        }
        float dc = 1.f;
#pragma unroll
        for (int r = 0; r < kWaveLanes; ++r) dc = (r == lane) ? t[r] : dc;
        dc = (fabsf(dc) < 1e-30f) ? 1e-30f : dc;
        const float ic = rcp(dc);
        wave_lds_sync();
#pragma unroll
        for (int r = 0; r < kWaveLanes; ++r) {
            if (r > lane) Lf[o + static_cast<size_t>(r) * R + lane] = t[r];
            S.T0[r * kWaveLanes + lane] = (r > lane) ? t[r] * ic : ((r == lane) ? dc : 0.f);
        }
        dd[kWaveLanes * k + lane] = dc;
        wave_lds_sync();
        __threadfence_block();
        // panels below: W_ik = A_ik L_kk^-T (= L_ik D_k), lane = row of tile i
        for (int i = k + 1; i < nb; ++i) {
            float* row = Lf + static_cast<size_t>(kWaveLanes * i + lane) * R + kWaveLanes * k;
            float x[kWaveLanes];
#pragma unroll
            for (int c = 0; c < kWaveLanes; ++c) x[c] = row[c];
#pragma unroll
            for (int c = 1; c < kWaveLanes; ++c) {
#pragma unroll
                for (int j = 0; j < c; ++j) x[c] = fmaf(-x[j], S.T0[c * kWaveLanes + j], x[c]);
            }
#pragma unroll
            for (int c = 0; c < kWaveLanes; ++c) row[c] = x[c];
        }
        __threadfence_block();
        // trailing tiles (i, j), k < j <= i: S_ij -= W_ik D_k^-1 W_jk^T, lane = column of tile j
        for (int j = k + 1; j < nb; ++j) {
            const float* wrow = Lf + static_cast<size_t>(kWaveLanes * j + lane) * R + kWaveLanes * k;
            float wj[kWaveLanes];
#pragma unroll
            for (int kk = 0; kk < kWaveLanes; ++kk) wj[kk] = wrow[kk] * rcp(S.T0[kk * kWaveLanes + kk]);
            for (int i = j; i < nb; ++i) {
                wave_lds_sync();
                for (int r = 0; r < kWaveLanes; ++r)
                    S.T1[r * kWaveLanes + lane] = Lf[static_cast<size_t>(kWaveLanes * i + r) * R + kWaveLanes * k + lane];
                wave_lds_sync();
                for (int r = 0; r < kWaveLanes; ++r) {
                    float* a = Lf + static_cast<size_t>(kWaveLanes * i + r) * R + kWaveLanes * j + lane;
                    float acc = *a;
#pragma unroll
                    for (int kk = 0; kk < kWaveLanes; ++kk) acc = fmaf(-S.T1[r * kWaveLanes + kk], wj[kk], acc);
                    *a = acc;
                }
            }
        }
        __threadfence_block();
    }
}

// L D L^T v = vs in place (vs: LDS, rows 0 .. 64 nb)
__device__ __noinline__ void sc_big_solve(ScBigWs G, int nb, ScBigLds S) {
    const int lane = lane_id();
    const int R = G.R;
    const float* Lf = G.Lf();
    const float* dd = G.row(10);
    // forward: L z = v (unit lower, L_rc = Lf_rc / d_c)
    for (int k = 0; k < nb; ++k) {
        const int r = kWaveLanes * k + lane;
        const float* row = Lf + static_cast<size_t>(r) * R;
        float z = S.vs[r];
        for (int j = 0; j < k; ++j)
            for (int c = kWaveLanes * j; c < kWaveLanes * (j + 1); ++c) z = fmaf(-row[c], S.vs[c], z);   // vs: y = z / d
        float lr[kWaveLanes];
#pragma unroll
        for (int c = 0; c < kWaveLanes; ++c) lr[c] = row[kWaveLanes * k + c] * rcp(dd[kWaveLanes * k + c]);
#pragma unroll
        for (int c = 0; c < kWaveLanes; ++c) {
            const float zc = read_lane(z, c);
            z = (lane > c) ? fmaf(-lr[c], zc, z) : z;
        }
        wave_lds_sync();
        S.vs[r] = z * rcp(dd[r]);
        wave_lds_sync();
    }
    // backward: L^T x = y
    for (int k = nb - 1; k >= 0; --k) {
        const int r = kWaveLanes * k + lane;
        const float ir = rcp(dd[r]);
        float y = S.vs[r];
        for (int c = kWaveLanes * (k + 1); c < kWaveLanes * nb; ++c)
            y = fmaf(-Lf[static_cast<size_t>(c) * R + r] * ir, S.vs[c], y);
        float lc[kWaveLanes];
#pragma unroll
        for (int c = 0; c < kWaveLanes; ++c) lc[c] = Lf[static_cast<size_t>(kWaveLanes * k + c) * R + r] * ir;
#pragma unroll
        for (int c = kWaveLanes - 1; c >= 0; --c) {
            const float xc = read_lane(y, c);
            y = (lane < c) ? fmaf(-lc[c], xc, y) : y;
        }
        wave_lds_sync();
        S.vs[r] = y;
        wave_lds_sync();
    }
}

// PGS sweeps over the whole system (rows in order) from xs: fixed boxes
// (row fields 5 / 6: the exact solve's start) or, coupled, DART's PGS
// (friction boxed by the current normal, joint rows by fields 2 / 3).
// Lane l holds w of rows l + 64 k; the sweep stops once no row moved w by
// more than tol (tol < 0: never).
__device__ __noinline__ void sc_big_pgs(ScBigWs G, int NR, int ncr, float mu, int sweeps, bool coupled, float tol,
                                        ScBigLds S) {
    const int lane = lane_id();
    const int R = G.R;
    const float* A = G.A();
    const float* b = G.row(1);
    const float* lo = G.row(coupled ? 2 : 5);
    const float* hi = G.row(coupled ? 3 : 6);
    constexpr int KB = kScBigRows / kWaveLanes;
    for (int it = 0; it < sweeps; ++it) {
        float wk[KB];
#pragma unroll
        for (int k = 0; k < KB; ++k) {
            float mg;
            wk[k] = (k * kWaveLanes < NR) ? sc_big_dot(A, R, S.xs, k * kWaveLanes + lane, NR, mg) : 0.f;
        }
        float h = 0.f, moved = 0.f;
        for (int r = 0; r < NR; ++r) {
            const int kr = r / kWaveLanes;
            float wr = 0.f;
#pragma unroll
            for (int k = 0; k < KB; ++k) wr = (k == kr) ? read_lane(wk[k], r % kWaveLanes) : wr;
            const float xr = S.xs[r];
            const float arr = A[static_cast<size_t>(r) * R + r];
            float v = xr + (b[r] - wr) * rcp(arr);
            if (coupled && r < ncr) {
                if (r % 3 == 0) {
                    v = clamp_ordered(v, 0.f, kBig);
                    h = mu * v;
                } else {
                    v = clamp_ordered(v, -h, h);
                }
            } else {
                v = clamp_ordered(v, lo[r], hi[r]);
            }
            const float dl = v - xr;
            moved = fmaxf(moved, fabsf(dl * arr));
#pragma unroll
            for (int k = 0; k < KB; ++k)
                if (k * kWaveLanes < NR) wk[k] = fmaf(A[static_cast<size_t>(r) * R + k * kWaveLanes + lane], dl, wk[k]);
            if (lane == 0) S.xs[r] = v;   // read again in the next sweep (every lane holds v)
        }
        wave_lds_sync();
        if (moved <= tol) break;
    }
}

// One stage's box QP (bounds: row fields 5 / 6) over the whole system by
// wave_boxqp's primal active-set method (the same rules: several releases at
// once until a release blocks at zero length, frozen rows, refinement solves
// to the fp32 floor), from xs; budget linear solves.  Returns true when
// every row's complementarity residual is within tolerance.
__device__ __noinline__ bool sc_big_boxqp(ScBigWs G, int NR, int nb, int budget, ScBigLds S, int& solves) {
    const int lane = lane_id();
    const int R = G.R;
    const float* A = G.A();
    const float* b = G.row(1);
    const float* Ls = G.row(5);
    const float* Us = G.row(6);
    float* st = G.row(7);
    float* gg = G.row(8);
    float* tl = G.row(9);
    lds_float* xs = S.xs;
    auto set_st = [&](int r, int v) { st[r] = __int_as_float(v); };
    // working set from the start point (a row on a bound starts held there)
    {
        float xm = 0.f;
        for (int r = lane; r < NR; r += kWaveLanes) xm = fmaxf(xm, fabsf(xs[r]));
        const float t0 = 2e-6f * (1.f + wave_fmax(xm));
        for (int r = lane; r < 64 * nb; r += kWaveLanes) {
            int w = 1;
            if (r < NR) {
                const float L = Ls[r], U = Us[r];
                float x = fminf(fmaxf(xs[r], L), U);
                const bool pinned = U - L <= 0.f;
                w = pinned ? 1 : ((x <= L + t0) ? 1 : ((x >= U - t0) ? 2 : 0));
                x = (w == 1) ? L : ((w == 2) ? U : x);
                xs[r] = x;
            }
            set_st(r, w);
        }
    }
    wave_lds_sync();
    __threadfence_block();
    bool at_min = true;
    for (int r = lane; r < NR; r += kWaveLanes)
        if (sc_free(sc_st(st, r)) && Us[r] - Ls[r] > 0.f) at_min = false;
    at_min = __ballot(!at_min) == 0ull;
    bool stalled = false, fresh = false, single = false, factored = false;
    float rel = 0.f, xmax = 0.f, rel_refine = 3.4e38f;
    for (int it = 0; it < 4 * budget + 8 + NR; ++it) {
        if (!fresh) {
            float xm = 0.f;
            for (int r = lane; r < NR; r += kWaveLanes) xm = fmaxf(xm, fabsf(xs[r]));
            xmax = wave_fmax(xm);
            float e = 0.f;
            for (int r = lane; r < 64 * nb; r += kWaveLanes) {
                const bool live = r < NR;
                float mg = 0.f;
                const float w = live ? sc_big_dot(A, R, xs, r, NR, mg) : 0.f;
                const float br = live ? b[r] : 0.f;
                gg[r] = w - br;
                tl[r] = kLcpRelTol * (fabsf(br) + mg) + kLcpAbsTol;
                float ea;
                e = fmaxf(e, lcp_row_residual(live, br, live ? xs[r] : 0.f, w, mg,
                                              live ? A[static_cast<size_t>(r) * R + r] : 1.f, live ? Ls[r] : 0.f,
                                              live ? Us[r] : 0.f, 2e-6f * (1.f + xmax), ea));
            }
            rel = wave_fmax(e);
            __threadfence_block();
            if (rel <= 1.f) return true;
            fresh = true;
        }
        if (at_min) {
            at_min = false;
            // held rows whose multiplier is wrongly signed beyond tolerance leave
            float vmax = 0.f, vrow = 3.4e38f;
            for (int r = lane; r < NR; r += kWaveLanes) {
                const int s = sc_st(st, r);
                const bool pinned = Us[r] - Ls[r] <= 0.f;
                float v = ((s & 3) == 1) ? -gg[r] : (((s & 3) == 2) ? gg[r] : 0.f);
                v = (pinned || (s & 4)) ? 0.f : v * rcp(tl[r]);
                if (v > vmax) { vmax = v; vrow = static_cast<float>(r); }
            }
            const float vm = wave_fmax(vmax);
            if (vm > 1.f) {
                const float first = wave_fmin((vmax == vm) ? vrow : 3.4e38f);
                for (int r = lane; r < NR; r += kWaveLanes) {
                    int s = sc_st(st, r) & ~8;
                    const bool pinned = Us[r] - Ls[r] <= 0.f;
                    float v = ((s & 3) == 1) ? -gg[r] : (((s & 3) == 2) ? gg[r] : 0.f);
                    v = (pinned || (s & 4)) ? 0.f : v * rcp(tl[r]);
                    const bool rel_me = single ? (static_cast<float>(r) == first) : (v > 1.f);
                    if (rel_me) s = (s & ~3) | 8;
                    set_st(r, s);
                }
                __threadfence_block();
                factored = false;
                stalled = false;
                continue;
            }
            if (stalled || rel > 0.5f * rel_refine) return rel <= kLcpFloorAccept;
            rel_refine = rel;
        } else {
            rel_refine = 3.4e38f;
        }
        if (solves >= budget) return false;
        // ---- one linear solve over the free rows
        if (!factored) {
            sc_big_factor(G, NR, nb, S);
            factored = true;
        }
        for (int r = lane; r < 64 * nb; r += kWaveLanes) {
            const bool fr = r < NR && sc_free(sc_st(st, r)) && Us[r] - Ls[r] > 0.f;
            S.vs[r] = fr ? -gg[r] : 0.f;
        }
        wave_lds_sync();
        sc_big_solve(G, nb, S);
        ++solves;
        float dmax = 0.f, dres = 0.f;
        for (int r = lane; r < NR; r += kWaveLanes) {
            const bool fr = sc_free(sc_st(st, r)) && Us[r] - Ls[r] > 0.f;
            const float d = fr ? S.vs[r] : 0.f;
            dmax = fmaxf(dmax, fabsf(d));
            dres = fmaxf(dres, fabsf(d) * A[static_cast<size_t>(r) * R + r] * rcp(tl[r]));
        }
        dmax = wave_fmax(dmax);
        dres = wave_fmax(dres);
        if (dmax <= kLcpStall * (1.f + xmax) && dres <= 1.f) {
            // the release moved nothing: its rows back to their bounds, frozen
            bool any = false;
            for (int r = lane; r < NR; r += kWaveLanes) {
                int s = sc_st(st, r);
                if (s & 8) {
                    s = (s & ~(3 | 8)) | 4 | ((xs[r] <= Ls[r]) ? 1 : 2);
                    set_st(r, s);
                    any = true;
                }
            }
            if (__ballot(any)) factored = false;
            __threadfence_block();
            at_min = true;
            stalled = true;
            continue;
        }
        stalled = false;
        fresh = false;
        // the longest feasible step along d (at most 1) and the first row it blocks
        float amin_l = 1.f, arow = 3.4e38f;
        for (int r = lane; r < NR; r += kWaveLanes) {
            const bool fr = sc_free(sc_st(st, r)) && Us[r] - Ls[r] > 0.f;
            const float d = S.vs[r], x = xs[r];
            float al = 1.f;
            if (fr && d < 0.f && x + d < Ls[r]) al = (Ls[r] - x) * rcp(d);
            else if (fr && d > 0.f && x + d > Us[r]) al = (Us[r] - x) * rcp(d);
            al = fmaxf(al, 0.f);
            if (al < amin_l) { amin_l = al; arow = static_cast<float>(r); }
        }
        const float amin = wave_fmin(amin_l);
        int nrel = 0;   // released rows
        for (int k = 0; k < nb; ++k) {
            const int r = kWaveLanes * k + lane;
            nrel += __builtin_popcountll(__ballot(r < NR && (sc_st(st, r) & 8)));
        }
        wave_lds_sync();
        if (amin < 1.f) {
            const int block = static_cast<int>(wave_fmin((amin_l == amin) ? arow : 3.4e38f));
            bool back = false;
            const bool block_rel = (sc_st(st, block) & 8) != 0;   // uniform read
            if (amin <= 0.f && block_rel) {
                if (nrel > 1) {
                    single = true;
                } else {
                    back = true;   // the single released row blocks at once: frozen, back to the working set before
                }
            }
            for (int r = lane; r < NR; r += kWaveLanes) {
                int s = sc_st(st, r);
                const bool fr = sc_free(s) && Us[r] - Ls[r] > 0.f;
                const float d = S.vs[r];
                float x = xs[r];
                if (fr) x += amin * d;
                int side = 0;
                float al = 1.f;
                if (fr && d < 0.f && xs[r] + d < Ls[r]) { al = (Ls[r] - xs[r]) * rcp(d); side = 1; }
                else if (fr && d > 0.f && xs[r] + d > Us[r]) { al = (Us[r] - xs[r]) * rcp(d); side = 2; }
                al = fmaxf(al, 0.f);
                if (r == block) side = (side == 0) ? ((d < 0.f) ? 1 : 2) : side;
                // the blocking row, and on a zero-length step every row it blocks, join their bound
                if (r == block || (amin <= 0.f && fr && side != 0 && al <= 0.f)) {
                    x = (side == 1) ? Ls[r] : Us[r];
                    s = (s & ~3) | side;
                }
                if (back && (s & 8)) s |= 4;
                s &= ~8;
                xs[r] = x;
                set_st(r, s);
            }
            at_min = back;
        } else {
            for (int r = lane; r < NR; r += kWaveLanes) {
                const int s = sc_st(st, r);
                const bool fr = sc_free(s) && Us[r] - Ls[r] > 0.f;
                if (fr) xs[r] += S.vs[r];
                set_st(r, s & ~8);
            }
            at_min = true;
            single = false;
        }
        factored = factored && amin >= 1.f;
        wave_lds_sync();
        __threadfence_block();
    }
    return false;
}

struct ScBigOut {
    int nc, ovf, unconv;
};

// The constraint phase of a large-contact world-step (header above): rows,
// responses, Delassus, LCP, nu += MJ^T x and the contacts' impulses.  Joint
// rows of body `lane`: jbits (bit t: limit / servo / friction), their b / lo /
// hi, jbefore of them on lower lanes, tj in all.
template <int MAXNV>
__device__ __noinline__ ScBigOut sc_big_constraints(const SceneF* __restrict__ P, ScWorld<MAXNV>& L, ScBigWs G,
                                                    int nc_all, uint32_t jbits, float jb0, float jb1, float jb2,
                                                    float jlo0, float jlo1, float jlo2, float jhi0, float jhi1,
                                                    float jhi2, int jbefore, int tj, float dt, float mu,
                                                    int pgs_iters, int lcp_solves) {
    const int lane = lane_id();
    const int NV = P->nv, R = G.R;
    ScBigOut out{0, 0, 0};
    const int nc = nc_all < G.cmax ? nc_all : G.cmax;
    if (nc_all > G.cmax) out.ovf += nc_all - G.cmax;
    out.nc = nc;
    // the first kScMaxContacts points sit in the LDS record
    if (lane < nc && lane < kScMaxContacts)
        sc_big_put(G, lane, mk(L.c_p[lane][0], L.c_p[lane][1], L.c_p[lane][2]),
                   mk(L.c_n[lane][0], L.c_n[lane][1], L.c_n[lane][2]), L.c_d[lane], L.c_na[lane], L.c_nb[lane],
                   L.c_key[lane]);
    __threadfence_block();
    for (int c = lane; c < nc; c += kWaveLanes) {
        float* o = G.ct(c);
        f3 t1, t2;
        plane_space_f(mk(o[3], o[4], o[5]), t1, t2);
        o[6] = t1.x; o[7] = t1.y; o[8] = t1.z;
        o[9] = t2.x; o[10] = t2.y; o[11] = t2.z;
        o[16] = o[17] = o[18] = 0.f;
    }
    // ---- rows: contact c's rows 3 c + d, then the joint rows
    const int ncr = 3 * nc;
    int NR = ncr + tj;
    if (NR > R) {
        out.ovf += NR - R;
        NR = R;
    }
    float* rsrc = G.row(0);
    float* rb = G.row(1);
    float* rlo = G.row(2);
    float* rhi = G.row(3);
    float* rx1 = G.row(4);
    float* rL = G.row(5);
    float* rU = G.row(6);
    if (jbits) {
        int r = ncr + jbefore;
        const float jbv[3] = {jb0, jb1, jb2}, jlov[3] = {jlo0, jlo1, jlo2}, jhiv[3] = {jhi0, jhi1, jhi2};
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            if (((jbits >> t) & 1u) && r < NR) {
                rsrc[r] = __int_as_float(3 * lane + t);
                rb[r] = jbv[t];
                rlo[r] = jlov[t];
                rhi[r] = jhiv[t];
                ++r;
            }
        }
    }
    for (int r = lane; r < ncr && r < NR; r += kWaveLanes) {
        rlo[r] = 0.f;
        rhi[r] = kBig;
    }
    __threadfence_block();
    float* JT = G.JT();
    float* MJT = G.MJT();
    float* A = G.A();
    // ---- responses, 64 rows at a time through the LDS rows (lane = row)
    for (int r0 = 0; r0 < NR; r0 += kWaveLanes) {
        const int r = r0 + lane;
        float* Jr = L.J[lane];
        float* MJr = L.MJ[lane];
        for (int e = 0; e < MAXNV; ++e) { Jr[e] = 0.f; MJr[e] = 0.f; }
        if (r < NR) {
            if (r < ncr) {
                const int c = r / 3, d = r % 3;
                const float* o = G.ct(c);
                const f3 dw = mk(o[3 + 3 * d], o[4 + 3 * d], o[5 + 3 * d]);
                const f3 xp = mk(o[0], o[1], o[2]);
                float jv = 0.f;
#pragma unroll
                for (int side = 0; side < 2; ++side) {
                    const int k = __float_as_int(o[side ? 14 : 13]);
                    if (k >= 0) {
                        const ScNode& nd = L.node[k];
                        const f3 bpt = mulT(nd.Rw, xp - nd.pw);
                        const f3 dk = mulT(nd.Rw, dw);
                        const float sg = side ? -1.f : 1.f;
                        const SV f = {sg * cross(bpt, dk), sg * dk};
                        jv += sc_response<MAXNV>(P, L, k, -1, f, Jr, MJr);
                    }
                }
                const float bounce = (d == 0) ? fminf(kContactErp * o[12] * rcp(dt), kContactMaxErv) : 0.f;
                rb[r] = bounce - jv;
            } else {
                const int j = __float_as_int(rsrc[r]) / 3;
                (void)sc_response<MAXNV>(P, L, -1, j, SV{{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}}, Jr, MJr);
                for (int e = 0; e < MAXNV; ++e) Jr[e] = 0.f;
                Jr[P->body_coord[j]] = 1.f;
            }
            for (int e = 0; e < NV; ++e) {
                JT[static_cast<size_t>(e) * R + r] = Jr[e];
                MJT[static_cast<size_t>(e) * R + r] = MJr[e];
            }
        }
    }
    __threadfence_block();
    // ---- Delassus A = J MJ^T, block by block on the matrix cores (rows and
    // columns NR .. 64 nb zero)
    const int nblk = (NR + kWaveLanes - 1) / kWaveLanes;
    for (int bi = 0; bi < nblk; ++bi) {
        wave_lds_sync();
        {
            const int r = bi * kWaveLanes + lane;
            for (int e = 0; e < MAXNV; ++e)
                L.J[lane][e] = (r < NR && e < NV) ? JT[static_cast<size_t>(e) * R + r] : 0.f;
        }
        for (int bj = 0; bj < nblk; ++bj) {
            wave_lds_sync();
            {
                const int r = bj * kWaveLanes + lane;
                for (int e = 0; e < MAXNV; ++e)
                    L.MJ[lane][e] = (r < NR && e < NV) ? MJT[static_cast<size_t>(e) * R + r] : 0.f;
            }
            wave_lds_sync();
            float a[kWaveLanes];
            sc_tile64<MAXNV>(L, NV, a);
            const int gc = bj * kWaveLanes + lane;
#pragma unroll
            for (int i = 0; i < kWaveLanes; ++i) {
                const int gr = bi * kWaveLanes + i;
                float v = (gr < NR && gc < NR) ? a[i] : 0.f;
                if (gr == gc && gr < NR) v *= 1.f + ((gr >= ncr) ? kJointCfm : kContactCfm);
                A[static_cast<size_t>(gr) * R + gc] = v;
            }
        }
    }
    __threadfence_block();
    // ---- the LCP (scratch in the LDS union, dead since the responses)
    static_assert(sizeof(L.big) >= (kScBigRows + 64 * 64) * sizeof(float), "large-contact LCP scratch");
    static_assert(sizeof(L.J) + sizeof(L.MJ) >= 64 * 64 * sizeof(float) &&
                      offsetof(ScWorld<MAXNV>, MJ) == offsetof(ScWorld<MAXNV>, J) + sizeof(L.J),
                  "the T1 tile spans J and MJ");
    static_assert(offsetof(ScWorld<MAXNV>, rhi) + sizeof(L.rhi) - offsetof(ScWorld<MAXNV>, rc) ==
                      sizeof(L.rc) + sizeof(L.src) + sizeof(L.rb) + sizeof(L.rlo) + sizeof(L.rhi),
                  "the impulses span the contiguous row arrays");
    static_assert(sizeof(L.rc) + sizeof(L.src) + sizeof(L.rb) + sizeof(L.rlo) + sizeof(L.rhi) >= kScBigRows * sizeof(float),
                  "xs spans the compact row arrays");
    lds_float* base = (lds_float*)L.big;
    const ScBigLds S{(lds_float*)&L.rc[0], base, base + kScBigRows, (lds_float*)&L.J[0][0]};
    for (int r = lane; r < kWaveLanes * nblk; r += kWaveLanes) S.xs[r] = 0.f;
    wave_lds_sync();
    bool ok = true;
    if (lcp_solves > 0) {
        for (int s = 1; s <= 2; ++s) {
            int solves = 0;
            // the stage's boxes: stage 1 friction pinned at 0; stage 2 friction
            // boxed by mu x_n of the contact's stage-1 normal
            for (int r = lane; r < NR; r += kWaveLanes) {
                float lo = rlo[r], hi = rhi[r];
                if (r < ncr && r % 3 != 0) {
                    hi = (s == 1) ? 0.f : mu * fmaxf(rx1[r - r % 3], 0.f);
                    lo = -hi;
                }
                rL[r] = lo;
                rU[r] = hi;
                S.xs[r] = fminf(fmaxf(S.xs[r], lo), hi);
            }
            wave_lds_sync();
            __threadfence_block();
            // (a cold start: more sweeps than the compact path's, and a budget
            // that grows with the rows -- fp64 emulation on rows of eight
            // cubes: 6 sweeps then 10-54 solves in stage 2, 24 sweeps then 5-28)
            sc_big_pgs(G, NR, ncr, mu, kScBigSweeps, false, kScExactPgsTol, S);
            ok = sc_big_boxqp(G, NR, nblk, lcp_solves + NR / 2, S, solves) && ok;
            wave_lds_sync();
            if (s == 1) {
                for (int r = lane; r < NR; r += kWaveLanes) rx1[r] = S.xs[r];
                __threadfence_block();
            }
        }
    } else {
        sc_big_pgs(G, NR, ncr, mu, pgs_iters, true, -1.f, S);
    }
    if (!ok) out.unconv = 1;
    // ---- nu += MJ^T x (lane = coordinate); the contacts' impulses
    if (lane < NV) {
        float dnu = 0.f;
        for (int r = 0; r < NR; ++r) dnu = fmaf(MJT[static_cast<size_t>(lane) * R + r], S.xs[r], dnu);
        L.nu[lane] += dnu;
    }
    for (int r = lane; r < ncr && r < NR; r += kWaveLanes) G.ct(r / 3)[16 + r % 3] = S.xs[r];
    __threadfence_block();
    wave_lds_sync();
    return out;
}

// ------------------------------------------------------------------- step
// (a real call, not inlined: __forceinline__ took scratch 944 -> 768 B per
// lane but the scene leg 0.909 -> 0.976 ms, profiles/r05ag)
template <int MAXNV>
__device__ void sc_step(const SceneF* __restrict__ P, ScWorld<MAXNV>& L, FreeState& base, uint32_t present,
                        const float (&wr)[kScWrenchSlots][6], const int32_t (&wl)[kScWrenchSlots], int iter,
                        float dt, int pgs_iters, int lcp_solves, const ScWarm& warm, const f3 gw, float mu,
                        ScBigWs big, int& nc_out, bool& big_out, int& ovf, int& unconv) {
    const int lane = lane_id();
    MW_PROF_T(t_in);
#ifdef MW_SC_NANCHECK
    bool nan_reported = false;
    MW_SC_CHECK(0, 0);
#endif
    const int NB = P->n_bodies, NV = P->nv;
    const bool isnode = lane < P->n_nodes;
    const int nbody = isnode ? P->node_body[lane] : -1;
    const bool isbase = isnode && nbody < 0;
    const bool isbody = isnode && nbody >= 0;
    const int bi = isbody ? nbody : 0;
    const int m = isnode ? P->node_model[lane] : 0;
    const bool alive = isnode && ((present >> m) & 1u);
    const SceneModelF& md = P->model[m];
    const BodyF b = P->b[bi];
    const int depth = alive ? P->node_depth[lane] : -1;
    const int srank = P->node_srank[lane];
    const int pnode = isbody ? (b.parent >= 0 ? P->body_node[b.parent] : md.node0) : 0;
    const int levels = P->levels, fanout = P->fanout;
    const bool dual = P->dual != 0;
    // external wrench of this node at this iteration (world force at the
    // origin, world torque), summed over the active records
    f3 Fw = {0.f, 0.f, 0.f}, Tw = {0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < kScWrenchSlots; ++k)
        if (wl[k] >= iter) {
            Fw = Fw + mk(wr[k][0], wr[k][1], wr[k][2]);
            Tw = Tw + mk(wr[k][3], wr[k][4], wr[k][5]);
        }
    if (lane < kScMaxNodes) L.acc[lane] = WaveAcc{};
    M3 R, Rw;
    f3 p, pw;
    SV V, eta, B;
    const M3 Rb0 = md.floating ? quat_to_R(base.qw, base.qx, base.qy, base.qz)
                               : M3{{md.R0[0], md.R0[1], md.R0[2], md.R0[3], md.R0[4], md.R0[5], md.R0[6], md.R0[7], md.R0[8]}};
    // ---- outward: kinematics, velocities, bias forces
    for (int d = 0; d < levels; ++d) {
        if (depth == d) {
            if (isbase) {
                Rw = Rb0;
                pw = md.floating ? base.p : mk(md.p0[0], md.p0[1], md.p0[2]);
                V = md.floating ? base.V : SV{{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
                B = rigid_bias(md.mass, mk(md.com[0], md.com[1], md.com[2]),
                               Sy{md.Io[0], md.Io[1], md.Io[2], md.Io[3], md.Io[4], md.Io[5]}, V, mulT(Rw, gw));
                R = Rw;
                p = pw;
                eta = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
            } else {
                joint_pose_tree(b, L.q, bi, R, p);
                const SV Sq = motion(b, L.qd[bi]);
                const ScNode& pn = L.node[pnode];
                V = ad_inv(R, p, pn.V) + Sq;
                Rw = mul3(pn.Rw, R);
                pw = pn.pw + mul(pn.Rw, p);
                const SV Ve = ball_bias_velocity(b, L.qd, bi, V);
                eta = {cross(Ve.w, Sq.w), cross(Ve.w, Sq.v) + cross(Ve.v, Sq.w)};
                B = rigid_bias(b.mass, mk(b.com[0], b.com[1], b.com[2]), inertia_origin(b, b.mass), V, mulT(Rw, gw));
            }
            B = B + (-1.f) * SV{mulT(Rw, Tw), mulT(Rw, Fw)};
            L.node[lane].V = V;
            L.node[lane].Rw = Rw;
            L.node[lane].pw = pw;
        }
    }
    float tau = 0.f, qdi = 0.f;
    if (isbody && alive) { tau = L.tau[bi]; qdi = L.qd[bi]; }
    MW_SC_CHECK(1, 0);
    // ---- inward, deepest level first
    SV U = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}}, Un = U;
    float psi = 0.f, tt = 0.f, psin = 0.f;
    for (int d = levels - 1; d >= 1; --d) {
        const bool mine = (depth == d);
        SI c, cn;
        SV cb;
        if (mine) {
            SI AI = rigid(b, b.mass);
            AI += L.acc[lane].I;
            const SV Bt = B + L.acc[lane].B;
            U = ais(AI, b);
            psi = rcp(proj(b, U) + dt * b.damping);
            const SV AIeta = mul(AI, eta);
            tt = tau - b.damping * qdi - proj(b, AIeta + Bt);
            c = to_parent(R, p, downdate(AI, U, psi));
            cb = dad_inv(R, p, Bt + AIeta + (psi * tt) * U);
            if (dual) {
                SI AIn = rigid(b, b.mass);
                AIn += L.acc[lane].In;
                Un = ais(AIn, b);
                psin = rcp(proj(b, Un));
                cn = to_parent(R, p, downdate(AIn, Un, psin));
            }
        }
        // the level's own fan-out (sibling ranks are contiguous from 0; as wave_aba)
        for (int k = 0; k < fanout; ++k) {
            const bool me = mine && srank == k;
            if (__ballot(me) == 0ull) break;
            if (me) {
                WaveAcc& acc = L.acc[pnode];
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
    // ---- floating bases: a0 = -IA0^-1 B0 on the base's own lane
    SV a0 = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
    if (isbase && alive && md.floating) {
        SI IA0;
        IA0.A = {md.Io[0], md.Io[1], md.Io[2], md.Io[3], md.Io[4], md.Io[5]};
        const float mm = md.mass, cx = md.com[0], cy = md.com[1], cz = md.com[2];
        IA0.B.m[0] = 0.f;      IA0.B.m[1] = -mm * cz; IA0.B.m[2] = mm * cy;
        IA0.B.m[3] = mm * cz;  IA0.B.m[4] = 0.f;      IA0.B.m[5] = -mm * cx;
        IA0.B.m[6] = -mm * cy; IA0.B.m[7] = mm * cx;  IA0.B.m[8] = 0.f;
        IA0.C = {mm, mm, mm, 0.f, 0.f, 0.f};
        SI IAn = IA0;
        IA0 += L.acc[lane].I;
        Chol6 L0;
        L0.factor(IA0);
        a0 = L0.solve(-1.f * (B + L.acc[lane].B));
        if (dual) {
            IAn += L.acc[lane].In;
            L0.factor(IAn);
        }
#pragma unroll
        for (int e = 0; e < 21; ++e) L.l0[m][e] = L0.l[e];
#pragma unroll
        for (int e = 0; e < 6; ++e) L.l0[m][21 + e] = L0.id[e];
    }
    if (isbase && alive) L.node[lane].V = a0;  // the V record now carries a
    MW_SC_CHECK(2, 0);
    // ---- outward: accelerations
    float qddi = 0.f;
    for (int d = 1; d < levels; ++d) {
        if (depth == d) {
            const SV ap = ad_inv(R, p, L.node[pnode].V);
            qddi = psi * (tt - dot(U, ap));
            L.node[lane].V = ap + eta + motion(b, qddi);
        }
    }
    if (alive) {
        ScNode& s = L.node[lane];
        s.R = R;
        s.p = p;
        s.U = {{dual ? Un.w.x : U.w.x, dual ? Un.w.y : U.w.y, dual ? Un.w.z : U.w.z},
               {dual ? Un.v.x : U.v.x, dual ? Un.v.y : U.v.y, dual ? Un.v.z : U.v.z}};
        s.psi = dual ? psin : psi;
        s.tt = tt;
        s.depth = depth;
    }
    // ---- integrateVelocities
    if (isbody && alive) {
        L.qdd[bi] = qddi;
        L.nu[P->body_coord[bi]] = qdi + dt * qddi;
    }
    if (isbase && alive && md.floating) {
        const float a[6] = {a0.w.x, a0.w.y, a0.w.z, a0.v.x, a0.v.y, a0.v.z};
        const float v0[6] = {base.V.w.x, base.V.w.y, base.V.w.z, base.V.v.x, base.V.v.y, base.V.v.z};
#pragma unroll
        for (int e = 0; e < 6; ++e) L.nu[md.coff + e] = v0[e] + dt * a[e];
    }

    MW_SC_CHECK(3, 0);
    MW_PROF_T(t_aba);
    // ---- contacts: ground slots, then shape pairs
    int nc = 0;
    if (P->ground && (present & kScGroundBit)) {
        for (int s0 = 0; s0 < P->n_slots; s0 += kWaveLanes) {
            const int slot = s0 + lane;
            bool hit = false;
            f3 xw = {0.f, 0.f, 0.f};
            float dep = 0.f;
            int na = 0;
            if (slot < P->n_slots) {
                const int sh = P->slot_shape[slot];
                const int mo = P->shape_model[sh];
                if ((present >> mo) & 1u) {
                    const int c = slot - P->shape_slot0[sh];
                    na = P->shape_node[sh];
                    const ScNode& nd = L.node[na];
                    const bool sphere = (P->shape_type[sh] == 1);
                    const float* h = P->shape_size[sh];
                    const float* SR = P->shape_R[sh];
                    const f3 lp = (P->shape_type[sh] == 3)
                                      ? mk(P->slot_pt[slot][0], P->slot_pt[slot][1], P->slot_pt[slot][2])
                                      : shape_slot_point(P->shape_type[sh], h, shape_plane_normal(nd.Rw, SR), c);
                    const float lx = lp.x, ly = lp.y, lz = lp.z;
                    const f3 bb = {P->shape_p[sh][0] + SR[0] * lx + SR[1] * ly + SR[2] * lz,
                                   P->shape_p[sh][1] + SR[3] * lx + SR[4] * ly + SR[5] * lz,
                                   P->shape_p[sh][2] + SR[6] * lx + SR[7] * ly + SR[8] * lz};
                    xw = nd.pw + mul(nd.Rw, bb);
                    dep = -xw.z;
                    if (sphere) {
                        dep = h[0] - xw.z;
                        xw.z -= h[0];
                    }
                    hit = dep > 0.f;
                }
            }
            const uint64_t bal = __ballot(hit);
            const int rank = __popcll(bal & ((uint64_t{1} << lane) - 1u));
            if (hit && nc + rank < kScMaxContacts) {
                const int c = nc + rank;
                L.c_p[c][0] = xw.x; L.c_p[c][1] = xw.y; L.c_p[c][2] = xw.z;
                L.c_n[c][0] = 0.f; L.c_n[c][1] = 0.f; L.c_n[c][2] = 1.f;
                L.c_d[c] = dep;
                L.c_na[c] = na;
                L.c_nb[c] = -1;
                L.c_key[c] = slot;
            } else if (hit && big.base && nc + rank < big.cmax) {
                sc_big_put(big, nc + rank, xw, mk(0.f, 0.f, 1.f), dep, na, -1, slot);
            }
            nc += __popcll(bal);
        }
    }
    MW_PROF_T(t_gnd);
#ifdef MW_WAVE_PROF
    long long t_np = t_gnd;
#endif
    for (int p0 = 0; p0 < P->n_pairs; p0 += kScClipLanes) {
        const int pr = (lane < kScClipLanes) ? p0 + lane : P->n_pairs;
        int np = 0;
        f3 nrm = {0.f, 0.f, 1.f};
        float* ws = &L.clip[0][lane & (kScClipLanes - 1)];
        const ScWsPts out{ws + kScWsOut * kScClipLanes};
        int na = 0, nb = 0;
        if (pr < P->n_pairs) {
            const int sa = P->pair_a[pr], sb = P->pair_b[pr];
            if (((present >> P->shape_model[sa]) & 1u) && ((present >> P->shape_model[sb]) & 1u)) {
                na = P->shape_node[sa];
                nb = P->shape_node[sb];
                const ScNode& A_ = L.node[na];
                const ScNode& B_ = L.node[nb];
                const M3 SRa = {{P->shape_R[sa][0], P->shape_R[sa][1], P->shape_R[sa][2], P->shape_R[sa][3],
                                 P->shape_R[sa][4], P->shape_R[sa][5], P->shape_R[sa][6], P->shape_R[sa][7],
                                 P->shape_R[sa][8]}};
                const M3 SRb = {{P->shape_R[sb][0], P->shape_R[sb][1], P->shape_R[sb][2], P->shape_R[sb][3],
                                 P->shape_R[sb][4], P->shape_R[sb][5], P->shape_R[sb][6], P->shape_R[sb][7],
                                 P->shape_R[sb][8]}};
                const f3 ca = A_.pw + mul(A_.Rw, mk(P->shape_p[sa][0], P->shape_p[sa][1], P->shape_p[sa][2]));
                const f3 cb = B_.pw + mul(B_.Rw, mk(P->shape_p[sb][0], P->shape_p[sb][1], P->shape_p[sb][2]));
                // a mesh with a hull against a box or such a mesh: the hull narrow
                // phase; a box-shaped or flat mesh, and a mesh against a sphere or
                // a cylinder, collide as the mesh's bounding box (type 3 -> 0)
                const int ha = P->shape_type[sa] == 3 ? P->shape_hull[sa] : -1;
                const int hb = P->shape_type[sb] == 3 ? P->shape_hull[sb] : -1;
                const int ta = P->shape_type[sa] == 3 ? 0 : P->shape_type[sa];
                const int tb = P->shape_type[sb] == 3 ? 0 : P->shape_type[sb];
                const f3 za = mk(P->shape_size[sa][0], P->shape_size[sa][1], P->shape_size[sa][2]);
                const f3 zb = mk(P->shape_size[sb][0], P->shape_size[sb][1], P->shape_size[sb][2]);
                if ((ha >= 0 || hb >= 0) && ta == 0 && tb == 0) {
                    const ScPoly pa = ha >= 0 ? ScPoly{&P->hull[ha], mk(1.f, 1.f, 1.f), false}
                                              : ScPoly{&P->box_hull, za, true};
                    const ScPoly pb = hb >= 0 ? ScPoly{&P->hull[hb], mk(1.f, 1.f, 1.f), false}
                                              : ScPoly{&P->box_hull, zb, true};
                    np = sc_hull_pair(pa, ca, mul3(A_.Rw, SRa), pb, cb, mul3(B_.Rw, SRb), nrm, out);
                } else {
                    np = sc_collide(ta, za, ca, mul3(A_.Rw, SRa), tb, zb, cb, mul3(B_.Rw, SRb), nrm, ws);
                }
            }
        }
#ifdef MW_WAVE_PROF
        if (p0 == 0) t_np = clock64();
#endif
        int total = 0;
        const int pre = wave_prefix7(np, total);
        for (int i = 0; i < np; ++i) {
            const int c = nc + pre + i;
            if (c < kScMaxContacts) {
                const f3 x = out.pt(i);
                L.c_p[c][0] = x.x; L.c_p[c][1] = x.y; L.c_p[c][2] = x.z;
                L.c_n[c][0] = nrm.x; L.c_n[c][1] = nrm.y; L.c_n[c][2] = nrm.z;
                L.c_d[c] = out.dep(i);
                L.c_na[c] = na;
                L.c_nb[c] = nb;
                L.c_key[c] = P->n_slots + 4 * pr + i;
            } else if (big.base && c < big.cmax) {
                sc_big_put(big, c, out.pt(i), nrm, out.dep(i), na, nb, P->n_slots + 4 * pr + i);
            }
        }
        nc += total;
    }
    // more points than the LDS record: the large-contact path when the scene
    // has its workspace, else the excess is dropped (counted)
    const int nc_all = nc;
    if (nc > kScMaxContacts) {
        if (!big.base) ovf += nc - kScMaxContacts;
        nc = kScMaxContacts;
    }
    if (lane < nc) {
        const f3 n = mk(L.c_n[lane][0], L.c_n[lane][1], L.c_n[lane][2]);
        (void)n;
        L.c_x[lane][0] = L.c_x[lane][1] = L.c_x[lane][2] = 0.f;
    }

    MW_PROF_T(t_pairs);
    MW_SC_CHECK(4, nc);
    // ---- joint rows of body `lane` (bit t: limit / servo / friction)
    uint32_t jbits = 0u;
    float jb[3] = {0.f, 0.f, 0.f}, jlo[3] = {0.f, 0.f, 0.f}, jhi[3] = {0.f, 0.f, 0.f};
    const bool jlane = lane < NB && ((present >> P->body_model[lane < NB ? lane : 0]) & 1u);
    if (jlane) {
        const BodyF& bj = P->b[lane];
        const float qv = L.nu[P->body_coord[lane]];
        if (bj.limited) {
            float viol = L.q[lane] - bj.lower;
            bool lim = false, up = false;
            if (viol <= 0.f) {
                lim = true;
            } else {
                viol = L.q[lane] - bj.upper;
                if (viol >= 0.f) { lim = true; up = true; }
            }
            if (lim) {
                jbits |= 1u;
                jb[0] = fminf(fmaxf(-viol * kErp * rcp(dt), -kMaxErv), kMaxErv) - qv;
                jlo[0] = up ? -kBig : 0.f;
                jhi[0] = up ? 0.f : kBig;
            }
        }
        if (L.act[lane] == kActServo) {
            const float vcv = fminf(fmaxf(L.vc[lane], -bj.vel_limit), bj.vel_limit);
            if (vcv - qv != 0.f) {
                jbits |= 2u;
                jb[1] = vcv - qv;
                jhi[1] = bj.effort * dt;
                jlo[1] = -jhi[1];
            }
        }
        if (bj.friction != 0.f && qv != 0.f) {
            jbits |= 4u;
            jb[2] = -qv;
            jhi[2] = bj.friction * dt;
            jlo[2] = -jhi[2];
        }
    }
    int tj = 0;
    const int jbefore = wave_prefix7(__builtin_popcount(jbits), tj);
    const bool use_big = big.base != nullptr && (nc_all > kScMaxContacts || 3 * nc_all + tj > kWaveLanes);
    big_out = use_big;
    const int ncr = 3 * nc;
    int NR = use_big ? 0 : ncr + tj;   // a large-contact step skips the compact constraint phase
    if (NR > kScMaxRows) {
        ovf += NR - kScMaxRows;
        NR = kScMaxRows;
    }
    if (lane < nc && !use_big) {
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            L.src[3 * lane + d] = 3 * lane + d;
            L.rlo[3 * lane + d] = 0.f;
            L.rhi[3 * lane + d] = kBig;
        }
    }
    if (jlane && !use_big) {
        int r = ncr + jbefore;
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            if (((jbits >> t) & 1u) && r < NR) {
                L.src[r] = kJointRow + 3 * lane + t;
                L.rb[r] = jb[t];
                L.rlo[r] = jlo[t];
                L.rhi[r] = jhi[t];
                ++r;
            }
        }
    }

    float x1s = 0.f;  // the exact solve's stage-1 impulse of row `lane` (warm record)
    float x0 = 0.f;   // the impulse of row `lane`
    MW_PROF_T(t_rows);
#ifdef MW_WAVE_PROF
    long long t_resp = t_rows, t_del = t_rows, t_lcp = t_rows;
#endif
    if (use_big) {
        const ScBigOut bo = sc_big_constraints<MAXNV>(P, L, big, nc_all, jbits, jb[0], jb[1], jb[2], jlo[0], jlo[1],
                                                      jlo[2], jhi[0], jhi[1], jhi[2], jbefore, tj, dt, mu, pgs_iters,
                                                      lcp_solves);
        nc = bo.nc;
        ovf += bo.ovf;
        unconv += bo.unconv;
    }
    if (NR > 0) {
        // ---- responses, lane = row
        for (int r0 = 0; r0 < NR; r0 += kWaveLanes) {
            const int r = r0 + lane;
            if (r < NR) {
                float* Jr = L.J[r];
                float* MJr = L.MJ[r];
                for (int e = 0; e < MAXNV; ++e) { Jr[e] = 0.f; MJr[e] = 0.f; }
                const int src = L.src[r];
                if (src < kJointRow) {
                    const int c = src / 3, d = src % 3;
                    const f3 cn = mk(L.c_n[c][0], L.c_n[c][1], L.c_n[c][2]);
                    f3 ct1, ct2;
                    plane_space_f(cn, ct1, ct2);
                    const f3 dw = d == 0 ? cn : (d == 1 ? ct1 : ct2);
                    const f3 xp = mk(L.c_p[c][0], L.c_p[c][1], L.c_p[c][2]);
                    float jv = 0.f;
#pragma unroll
                    for (int side = 0; side < 2; ++side) {
                        const int k = side ? L.c_nb[c] : L.c_na[c];
                        if (k >= 0) {
                            const ScNode& nd = L.node[k];
                            const f3 bpt = mulT(nd.Rw, xp - nd.pw);
                            const f3 dk = mulT(nd.Rw, dw);
                            const float sg = side ? -1.f : 1.f;
                            const SV f = {sg * cross(bpt, dk), sg * dk};
                            jv += sc_response<MAXNV>(P, L, k, -1, f, Jr, MJr);
                        }
                    }
                    const float bounce = (d == 0) ? fminf(kContactErp * L.c_d[c] * rcp(dt), kContactMaxErv) : 0.f;
                    L.rb[r] = bounce - jv;
                } else {
                    const int j = (src - kJointRow) / 3;
                    (void)sc_response<MAXNV>(P, L, -1, j, SV{{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}}, Jr, MJr);
                    for (int e = 0; e < MAXNV; ++e) Jr[e] = 0.f;
                    Jr[P->body_coord[j]] = 1.f;
                }
            }
        }
#ifdef MW_WAVE_PROF
        t_resp = clock64();
#endif
        // ---- Delassus A = J MJ^T.  Up to 64 rows: on the matrix cores
        // (wave_tree.hpp's tiles, v_mfma_f32_32x32x2_f32: in k-step k lane l
        // supplies J[m0 + l%32][2k + l/32] and MJ[n0 + l%32][2k + l/32]; the
        // 32x32 result holds column n0 + l%32 in lane l, rows 8(i/4) + 4(l/32)
        // + i%4 in accumulator i; one exchange of the 32-lane halves gives
        // lane c all of column c = row c), straight into the registers the
        // PGS and the exact solve keep it in.  Columns >= NV of J and MJ are
        // zero (the response pass clears them); rows / columns >= NR are
        // masked.  (The lane = column FMA loop over LDS took 21.8k cycles per
        float a[kWaveLanes];
        {
            const int lr = lane & 31, lh = lane >> 5;
            const bool hi2 = NR > 32;
            v16f t00 = {}, t01 = {}, t10 = {}, t11 = {};
            constexpr int kKs = MAXNV / 2;
#pragma unroll
            for (int k0 = 0; k0 < kKs; k0 += 4) {
                if (2 * k0 >= NV) break;
                float jv0[4], mv0[4], jv1[4], mv1[4];
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    const int e = 2 * (k0 + kk) + lh;
                    jv0[kk] = L.J[lr][e];
                    mv0[kk] = L.MJ[lr][e];
                    jv1[kk] = hi2 ? L.J[32 + lr][e] : 0.f;
                    mv1[kk] = hi2 ? L.MJ[32 + lr][e] : 0.f;
                }
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    t00 = __builtin_amdgcn_mfma_f32_32x32x2f32(jv0[kk], mv0[kk], t00, 0, 0, 0);
                    if (hi2) {
                        t01 = __builtin_amdgcn_mfma_f32_32x32x2f32(jv0[kk], mv1[kk], t01, 0, 0, 0);
                        t10 = __builtin_amdgcn_mfma_f32_32x32x2f32(jv1[kk], mv0[kk], t10, 0, 0, 0);
                        t11 = __builtin_amdgcn_mfma_f32_32x32x2f32(jv1[kk], mv1[kk], t11, 0, 0, 0);
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) {
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
            for (int r = 0; r < kWaveLanes; ++r) {
                a[r] = (r < NR && lane < NR) ? a[r] : 0.f;
                if (lane == r && r < NR) {
                    a[r] *= 1.f + ((r >= ncr) ? kJointCfm : kContactCfm);
                    dg = a[r];
                }
            }
            if (lane < NR) L.rc[lane] = F4{L.rb[lane], rcp(dg), L.rlo[lane], L.rhi[lane]};
        }
        // ---- PGS (rows in order)
        {
            // up to 64 rows: the register form of wave_tree.hpp -- lane c holds
            // column c of A (= row c) in registers, the impulses are uniform
            // registers, the residual w_c = sum_r A[c][r] x_r is rebuilt per
            // sweep and updated by one column per row; rows padded to blocks
            // of 8 with inert rows (zero column, b = 0, bounds [0, 0])
            const int Rpad = (NR + 7) & ~7;
            if (lane >= NR && lane < Rpad) L.rc[lane] = F4{0.f, 0.f, 0.f, 0.f};
            // warm start (exact mode): every row from the previous step's
            // impulse of the same contact key / joint row, else 0
            float xw = 0.f, xw1 = 0.f;  // final and stage-1 impulses of the previous step
            if (warm.rec) {
                // the previous record's keys one per lane (one load, not a
                // search loop of dependent loads per row), matched by lane reads
                const int np = warm.n();
                const int pk = (lane < np) ? warm.key(lane) : -1;
                const int src = L.src[lane < NR ? lane : 0];
                const bool crow = lane < NR && src < kJointRow;
                const int key = crow ? L.c_key[src / 3] : -2;
                int idx = -1;
                for (int j = 0; j < np; ++j) {
                    const int kj = __builtin_amdgcn_readlane(pk, j);
                    idx = (idx < 0 && kj == key) ? j : idx;
                }
                const int wi = (crow && idx >= 0) ? 3 * idx + src % 3
                                                  : ((lane < NR && !crow) ? kScWarmJoint0 + (src - kJointRow) : -1);
                if (wi >= 0) {
                    xw = warm.x(wi);
                    xw1 = warm.x1(wi);
                }
            }
            float x[kWaveLanes];
#pragma unroll
            for (int r = 0; r < kWaveLanes; ++r) x[r] = read_lane(xw, r);
            // exact mode: no coupled sweeps -- each stage of the exact solve
            // runs its own (wave_lcp.hpp), as on the world-per-wavefront kernel
            for (int it = 0; it < (lcp_solves > 0 ? 0 : pgs_iters); ++it) {
                float w = 0.f;
#pragma unroll
                for (int rb = 0; rb < kWaveLanes; rb += 8) {
                    if (rb >= Rpad) break;
#pragma unroll
                    for (int k = 0; k < 8; ++k) w += a[rb + k] * x[rb + k];
                }
                const float w_start = w;
                float h = 0.f;
#pragma unroll
                for (int rb = 0; rb < kWaveLanes; rb += 8) {
                    if (rb >= Rpad) break;
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const int r = rb + k;
                        const F4 c = L.rc[r];
                        const float xb = fmaf(c.x, c.y, x[r]);
                        const float wpre = fmaf(-a[r], x[r], w);
                        float v = fmaf(-read_lane(w, r), c.y, xb);
                        if (r % 3 == 0) {
                            v = clamp_ordered(v, c.z, c.w);  // normal row [0, inf) or joint row
                            h = mu * v;
                        } else {
                            const bool fr = r < ncr;      // friction |x| <= mu x_normal, or joint row
                            v = clamp_ordered(v, fr ? -h : c.z, fr ? h : c.w);
                        }
                        w = fmaf(a[r], v, wpre);
                        x[r] = v;
                    }
                }
                if (lcp_solves > 0 && wave_fmax(fabsf(w - w_start)) <= kScExactPgsTol) break;
            }
#pragma unroll
            for (int r = 0; r < kWaveLanes; ++r) x0 = (lane == r) ? x[r] : x0;
            if (lcp_solves > 0) {
                // exact boxed LCP (wave_lcp.hpp; oracle OR_PGS_CONVERGED), lane
                // r = row r, each stage from the previous step's record of that
                // stage; the pivot rows go to the Delassus matrix's LDS, dead
                // once it sits in the registers; the stages' sweeps use L.rc
                LcpRow Rw;
                Rw.live = lane < NR;
                const F4 c = L.rc[lane < Rpad ? lane : 0];
                Rw.kind = (lane < ncr) ? ((lane % 3 == 0) ? 0 : 1) : 2;
                Rw.nrow = (Rw.kind == 1) ? lane - lane % 3 : lane;
                Rw.b = Rw.live ? c.x : 0.f;
                Rw.lo = Rw.live ? c.z : 0.f;
                Rw.hi = Rw.live ? c.w : 0.f;
                float* Uw = L.lcp;
                int nsolve = 0, nround = 0, nsolve1 = 0;
                long long cyc[3] = {0, 0, 0};
                x1s = xw1;
                // long-row elimination (wave_lcp.hpp lcp_ge_solve)
#ifdef MW_WAVE_PROF
                const long long t_ex0 = clock64();
#endif
                // (sweeps skipped when every contact has a warm record: 0.730 ->
                // 0.665 ms, but a resting cube then drifts by 1.7e-4 m/s,
                // test_gpu_scenario_scene.py::test_cube_contact: kept)
                const int sweeps = pgs_iters;
                const bool ok = (NR <= 32) ? wave_lcp_exact<32, true, kScStageSweeps, kLcpMfmaAll>(a, Rw, mu, NR, lcp_solves, sweeps,
                                                                      kScExactPgsTol, L.rc, Uw, x1s, x0, nsolve,
                                                                      nround, nsolve1, cyc)
                                           : wave_lcp_exact<kWaveMaxRows, true, kScStageSweeps, kLcpMfmaAll>(a, Rw, mu, NR, lcp_solves, sweeps,
                                                                                kScExactPgsTol, L.rc, Uw, x1s, x0,
                                                                                nsolve, nround, nsolve1, cyc);
                if (!ok && lane == 0) unconv += 1;
#ifdef MW_WAVE_PROF
                if (lane == 0) atomicAdd(&g_wave_prof[12], static_cast<unsigned long long>(clock64() - t_ex0));
                // debug dump of up to kDumpSlots hard LCPs (>= 8 solves, or
                // the unconverged ones with -DMW_DUMP_FAIL): n, A, b, lo, hi,
                // the two warm records, the result, kind, the stage-1 result
                if (MW_DUMP_WHEN(ok, nsolve) && NR <= kWaveLanes) {
                    unsigned int claim = 0u;
                    if (lane == 0) claim = atomicAdd(&g_sc_dump_claim, 1u);
                    claim = __builtin_amdgcn_readfirstlane(claim);
                    if (claim < static_cast<unsigned int>(kDumpSlots)) {
                        float* D0 = g_sc_dump + claim * kScDumpFloats;
                        for (int r = 0; r < NR; ++r) D0[8 + r * kWaveLanes + lane] = (lane < NR) ? a[r] : 0.f;
                        float* V = D0 + 8 + kWaveLanes * kWaveLanes;
                        if (lane < NR) {
                            V[lane] = Rw.b;
                            V[kWaveLanes + lane] = Rw.lo;
                            V[2 * kWaveLanes + lane] = Rw.hi;
                            V[3 * kWaveLanes + lane] = xw;
                            V[4 * kWaveLanes + lane] = xw1;
                            V[5 * kWaveLanes + lane] = x0;
                            V[6 * kWaveLanes + lane] = static_cast<float>(Rw.kind);
                            V[7 * kWaveLanes + lane] = x1s;
                        }
                        if (lane == 0) {
                            D0[0] = static_cast<float>(NR);
                            D0[1] = static_cast<float>(nsolve);
                            D0[2] = static_cast<float>(nsolve1);
                            D0[3] = mu;
                            D0[4] = ok ? 1.f : 0.f;
                        }
                    }
                }
                if (lane == 0) {
                    atomicAdd(&g_wave_prof[8], static_cast<unsigned long long>(nsolve));
                    atomicAdd(&g_wave_prof[9], static_cast<unsigned long long>(nround));
                    atomicAdd(&g_wave_prof[10], static_cast<unsigned long long>(nsolve1));
                    atomicMax(&g_wave_prof[11], static_cast<unsigned long long>(nsolve));
                    atomicAdd(&g_wave_prof[13], nsolve > 4 ? 1ull : 0ull);
                    atomicAdd(&g_wave_prof[14], static_cast<unsigned long long>(cyc[0]));
                    atomicAdd(&g_wave_prof[15], ok ? 0ull : 1ull);
                    atomicAdd(&g_wave_prof[16], static_cast<unsigned long long>(cyc[1]));
                    atomicAdd(&g_wave_prof[17], static_cast<unsigned long long>(cyc[2]));
                    atomicAdd(&g_wave_prof[18], 1ull);
                }
#endif
                x0 = Rw.live ? x0 : 0.f;
            }
        }
#ifdef MW_WAVE_PROF
        t_lcp = clock64();
#endif
        // ---- nu += MJ^T x (lane = coordinate); impulses of the contacts.
        // The lane reads of x run with every lane active: inside a branch on
        // the lane index the compiler may keep x only in the active lanes.
        {
            // blocks of 8 rows: the block's MJ loads go out together (a row
            // at a time waited on each load)
            const int lc = lane < NV ? lane : 0;
            float dnu = 0.f;
            for (int r0 = 0; r0 < NR; r0 += 8) {
                float mj[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) mj[k] = L.MJ[(r0 + k < NR) ? r0 + k : r0][lc];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const int r = r0 + k;
                    const float xr = read_lane(x0, r & (kWaveLanes - 1));
                    dnu += (r < NR) ? xr * mj[k] : 0.f;
                }
            }
            if (lane < NV) L.nu[lane] += dnu;
        }
        for (int r0 = 0; r0 < NR && r0 < ncr; r0 += kWaveLanes) {
            const int r = r0 + lane;
            if (r < ncr && r < NR) L.c_x[r / 3][r % 3] = x0;
        }
    }
    if (warm.rec) {
        // the next step's record, every word written once (no zero-then-
        // overwrite: each ordering fence waited for all of the wave's stores,
        // 9.9k cycles per world-step in this tail on the three-cube scene).
        // Joint rows, lane = body: its three entries, this step's impulse of
        // each of its rows, 0 without one (the lane reads of x with every lane
        // active)
        const bool rec_rows = NR > 0 && NR <= kWaveLanes;
        float jx[3], jx1[3];
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            const int r = ncr + jbefore + __builtin_popcount(jbits & ((1u << t) - 1u));
            const bool has = rec_rows && ((jbits >> t) & 1u) && r < NR;
            const int rl = has ? r : 0;
            const float xv = __shfl(x0, rl), x1v = __shfl(x1s, rl);
            jx[t] = has ? xv : 0.f;
            jx1[t] = has ? x1v : 0.f;
        }
        if (lane < NB) {
#pragma unroll
            for (int t = 0; t < 3; ++t) {
                warm.x(kScWarmJoint0 + 3 * lane + t) = jx[t];
                warm.x1(kScWarmJoint0 + 3 * lane + t) = jx1[t];
            }
        }
        // ... and of the contacts, by key (contact c's rows are 3 c + d, so
        // lane r < ncr holds row r's stage-1 impulse in x1s)
        const int nrec = NR > 0 ? nc : 0;
        if (lane == 0) warm.n() = nrec;
        if (lane < nrec) {
            warm.key(lane) = L.c_key[lane];
#pragma unroll
            for (int d = 0; d < 3; ++d) warm.x(3 * lane + d) = L.c_x[lane][d];
        }
        for (int r = lane; r < 3 * nrec; r += kWaveLanes)
            warm.x1(r) = (r == lane && r < ncr && r < NR && NR <= kWaveLanes) ? x1s : 0.f;
        // the next substep reads the record (other lanes' words)
        __threadfence_block();
    }
    nc_out = nc;

    MW_SC_CHECK(5, nc);
    // ---- integratePositions
    // (a ball joint's three lanes read each other's coordinates: every lane
    // forms its new q before any is stored)
    float q_new = 0.f;
    if (isbody && alive) {
        const float qn = L.nu[P->body_coord[bi]];
        L.qdd[bi] = (qn - L.qd[bi]) * rcp(dt);
        L.qd[bi] = qn;
        q_new = L.q[bi] + dt * qn;
        const int bp = ball_part(P->b[bi]);
        if (bp) {
            const int i0 = bi - bp + 1;
            q_new = ball_integrate(L.q[i0], L.q[i0 + 1], L.q[i0 + 2], L.nu[P->body_coord[i0]],
                                   L.nu[P->body_coord[i0 + 1]], L.nu[P->body_coord[i0 + 2]], dt, bp - 1);
        }
    }
    wave_lds_sync();
    if (isbody && alive) L.q[bi] = q_new;
    if (isbase && alive && md.floating) {
        const int o = md.coff;
        const SV Vn = {{L.nu[o], L.nu[o + 1], L.nu[o + 2]}, {L.nu[o + 3], L.nu[o + 4], L.nu[o + 5]}};
        integrate_pose(Rb0, Vn, dt, base);
        base.V = Vn;
    }
#ifdef MW_WAVE_PROF
    // phase cycles per world-step (scripts/wave_prof.py MW_PROF_MODEL=scene3):
    // [0] ABA + integrateVelocities, [1] contacts + row setup, [2] responses,
    // [3] Delassus, [4] PGS / exact LCP, [5] impulses .. integratePositions,
    // [6] the whole step, [7] world-steps; inside [1]: [19] ground slots,
    // [20] shape pairs
    const long long t_out = clock64();
    if (lane == 0) {
        atomicAdd(&g_wave_prof[0], static_cast<unsigned long long>(t_aba - t_in));
        atomicAdd(&g_wave_prof[1], static_cast<unsigned long long>(t_rows - t_aba));
        atomicAdd(&g_wave_prof[2], static_cast<unsigned long long>(t_resp - t_rows));
        atomicAdd(&g_wave_prof[3], static_cast<unsigned long long>(t_del - t_resp));
        atomicAdd(&g_wave_prof[4], static_cast<unsigned long long>(t_lcp - t_del));
        atomicAdd(&g_wave_prof[5], static_cast<unsigned long long>(t_out - (NR > 0 ? t_lcp : t_rows)));
        atomicAdd(&g_wave_prof[6], static_cast<unsigned long long>(t_out - t_in));
        atomicAdd(&g_wave_prof[7], 1ull);
        atomicAdd(&g_wave_prof[19], static_cast<unsigned long long>(t_gnd - t_aba));
        atomicAdd(&g_wave_prof[20], static_cast<unsigned long long>(t_pairs - t_gnd));
        atomicAdd(&g_wave_prof[21], static_cast<unsigned long long>(t_np - t_gnd));
    }
#endif
}

template <int MAXNV>
__global__ void __launch_bounds__(64) scene_run_kernel(const SceneF* __restrict__ P, SceneDev D,
                                                       const PidF* __restrict__ pid, SceneGates G, int W,
                                                       SceneArgs A) {
    const int w = xcd_block();  // XCD-aware (xcd.hpp): neighbouring worlds share state lines
    const int lane = lane_id();
    __shared__ ScWorld<MAXNV> L;
    const int NB = P->n_bodies, NN = P->n_nodes;
    const uint32_t present = D.present[w];
    // the world's gravity and ground friction (uniform loads)
    const f3 gw = mk(D.wphys[w], D.wphys[static_cast<size_t>(W) + w], D.wphys[2 * static_cast<size_t>(W) + w]);
    const float mu = D.wphys[3 * static_cast<size_t>(W) + w];
    // the base lanes: node0 of every model (lane m of the base arrays = model)
    const bool baselane = lane < NN && P->node_body[lane] < 0;
    const int bm = baselane ? P->node_model[lane] : 0;
    // ---- joints: resets and commands (lane = body)
    uint32_t act = 0u;
    float cmd = 0.f, vc = 0.f;
    if (lane < NB) {
        const size_t k = static_cast<size_t>(lane) * W + w;
        float q = D.q[k], qd = D.qd[k];
        if (A.first) {
            // reset values load with their flag (one round trip, as the wave kernel)
            const uint8_t f = D.rflag[k];
            const float rq = D.rq[k], rqd = D.rqd[k];
            if (f) {
                if (f & 2u) qd = rqd;
                if (f & 1u) q = rq;
                if (f & 4u) { D.pid_e[k] = 0.f; D.pid_i[k] = 0.f; D.pid_u[k] = 0.f; }
                D.rflag[k] = 0;
            }
        }
        act = D.act[k];
        vc = D.vtgt[k];
        cmd = A.first ? D.cmd[k] : 0.f;
        L.q[lane] = q;
        L.qd[lane] = qd;
        L.act[lane] = act;
        L.vc[lane] = vc;
        L.qdd[lane] = 0.f;
    }
    // ---- bases (lane = model): pending pose / velocity resets
    FreeState base{};
    if (baselane) {
        auto at = [&](int f) -> float { return D.base[static_cast<size_t>(13 * bm + f) * W + w]; };
        base.p = {at(0), at(1), at(2)};
        base.qw = at(3); base.qx = at(4); base.qy = at(5); base.qz = at(6);
        base.V = {{at(7), at(8), at(9)}, {at(10), at(11), at(12)}};
        if (A.first) {
            const size_t fk = static_cast<size_t>(bm) * W + w;
            const uint8_t fl = D.bflag[fk];
            float rp[7], rv[6];
#pragma unroll
            for (int f = 0; f < 7; ++f) rp[f] = D.rpose[static_cast<size_t>(7 * bm + f) * W + w];
#pragma unroll
            for (int f = 0; f < 6; ++f) rv[f] = D.rvel[static_cast<size_t>(6 * bm + f) * W + w];
            if (fl & 1u) {
                base.p = {rp[0], rp[1], rp[2]};
                const float inv = 1.f / sqrtf(rp[3] * rp[3] + rp[4] * rp[4] + rp[5] * rp[5] + rp[6] * rp[6]);
                base.qw = rp[3] * inv; base.qx = rp[4] * inv; base.qy = rp[5] * inv; base.qz = rp[6] * inv;
            }
            if (fl & 2u) {
                const M3 Rq = quat_to_R(base.qw, base.qx, base.qy, base.qz);
                base.V = {mulT(Rq, mk(rv[3], rv[4], rv[5])), mulT(Rq, mk(rv[0], rv[1], rv[2]))};
            }
            if (fl) D.bflag[fk] = 0;
        }
    }
    // ---- wrench records of this node (lane = node)
    float wr[kScWrenchSlots][6];
    int32_t wl[kScWrenchSlots];
#pragma unroll
    for (int s = 0; s < kScWrenchSlots; ++s) {
        wl[s] = -1;
#pragma unroll
        for (int e = 0; e < 6; ++e) wr[s][e] = 0.f;
        if (lane < NN) {
            wl[s] = D.wlast[(static_cast<size_t>(s) * kScMaxNodes + lane) * W + w];
            if (wl[s] > A.iter0) {
#pragma unroll
                for (int e = 0; e < 6; ++e)
                    wr[s][e] = D.wrench[((static_cast<size_t>(s) * 6 + e) * kScMaxNodes + lane) * W + w];
            }
        }
    }
    int nc = 0, ovf = 0, unconv = 0;
    bool big_last = false;   // the last substep took the large-contact path: its contacts are in big
    const ScWarm warm{A.lcp_solves > 0 ? D.warm : nullptr, W, w};
    const ScBigWs big{D.big ? D.big + static_cast<size_t>(w) * static_cast<size_t>(D.big_stride) : nullptr, D.big_cmax,
                      D.big_rows, MAXNV};
    if (!A.paused) {
        for (int s = 0; s < A.substeps; ++s) {
            if (lane < NB && ((present >> P->body_model[lane]) & 1u))
                L.tau[lane] = sc_dof_force(P, D, pid, G, W, w, A, s, lane, act, cmd, vc, L.q[lane], L.qd[lane]);
            sc_step<MAXNV>(P, L, base, present, wr, wl, A.iter0 + s + 1, A.dt, A.pgs_iters, A.lcp_solves, warm, gw,
                           mu, big, nc, big_last, ovf, unconv);
        }
    }
    bool bad = false;
    if (lane < NB) {
        const size_t k = static_cast<size_t>(lane) * W + w;
        D.q[k] = L.q[lane];
        D.qd[k] = L.qd[lane];
        // only the world's present models count (a removed model's state is
        // stale: it is re-initialised when the model is placed again)
        bad = ((present >> P->body_model[lane]) & 1u) &&
              (nonfinite_bits(L.q[lane]) || nonfinite_bits(L.qd[lane]));  // finite.hpp
        if (!A.paused) D.qdd[k] = L.qdd[lane];
        D.cmd[k] = 0.f;
        if (D.rb) {
            D.rb[k] = L.q[lane];
            D.rb[D.rb_plane + k] = L.qd[lane];
            if (!A.paused) D.rb[2 * static_cast<size_t>(D.rb_plane) + k] = L.qdd[lane];
        }
    }
    if (baselane) {
        auto at = [&](int f) -> float& { return D.base[static_cast<size_t>(13 * bm + f) * W + w]; };
        at(0) = base.p.x; at(1) = base.p.y; at(2) = base.p.z;
        at(3) = base.qw; at(4) = base.qx; at(5) = base.qy; at(6) = base.qz;
        at(7) = base.V.w.x; at(8) = base.V.w.y; at(9) = base.V.w.z;
        at(10) = base.V.v.x; at(11) = base.V.v.y; at(12) = base.V.v.z;
        const float v[13] = {base.p.x, base.p.y, base.p.z, base.qw, base.qx, base.qy, base.qz,
                             base.V.w.x, base.V.w.y, base.V.w.z, base.V.v.x, base.V.v.y, base.V.v.z};
        bool bb = false;
#pragma unroll
        for (int f = 0; f < 13; ++f) bb = bb || nonfinite_bits(v[f]);
        bad = bad || (bb && ((present >> bm) & 1u));
    }
    if (__ballot(bad) != 0 && lane == 0 && !D.diverged[w]) {
        D.diverged[w] = 1;  // sticky until mw_scene_clear_diverged
        atomicAdd(reinterpret_cast<unsigned long long*>(D.overflow + 4), 1ull);
    }
    if (!A.paused) {
        if (lane == 0) {
            D.ncontact[w] = nc;
            if (ovf) atomicAdd(D.overflow, ovf);
            if (unconv) atomicAdd(reinterpret_cast<unsigned long long*>(D.overflow + 2), static_cast<unsigned long long>(unconv));
        }
        if (A.want_contacts && big_last) {
            for (int c = lane; c < nc; c += kWaveLanes) {
                const float* g = big.ct(c);
                float* o = D.contact + static_cast<size_t>(c) * 12 * W + w;
                const f3 n = mk(g[3], g[4], g[5]);
                const f3 f = A.inv_dt * (g[16] * n + g[17] * mk(g[6], g[7], g[8]) + g[18] * mk(g[9], g[10], g[11]));
                o[0 * W] = g[0]; o[1 * W] = g[1]; o[2 * W] = g[2];
                o[3 * W] = n.x; o[4 * W] = n.y; o[5 * W] = n.z;
                o[6 * W] = f.x; o[7 * W] = f.y; o[8 * W] = f.z;
                o[9 * W] = g[12];
                o[10 * W] = g[13];
                o[11 * W] = g[14];
            }
        } else if (A.want_contacts && lane < nc) {
            const float inv_dt = A.inv_dt;
            float* o = D.contact + static_cast<size_t>(lane) * 12 * W + w;
            const f3 n = mk(L.c_n[lane][0], L.c_n[lane][1], L.c_n[lane][2]);
            f3 t1, t2;
            plane_space_f(n, t1, t2);
            const f3 f = inv_dt * (L.c_x[lane][0] * n + L.c_x[lane][1] * t1 + L.c_x[lane][2] * t2);
            o[0 * W] = L.c_p[lane][0]; o[1 * W] = L.c_p[lane][1]; o[2 * W] = L.c_p[lane][2];
            o[3 * W] = n.x; o[4 * W] = n.y; o[5 * W] = n.z;
            o[6 * W] = f.x; o[7 * W] = f.y; o[8 * W] = f.z;
            o[9 * W] = L.c_d[lane];
            o[10 * W] = __int_as_float(L.c_na[lane]);
            o[11 * W] = __int_as_float(L.c_nb[lane]);
        }
    }
}

}  // namespace dev

hipError_t launch_scene_run(const SceneF* P, int nv, const SceneDev& D, const PidF* pid, const SceneGates& G, int W,
                            const SceneArgs& a, hipStream_t st) {
    if (nv <= 32)
        hipLaunchKernelGGL((dev::scene_run_kernel<32>), dim3(static_cast<unsigned>(W)), dim3(64), 0, st, P, D, pid,
                           G, W, a);
    else
        hipLaunchKernelGGL((dev::scene_run_kernel<64>), dim3(static_cast<unsigned>(W)), dim3(64), 0, st, P, D, pid,
                           G, W, a);
    return hipGetLastError();
}

}  // namespace mw

#ifdef MW_WAVE_PROF
// (declared above their use through the forward declarations below)
#endif
// debug builds (EXTRA=-DMW_WAVE_PROF): the scene kernel's exact-LCP counters
// (its own copy of g_wave_prof: [8] solves, [9] rounds, [10] stage-2 solves,
// [11] max solves, [13] solves > 4, [14] solve cycles, [15] unconverged,
// [16] sweep cycles, [17] stage-1 cycles, [18] exact solves); read and cleared
extern "C" int mw_debug_scene_prof(unsigned long long* out) {
#ifdef MW_WAVE_PROF
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(mw::dev::g_wave_prof), sizeof(mw::dev::g_wave_prof)) != hipSuccess)
        return 1;
    const unsigned long long z[mw::dev::kWaveProfPhases] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(mw::dev::g_wave_prof), z, sizeof(z)) == hipSuccess ? 0 : 1;
#else
    (void)out;
    return 1;
#endif
}

// debug builds: the dumped hard LCP (see scene_run_kernel), then re-armed
extern "C" int mw_debug_scene_dump(float* out, int n) {
#ifdef MW_WAVE_PROF
    if (n < static_cast<int>(sizeof(mw::dev::g_sc_dump) / sizeof(float))) return 2;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(mw::dev::g_sc_dump), sizeof(mw::dev::g_sc_dump)) != hipSuccess) return 1;
    const unsigned int z = 0u;
    return hipMemcpyToSymbol(HIP_SYMBOL(mw::dev::g_sc_dump_claim), &z, sizeof(z)) == hipSuccess ? 0 : 1;
#else
    (void)out;
    (void)n;
    return 1;
#endif
}
