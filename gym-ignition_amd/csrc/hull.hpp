// hull.hpp -- host side: the convex hull of a mesh shape's support points,
// for the scene kernel's mesh narrow phase (scene_kernel.hip sc_hull_pair).
//
// The reference attaches a <mesh> collision to DART as its triangle mesh
// (cpp/scenario/plugins/Physics/Physics.cpp:897-931) [EXT]; this build
// collides a mesh with boxes and other meshes as the convex hull of its
// support points (mesh.cpp: <= kMeshMaxPoints hull vertices, the points that
// also touch the ground plane; a mesh with at most that many hull vertices
// gets its exact hull).  Built once per model in fp64 by brute force (at most
// 16 points): a face is a plane through three points with every point on its
// inner side, coplanar points share one polygon face ordered
// counter-clockwise seen from outside, the edges are the polygons' sides.
// The oracle restates the same construction (oracle.c or_hull_make).
#pragma once

#include <array>
#include <cmath>
#include <utility>
#include <vector>

namespace mw {

constexpr int kHullMaxV = 16;
constexpr int kHullMaxF = 32;   // <= 2 n - 4 triangles for n points
constexpr int kHullMaxE = 48;   // <= 3 n - 6

struct HostHull {
    int nv = 0, nf = 0, ne = 0;
    std::array<std::array<double, 3>, kHullMaxV> v{};
    std::array<std::array<double, 3>, kHullMaxF> n{};   // outward unit normals
    std::array<double, kHullMaxF> d{};                  // inside: n . x <= d
    std::array<int, kHullMaxF> fnv{};
    std::array<std::array<int, kHullMaxV>, kHullMaxF> fv{};
    std::array<std::array<int, 2>, kHullMaxE> e{};
    std::array<std::array<int, 2>, kHullMaxE> ef{};      // the two faces meeting at each edge
    std::array<double, 3> ctr{};                         // vertex centroid (interior)
};

// false for a flat point set (no volume): the mesh then keeps its bounding box
inline bool build_hull(const std::vector<std::array<double, 3>>& pts, HostHull& h) {
    using V = std::array<double, 3>;
    auto dot = [](const V& a, const V& b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; };
    auto cross = [](const V& a, const V& b) {
        return V{a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
    };
    h = HostHull{};
    const int np = static_cast<int>(pts.size() < static_cast<size_t>(kHullMaxV) ? pts.size() : kHullMaxV);
    h.nv = np;
    double scale = 0.0;
    for (int i = 0; i < np; ++i)
        for (int k = 0; k < 3; ++k) {
            h.v[i][k] = pts[i][k];
            h.ctr[k] += pts[i][k] / np;
            scale = std::fmax(scale, std::fabs(pts[i][k]));
        }
    const double eps = 1e-9 * (scale > 0.0 ? scale : 1.0);
    for (int i = 0; i < np; ++i)
        for (int j = i + 1; j < np; ++j)
            for (int k = j + 1; k < np; ++k) {
                const V a = {h.v[j][0] - h.v[i][0], h.v[j][1] - h.v[i][1], h.v[j][2] - h.v[i][2]};
                const V b = {h.v[k][0] - h.v[i][0], h.v[k][1] - h.v[i][1], h.v[k][2] - h.v[i][2]};
                V n = cross(a, b);
                const double len = std::sqrt(dot(n, n));
                if (len <= 1e-12 * (scale * scale > 0.0 ? scale * scale : 1.0)) continue;   // collinear
                for (double& x : n) x /= len;
                double d = dot(n, h.v[i]), hi = -1e300, lo = 1e300;
                for (int m = 0; m < np; ++m) {
                    const double s = dot(n, h.v[m]) - d;
                    hi = std::fmax(hi, s);
                    lo = std::fmin(lo, s);
                }
                if (hi > eps && lo < -eps) continue;   // points on both sides: not a face
                if (hi > eps) {                         // all above: the outward normal is -n
                    for (double& x : n) x = -x;
                    d = -d;
                }
                bool dup = false;
                for (int f = 0; f < h.nf && !dup; ++f)
                    dup = std::fabs(dot(h.n[f], n) - 1.0) < 1e-9 && std::fabs(h.d[f] - d) <= 4 * eps;
                if (dup || h.nf >= kHullMaxF) continue;
                h.n[h.nf] = n;
                h.d[h.nf] = d;
                ++h.nf;
            }
    if (h.nf < 4) return false;
    for (int f = 0; f < h.nf; ++f) {
        int idx[kHullMaxV], m = 0;
        double ang[kHullMaxV];
        V c = {0, 0, 0};
        for (int i = 0; i < np; ++i)
            if (std::fabs(dot(h.n[f], h.v[i]) - h.d[f]) <= 4 * eps) idx[m++] = i;
        for (int t = 0; t < m; ++t)
            for (int q = 0; q < 3; ++q) c[q] += h.v[idx[t]][q] / m;
        V u = {h.v[idx[0]][0] - c[0], h.v[idx[0]][1] - c[1], h.v[idx[0]][2] - c[2]};
        const double ul = std::sqrt(dot(u, u));
        for (double& x : u) x /= ul;
        const V w = cross(h.n[f], u);
        for (int t = 0; t < m; ++t) {
            const V r = {h.v[idx[t]][0] - c[0], h.v[idx[t]][1] - c[1], h.v[idx[t]][2] - c[2]};
            ang[t] = std::atan2(dot(r, w), dot(r, u));
        }
        for (int a = 1; a < m; ++a)
            for (int b = a; b > 0 && ang[b] < ang[b - 1]; --b) {
                std::swap(ang[b], ang[b - 1]);
                std::swap(idx[b], idx[b - 1]);
            }
        h.fnv[f] = m;
        for (int t = 0; t < m; ++t) h.fv[f][t] = idx[t];
        for (int t = 0; t < m; ++t) {
            int a = idx[t], b = idx[(t + 1) % m];
            if (a > b) std::swap(a, b);
            int seen = -1;
            for (int e = 0; e < h.ne && seen < 0; ++e)
                if (h.e[e][0] == a && h.e[e][1] == b) seen = e;
            if (seen >= 0) {
                h.ef[seen][1] = f;
            } else if (h.ne < kHullMaxE) {
                h.e[h.ne] = {a, b};
                h.ef[h.ne] = {f, f};
                ++h.ne;
            }
        }
    }
    return true;
}

// A mesh whose support points are exactly its bounding box's 8 corners is
// that box: it keeps the box narrow phase (bit for bit like the box).
inline bool mesh_is_box(const std::vector<std::array<double, 3>>& pts, const std::array<double, 3>& size) {
    if (pts.size() != 8) return false;
    unsigned corners = 0u;
    for (const auto& p : pts) {
        bool ok = true;
        for (int k = 0; k < 3; ++k) ok = ok && std::fabs(std::fabs(p[k]) - size[k]) <= 1e-12 * (1.0 + size[k]);
        if (ok) corners |= 1u << ((p[0] > 0) * 4 + (p[1] > 0) * 2 + (p[2] > 0));
    }
    return corners == 0xffu;
}

}  // namespace mw
