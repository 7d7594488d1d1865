// Test-only host build of gym-ignition_amd/csrc/chain_dyn.hpp: runs the exact
// device substep code on the CPU (float32) so that tests can compare it with
// the fp64 oracle without a GPU.  Not part of the product.
#define MW_HOST_TEST 1
#include <cmath>
#include <cstring>

#include "chain_dyn.hpp"
#include "float_tree.hpp"

using namespace mw;

template <int N, Topo TOPO = chain_topo(N)>
static void run(const ChainF* P, float* q, float* qd, const float* tau, const unsigned char* act,
                const float* vcmd, float dt, int pgs, int cons, int dual, float* qdd) {
    float qq[N], qqd[N], t[N], vc[N], a[N];
    uint8_t ac[N];
    for (int i = 0; i < N; ++i) { qq[i] = q[i]; qqd[i] = qd[i]; t[i] = tau[i]; ac[i] = act[i]; vc[i] = vcmd[i]; }
    if (!cons) dev::substep<N, false, false, TOPO>(P, qq, qqd, t, ac, vc, dt, pgs, a);
    else if (!dual) dev::substep<N, false, true, TOPO>(P, qq, qqd, t, ac, vc, dt, pgs, a);
    else dev::substep<N, true, true, TOPO>(P, qq, qqd, t, ac, vc, dt, pgs, a);
    for (int i = 0; i < N; ++i) { q[i] = qq[i]; qd[i] = qqd[i]; qdd[i] = a[i]; }
}

extern "C" int hd_sizeof_chain() { return sizeof(ChainF); }

extern "C" int hd_substep(const ChainF* P, float* q, float* qd, const float* tau, const unsigned char* act,
                          const float* vcmd, float dt, int pgs, int cons, int dual, float* qdd) {
    bool chain = true;
    for (int i = 0; i < P->n; ++i) chain = chain && P->b[i].parent == i - 1;
    if (!chain) {
        bool panda = P->n == 9;
        for (int i = 0; i < P->n && panda; ++i) panda = P->b[i].parent == parent_of(kPandaTopo, i);
        if (!panda) return 2;
        run<9, kPandaTopo>(P, q, qd, tau, act, vcmd, dt, pgs, cons, dual, qdd);
        return 0;
    }
    switch (P->n) {
    case 1: run<1>(P, q, qd, tau, act, vcmd, dt, pgs, cons, dual, qdd); return 0;
    case 2: run<2>(P, q, qd, tau, act, vcmd, dt, pgs, cons, dual, qdd); return 0;
    case 3: run<3>(P, q, qd, tau, act, vcmd, dt, pgs, cons, dual, qdd); return 0;
    case 7: run<7>(P, q, qd, tau, act, vcmd, dt, pgs, cons, dual, qdd); return 0;
    case 9: run<9>(P, q, qd, tau, act, vcmd, dt, pgs, cons, dual, qdd); return 0;
    default: return 1;
    }
}

// floating-tree step (float_tree.hpp): base[13] = p xyz, q wxyz, twist w v;
// ws: FloatWs<N>::words(n_slots) floats (W = 1); returns -1 if not compiled
template <int N, Topo TOPO>
static int frun(const ChainF* P, const FloatF* F, float* base, float* q, float* qd, const float* tau, float dt,
                int pgs, int cons, float* ws, unsigned* active) {
    static dev::BodyState bs[N * dev::kLdsLanes];
    static dev::SV7 own[N * dev::kLdsLanes];
    dev::LdsStage<N, false> st{bs, nullptr, own, nullptr};
    dev::FloatBody<N> X;
    X.base.p = {base[0], base[1], base[2]};
    X.base.qw = base[3]; X.base.qx = base[4]; X.base.qy = base[5]; X.base.qz = base[6];
    X.base.V = {{base[7], base[8], base[9]}, {base[10], base[11], base[12]}};
    float t[N], vc[N], qdd[N];
    uint8_t act[N];
    for (int i = 0; i < N; ++i) { X.q[i] = q[i]; X.qd[i] = qd[i]; t[i] = tau[i]; vc[i] = 0.f; act[i] = kActForce; }
    const dev::WsRef wr = {ws, 1};
    static float rows[dev::kRowsLdsWords * dev::kLdsLanes];
    const dev::RowsLds rl{rows};
    if (cons) *active = dev::float_step<N, TOPO, true>(P, F, X, t, act, vc, dt, pgs, qdd, st, wr, rl);
    else *active = dev::float_step<N, TOPO, false>(P, F, X, t, act, vc, dt, pgs, qdd, st, wr, rl);
    base[0] = X.base.p.x; base[1] = X.base.p.y; base[2] = X.base.p.z;
    base[3] = X.base.qw; base[4] = X.base.qx; base[5] = X.base.qy; base[6] = X.base.qz;
    base[7] = X.base.V.w.x; base[8] = X.base.V.w.y; base[9] = X.base.V.w.z;
    base[10] = X.base.V.v.x; base[11] = X.base.V.v.y; base[12] = X.base.V.v.z;
    for (int i = 0; i < N; ++i) { q[i] = X.q[i]; qd[i] = X.qd[i]; }
    return 0;
}

extern "C" int hd_sizeof_float() { return sizeof(FloatF); }

extern "C" int hd_float_step(const ChainF* P, const FloatF* F, float* base, float* q, float* qd, const float* tau,
                             float dt, int pgs, int cons, float* ws, unsigned* active) {
    bool quad = P->n == 8;
    for (int i = 0; i < P->n && quad; ++i) quad = P->b[i].parent == parent_of(kQuadrupedTopo, i);
    if (quad) return frun<8, kQuadrupedTopo>(P, F, base, q, qd, tau, dt, pgs, cons, ws, active);
    switch (P->n) {
    case 1: return frun<1, chain_topo(1)>(P, F, base, q, qd, tau, dt, pgs, cons, ws, active);
    case 2: return frun<2, chain_topo(2)>(P, F, base, q, qd, tau, dt, pgs, cons, ws, active);
    case 3: return frun<3, chain_topo(3)>(P, F, base, q, qd, tau, dt, pgs, cons, ws, active);
    default: return -1;
    }
}

// the ball-joint integrator (chain_dyn.hpp ball_integrate) over n states:
// th[3 n], w[3 n] -> out[3 n]
extern "C" void hd_ball_integrate(const float* th, const float* w, float dt, int n, float* out) {
    for (int i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k)
            out[3 * i + k] = mw::dev::ball_integrate(th[3 * i], th[3 * i + 1], th[3 * i + 2], w[3 * i], w[3 * i + 1],
                                            w[3 * i + 2], dt, k);
}
