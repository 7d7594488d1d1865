// Test-only host build of gym-ignition_amd/csrc/chain_dyn.hpp: runs the exact
// device substep code on the CPU (float32) so that tests can compare it with
// the fp64 oracle without a GPU.  Not part of the product.
#define MW_HOST_TEST 1
#include <cmath>
#include <cstring>

#include "chain_dyn.hpp"

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
