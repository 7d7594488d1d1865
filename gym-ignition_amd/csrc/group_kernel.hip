// group_kernel.hip -- the position-target env (BASELINE config 4, the Panda)
// with one world per 16-lane row: lane i = dof i (group_tree.hpp).  Same task
// as vecenv_pid_step_kernel in kernels.hip (JointController PID every
// substep on error = q - target, JointController.cpp:195-262 / :308; obs =
// [q, qd]; reward = -|q - target|^2; TimeLimit; Philox auto-reset), but a
// world's dynamics run over 16 lanes, so 1024 worlds are 256 waves instead of
// 16 and each wave's dependent chain is a few hundred instructions per lane
// instead of thousands.
#include "group_tree.hpp"
#include "kernels.hpp"
#include "rng.hpp"
#include "xcd.hpp"

namespace mw {
namespace dev {

#ifdef MW_GROUP_PROF
__device__ unsigned long long g_group_prof[kGroupProfPhases];
#endif

template <int N, bool DUAL, bool CONS>
__global__ void __launch_bounds__(64) vecenv_pid_group_kernel(const ChainF* __restrict__ P, TaskF T, SimDev S,
                                                              VecDev V, const GLaneTask* __restrict__ lt,
                                                              const float* __restrict__ targets,
                                                              float* __restrict__ obs, float* __restrict__ reward,
                                                              uint8_t* __restrict__ done_out,
                                                              float* __restrict__ term_obs, int W, int n, float dt,
                                                              float inv_dt, int substeps, int pgs_iters) {
    unsigned long long prof[kGroupProfPhases] = {};
    MW_GPROF_T(k0);
    const int li = static_cast<int>(threadIdx.x) & (kGroupLanes - 1);
    // XCD-aware world blocks (xcd.hpp): a 128-B line of a [dof][world] array
    // holds 32 worlds = 8 workgroups, which then share one XCD's L2 (else
    // every XCD fetches and partially writes every line: 2.5x the traffic)
    const int wb = xcd_block();
    // rows past the last world run on a copy of it (every lane of the wave
    // takes part in the row exchanges) and store nothing
    const int wr = static_cast<int>((wb * blockDim.x + threadIdx.x) / kGroupLanes);
    const bool live = wr < W;
    const int w = live ? wr : W - 1;
    const bool body = li < n;
    const GBody<N> B = load_gbody<N>(P, li, n);
    const GTopo TT = load_gtopo(P);
    PidF g{};
    float home = 0.f;
    if (body) {
        g = lt[li].pid;
        home = lt[li].home;
    }
    const f3 grav = {P->g[0], P->g[1], P->g[2]};
    const int dl = body ? li : 0;
    float q = 0.f, qd = 0.f, qlo = 0.f, tgt = 0.f, pe = 0.f, pi = 0.f, pu = 0.f;
    if (body) {
        q = S.q[dl * W + w];
        qd = S.qd[dl * W + w];
        qlo = S.qlo[dl * W + w];
        tgt = targets[static_cast<size_t>(w) * n + dl];
        pe = S.pid_e[dl * W + w];
        pi = S.pid_i[dl * W + w];
        pu = S.pid_u[dl * W + w];
    }
    const uint32_t episode0 = V.episode[w];
    const uint32_t steps0 = V.steps[w];
    MW_GPROF_T(k1);
    MW_GPROF_ACC(0, k0, k1);
    for (int s = 0; s < substeps; ++s) {
        float tau = 0.f;
        if (body) {
            float u = pu;
            if (!pid_update(g, (q - tgt) + qlo, inv_dt, dt, pe, pi, u)) u = 0.f;
            else pu = u;
            tau = fminf(fmaxf(u, -B.effort), B.effort);
        }
        group_substep<N, DUAL, CONS>(B, li, n, TT, grav, q, qd, qlo, tau, dt, inv_dt, pgs_iters,
                                     prof);
    }
    MW_GPROF_T(k2);
    // reward: -sum_d (q_d - target_d)^2, summed in dof order
    const float e = body ? (q - tgt) * (q - tgt) : 0.f;
    float r = 0.f;
    sfor<N>([&](auto D) { r -= row_bcast<D>(e); });
    uint32_t steps = steps0 + 1u;
    const bool d_ = (T.max_steps > 0 && steps >= static_cast<uint32_t>(T.max_steps));
    if (live && li == 0) {
        reward[w] = r;
        done_out[w] = d_ ? 1 : 0;
    }
    const size_t ob = static_cast<size_t>(w) * 2 * n;
    if (d_) {
        if (live && body) {
            term_obs[ob + li] = q;
            term_obs[ob + n + li] = qd;
        }
        steps = 0u;
        if (live && li == 0) V.episode[w] = episode0 + 1u;
        // reset: home pose + U(-noise, noise), Philox block = dof / 4
        // (kernels.hip: pid_task_reset), clipped into the limits
        uint32_t rr[4];
        philox(T.seed_lo, T.seed_hi, T.world_offset + static_cast<uint32_t>(w), episode0 + 1u, rr,
               static_cast<uint32_t>(li >> 2));
        const int k = li & 3;
        const uint32_t x4 = (k == 0) ? rr[0] : (k == 1) ? rr[1] : (k == 2) ? rr[2] : rr[3];
        const float x = home + unif(x4, -T.home_noise, T.home_noise);
        q = B.limited ? fminf(fmaxf(x, B.lower), B.upper) : x;
        qd = 0.f;
        pe = pi = pu = qlo = 0.f;
    }
    if (live && body) {
        obs[ob + li] = q;
        obs[ob + n + li] = qd;
        S.q[dl * W + w] = q;
        S.qd[dl * W + w] = qd;
        S.qlo[dl * W + w] = qlo;
        S.pid_e[dl * W + w] = pe;
        S.pid_i[dl * W + w] = pi;
        S.pid_u[dl * W + w] = pu;
    }
    if (live && li == 0) V.steps[w] = steps;
#ifdef MW_GROUP_PROF
    MW_GPROF_T(k3);
    MW_GPROF_ACC(7, k2, k3);
    MW_GPROF_ACC(8, k0, k3);
    if (live && li == 0)
        for (int k = 0; k < kGroupProfPhases; ++k) atomicAdd(&g_group_prof[k], prof[k]);
#else
    (void)prof;
#endif
}

}  // namespace dev

#ifdef MW_GROUP_PROF
// debug builds only: read and clear the group kernel's phase counters
extern "C" int mw_debug_group_prof(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(dev::g_group_prof), sizeof(dev::g_group_prof)) != hipSuccess) return 1;
    const unsigned long long z[dev::kGroupProfPhases] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(dev::g_group_prof), z, sizeof(z)) == hipSuccess ? 0 : 1;
}
#endif

namespace {
template <int N>
hipError_t group_n(const ChainF* P, int n, bool cons, bool dual, const TaskF& T, const SimDev& S, const VecDev& V,
                   const GLaneTask* pid, const float* targets, float* obs, float* reward, uint8_t* done, float* term_obs,
                   int W, float dt, int substeps, int pgs, hipStream_t st) {
    const dim3 grid(static_cast<unsigned>((W + 3) / 4)), block(64);
    const float inv_dt = 1.f / dt;
    if (!cons)
        hipLaunchKernelGGL((dev::vecenv_pid_group_kernel<N, false, false>), grid, block, 0, st, P, T, S, V, pid,
                           targets, obs, reward, done, term_obs, W, n, dt, inv_dt, substeps, pgs);
    else if (!dual)
        hipLaunchKernelGGL((dev::vecenv_pid_group_kernel<N, false, true>), grid, block, 0, st, P, T, S, V, pid,
                           targets, obs, reward, done, term_obs, W, n, dt, inv_dt, substeps, pgs);
    else
        hipLaunchKernelGGL((dev::vecenv_pid_group_kernel<N, true, true>), grid, block, 0, st, P, T, S, V, pid,
                           targets, obs, reward, done, term_obs, W, n, dt, inv_dt, substeps, pgs);
    return hipGetLastError();
}
}  // namespace

hipError_t launch_vecenv_pid_group(const ChainF* P, int n, bool cons, bool dual, const TaskF& T, const SimDev& S,
                                   const VecDev& V, const GLaneTask* pid, const float* targets, float* obs,
                                   float* reward, uint8_t* done, float* term_obs, int W, float dt, int substeps,
                                   int pgs_iters, hipStream_t st) {
    if (n < 1 || n > kMaxKernelDofs || W < 1) return hipErrorInvalidValue;
    if (n <= 9)
        return group_n<9>(P, n, cons, dual, T, S, V, pid, targets, obs, reward, done, term_obs, W, dt, substeps,
                          pgs_iters, st);
    return group_n<kMaxKernelDofs>(P, n, cons, dual, T, S, V, pid, targets, obs, reward, done, term_obs, W, dt,
                                   substeps, pgs_iters, st);
}

}  // namespace mw
