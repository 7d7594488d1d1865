// kernels.hip -- HIP kernels of the many-worlds stepper (gfx950).
//
// One world per lane.  State is SoA [dof][world] so that every load/store of
// a wave is 256 contiguous bytes; model parameters are uniform (scalar path).
//
//  scenario_run   : GazeboSimulator::run() semantics for the ScenarI/O shim
//                   (resets -> commands -> substeps -> readback, force command
//                   consumed by the first substep), Physics.cpp:646-685,
//                   :1330-1440, :2226-2345.
//  vecenv_step    : one gym step of every world with the Task logic of
//                   python/gym_ignition_environments/tasks/*.py fused in
//                   (obs, reward, done, TimeLimit, auto-reset).
//  vecenv_reset   : initial reset of every world (Philox4x32-10).
#include <type_traits>

#include "baked_models.hpp"
#include "chain_dyn.hpp"
#include "float_tree.hpp"
#include "wave_tree.hpp"
#include "free_body.hpp"
#include "kernels.hpp"
#include "pid.hpp"
#include "rng.hpp"
#include "xcd.hpp"

namespace mw {
namespace dev {

// ------------------------------------------------- divergence detection ----
// A world whose stored state holds a non-finite value (finite.hpp: an
// exponent-bit test the finite-math build keeps) is flagged once (sticky until
// mw_clear_diverged) and counted; mw_run reports the new ones (MW_EDIVERGED).

__device__ __forceinline__ void mark_diverged(uint8_t* flags, unsigned long long* count, int w) {
    if (flags && !flags[w]) {
        flags[w] = 1;
        atomicAdd(count, 1ull);
    }
}

__device__ __forceinline__ bool base_nonfinite(const FreeState& b) {
    const float v[13] = {b.p.x, b.p.y, b.p.z, b.qw, b.qx, b.qy, b.qz, b.V.w.x, b.V.w.y, b.V.w.z,
                         b.V.v.x, b.V.v.y, b.V.v.z};
    bool bad = false;
#pragma unroll
    for (int k = 0; k < 13; ++k) bad = bad || nonfinite_bits(v[k]);
    return bad;
}

// ------------------------------------------------------ baked models ----
// The shipped models' parameter blocks as device constants: a kernel
// instantiated with BAKED != 0 reads the model from here, and the compiler
// folds the zeros / ones of its transforms, axes and inertias (CartPole
// substep: 1507 -> 672 instructions).  The host selects a baked kernel only
// when the loaded model's block is bit-identical (sim.cpp: baked_id).
__constant__ constexpr baked::CartpoleBlock kCartpoleDev = {{MW_BAKED_CARTPOLE_INIT}};
__constant__ constexpr baked::PendulumBlock kPendulumDev = {{MW_BAKED_PENDULUM_INIT}};
__constant__ constexpr baked::PandaBlock kPandaDev = {{MW_BAKED_PANDA_INIT}};

template <int BAKED>
__device__ __forceinline__ const ChainF* model_params(const ChainF* P) {
    if constexpr (BAKED == baked::kCartpoleId) return reinterpret_cast<const ChainF*>(&kCartpoleDev);
    else if constexpr (BAKED == baked::kPendulumId) return reinterpret_cast<const ChainF*>(&kPendulumDev);
    else if constexpr (BAKED == baked::kPandaId) return reinterpret_cast<const ChainF*>(&kPandaDev);
    else return P;
}

// ------------------------------------------------------- staging --------
// Generic models of >= kLdsMinDofs dofs keep their per-body substep state in
// LDS (chain_dyn.hpp: LdsStage): in registers it spills to scratch.  The
// constant-folded (baked) models need far fewer live values and keep it in
// VGPRs + AGPRs without scratch (the baked Panda: 256 + 136 registers);
// measured on the config-4 Panda env (scripts/ab_panda.py, graph replay):
// LDS 15.9 -> registers 9.3 us per step at 1024 worlds, 15.1 -> 9.0 at 128.
// Both kinds run 64-thread workgroups.
#ifndef MW_LDS_MIN_DOFS
#define MW_LDS_MIN_DOFS 7
#endif
constexpr int kLdsMinDofs = MW_LDS_MIN_DOFS;

template <int N, int BAKED>
constexpr bool lds_staged() { return N >= kLdsMinDofs && BAKED == 0; }

#define MW_DECLARE_STAGE(N, DUAL, BAKED, NAME)                                                       \
    constexpr bool kLds_##NAME = lds_staged<N, BAKED>();                                             \
    __shared__ BodyState sh_bs_[(kLds_##NAME ? N : 1) * kLdsLanes];                                  \
    __shared__ ImpulseFactor sh_nf_[((kLds_##NAME && DUAL) ? N : 1) * kLdsLanes];                    \
    __shared__ SV7 sh_own_[(kLds_##NAME ? N : 1) * kLdsLanes];                                       \
    __shared__ float sh_mv_[(kLds_##NAME ? N * N : 1) * kLdsLanes];                                  \
    using StageT = std::conditional_t<kLds_##NAME, LdsStage<N, DUAL>, RegStage<N, DUAL>>;           \
    StageT NAME = make_stage<N, DUAL, kLds_##NAME>(sh_bs_, sh_nf_, sh_own_, sh_mv_)

template <int N, bool DUAL, bool LDS>
__device__ __forceinline__ auto make_stage(BodyState* b, ImpulseFactor* f, SV7* o, float* m) {
    if constexpr (LDS) {
        return LdsStage<N, DUAL>{b + threadIdx.x, f + threadIdx.x, o + threadIdx.x, m + threadIdx.x};
    } else {
        (void)b; (void)f; (void)o; (void)m;
        return RegStage<N, DUAL>{};
    }
}

constexpr float kPi = 3.14159265358979323846f;

// ----------------------------------------------------------- tasks ------
// kinds: 0 CartPoleDiscreteBalancing, 1 CartPoleContinuousBalancing,
//        2 CartPoleContinuousSwingup, 3 PendulumSwingUp
template <int N, int KIND>
__device__ __forceinline__ void task_reset(const TaskF& T, uint32_t w, uint32_t episode,
                                           float (&q)[N], float (&qd)[N]) {
    uint32_t r[4];
    philox(T.seed_lo, T.seed_hi, w, episode, r);
    if constexpr (KIND == 0 || KIND == 1) {
        // x, dx, q, dq = U(-0.05, 0.05)   cartpole_discrete_balancing.py:137
        q[0] = unif(r[0], -0.05f, 0.05f); qd[0] = unif(r[1], -0.05f, 0.05f);
        q[1] = unif(r[2], -0.05f, 0.05f); qd[1] = unif(r[3], -0.05f, 0.05f);
    } else if constexpr (KIND == 2) {
        // q = pi - deg2rad(U(-60, 60)); x, dx, dq = U(-0.05, 0.05)  cartpole_continuous_swingup.py:145-146
        q[1] = kPi - unif(r[0], -60.f, 60.f) * (kPi / 180.f);
        q[0] = unif(r[1], -0.05f, 0.05f); qd[0] = unif(r[2], -0.05f, 0.05f);
        qd[1] = unif(r[3], -0.05f, 0.05f);
    } else {
        // cos, sin, dq = observation_space.sample(); q = atan2(sin, cos)  pendulum_swingup.py:117-127
        const float c = unif(r[0], -1.f, 1.f), s = unif(r[1], -1.f, 1.f);
        q[0] = atan2f(s, c);
        qd[0] = unif(r[2], -10.f, 10.f);
    }
}

template <int N, int KIND>
__device__ __forceinline__ void task_obs(const float (&q)[N], const float (&qd)[N], float (&o)[4]) {
    if constexpr (KIND == 3) {
        float s, c;
        sincosf(q[0], &s, &c);
        o[0] = c; o[1] = s; o[2] = qd[0]; o[3] = 0.f;
    } else {
        o[0] = q[0]; o[1] = qd[0]; o[2] = q[1]; o[3] = qd[1];   // [x, dx, q, dq]
    }
}

template <int KIND>
__device__ __forceinline__ bool task_done(const TaskF& T, const float (&o)[4]) {
    constexpr int no = (KIND == 3) ? 3 : 4;
    bool inside = true;
#pragma unroll
    for (int k = 0; k < no; ++k) inside = inside && (o[k] >= -T.hi[k]) && (o[k] <= T.hi[k]);
    return !inside;
}

template <int N, int KIND>
__device__ __forceinline__ float task_reward(const TaskF& T, const float (&q)[N], const float (&qd)[N],
                                             const float (&o)[4], bool done) {
    // no FMA contraction: the reward is bit-identical in the per-step and the
    // fused-rollout kernels (contraction would otherwise depend on context)
#pragma clang fp contract(off)
    if constexpr (KIND == 0 || KIND == 1) {
        float r = done ? 0.f : 1.f;
        if (T.reward_cart_at_center)
            r = r - 0.10f * fabsf(o[0]) - 0.10f * fabsf(o[1]) -
                10.0f * (o[0] >= T.x_factor * 2.4f ? 1.f : 0.f);
        return r;
    } else if constexpr (KIND == 2) {
        return (cosf(q[1]) + 1.f) * 0.5f - 0.1f * qd[0] * qd[0] -
               10.0f * (q[0] >= T.x_factor * 2.4f ? 1.f : 0.f);
    } else {
        // the force target read after the run is the zero-filled JointForceCmd
        // (Physics.cpp:2250-2254), so the 0.001 tau^2 term of
        // pendulum_swingup.py:86-88 is identically zero
        const float cost = (done ? 100.f : 0.f) + q[0] * q[0] + 0.1f * qd[0] * qd[0];
        return -cost;
    }
}

// Per-world physics sample of (world, episode): masses from Philox blocks
// 1.., gravity from block 8 by Box-Muller (SDFRandomizer.sample,
// randomizers/model/sdf.py:264-315: force_positive clips the SAMPLE at 0, so
// an additive mass change is max(U(lo, hi), 0); cartpole.py:51-56 gravity).
template <int N>
__device__ __forceinline__ Dyn<N> sample_dyn(const ChainF* __restrict__ P, const TaskF& T, uint32_t w,
                                             uint32_t episode, float& gz_out) {
    Dyn<N> D = nominal_dyn<N>(P);
    gz_out = 0.f;
    if (T.randomize & kRandMass) {
#pragma unroll
        for (int b = 0; b < (N + 3) / 4; ++b) {
            uint32_t r[4];
            philox(T.seed_lo, T.seed_hi, w, episode, r, 1u + static_cast<uint32_t>(b));
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (4 * b + k < N) D.m[4 * b + k] += fmaxf(unif(r[k], T.mass_lo, T.mass_hi), 0.f);
        }
    }
    if (T.randomize & kRandGravity) {
        uint32_t r[4];
        philox(T.seed_lo, T.seed_hi, w, episode, r, 8u);
        const float u1 = static_cast<float>((r[0] >> 8) + 1u) * (1.f / 16777216.f);  // (0, 1]
        const float u2 = static_cast<float>(r[1] >> 8) * (1.f / 16777216.f);
        const float z = sqrtf(-2.f * logf(u1)) * cosf(2.f * kPi * u2);
        const float gz = T.g_mean + T.g_std * z;
        D.g = {gz * T.gdir[0], gz * T.gdir[1], gz * T.gdir[2]};
        gz_out = gz;
    }
    return D;
}

template <int N>
__device__ __forceinline__ Dyn<N> load_dyn(const ChainF* __restrict__ P, const TaskF& T, const VecDev& V, int W,
                                           int w) {
    Dyn<N> D = nominal_dyn<N>(P);
    if (T.randomize & kRandMass) {
#pragma unroll
        for (int d = 0; d < N; ++d) D.m[d] = V.rmass[d * W + w];
    }
    if (T.randomize & kRandGravity) {
        const float gz = V.rgz[w];
        D.g = {gz * T.gdir[0], gz * T.gdir[1], gz * T.gdir[2]};
    }
    return D;
}

template <int N>
__device__ __forceinline__ void store_dyn(const TaskF& T, const VecDev& V, int W, int w, const Dyn<N>& D,
                                          float gz) {
    if (T.randomize & kRandMass) {
#pragma unroll
        for (int d = 0; d < N; ++d) V.rmass[d * W + w] = D.m[d];
    }
    if (T.randomize & kRandGravity) V.rgz[w] = gz;
}

template <int N>
__device__ __forceinline__ void load_state(const SimDev& S, int W, int w, float (&q)[N], float (&qd)[N]) {
#pragma unroll
    for (int d = 0; d < N; ++d) {
        q[d] = S.q[d * W + w];
        qd[d] = S.qd[d * W + w];
    }
}

template <int N>
__device__ __forceinline__ void store_state(const SimDev& S, int W, int w, const float (&q)[N],
                                            const float (&qd)[N]) {
#pragma unroll
    for (int d = 0; d < N; ++d) {
        S.q[d * W + w] = q[d];
        S.qd[d * W + w] = qd[d];
    }
}

template <int NO>
__device__ __forceinline__ void store_obs(float* __restrict__ dst, const float (&o)[4]) {
    if constexpr (NO == 4) {
        *reinterpret_cast<float4*>(dst) = make_float4(o[0], o[1], o[2], o[3]);
    } else {
#pragma unroll
        for (int k = 0; k < NO; ++k) dst[k] = o[k];
    }
}

// ---------------------------------------------------------- kernels -----

// Joint forces of substep s of a run: a Force-mode command (SetForce ->
// GenericJoint::setCommand clips to +-effort) acts on the first substep only
// (UpdateSim zero-fills it); Position / Velocity joints take the
// JointController PID force (JointController::PreUpdate,
// JointController.cpp:195-262), recomputed when the period gate opens,
// otherwise the last command (pid.Cmd()); error = current - target (:308).
template <int N>
__device__ __forceinline__ void joint_forces(const ChainF* __restrict__ P, const SimDev& S, const PidSet& pid, int W,
                                             int w, const RunArgs& A, int s, const uint8_t (&act)[N],
                                             const float (&cmd)[N], const float (&vc)[N], const float (&q)[N],
                                             const float (&qd)[N], const float (&qlo)[N], bool any_pid,
                                             float (&tau)[N]) {
    const bool gate = (A.pid_gate >> s) & 1u;
#pragma unroll
    for (int d = 0; d < N; ++d) {
        const float e = P->b[d].effort;
        tau[d] = (act[d] == kActForce && s == 0) ? fminf(fmaxf(cmd[d], -e), e) : 0.f;
    }
    if (any_pid) {
#pragma unroll
        for (int d = 0; d < N; ++d) {
            if (act[d] >= kActPidPos) {
                const size_t k = static_cast<size_t>(d) * W + w;
                float u = S.pid_u[k];
                if (gate) {
                    const bool pos = (act[d] == kActPidPos);
                    const float err = pos ? ((q[d] - S.ptgt[k]) + qlo[d]) : (qd[d] - vc[d]);
                    float el = S.pid_e[k], ie = S.pid_i[k];
                    if (pid_update(pid.g[d], err, A.inv_dt, A.dt, el, ie, u)) {
                        S.pid_e[k] = el; S.pid_i[k] = ie; S.pid_u[k] = u;
                    } else {
                        u = 0.f;
                    }
                }
                const float e = P->b[d].effort;
                tau[d] = fminf(fmaxf(u, -e), e);
            }
        }
    }
}

// Joint resets of a run's first launch: velocity reset, then position reset
// (UpdatePhysics, Physics.cpp:1330-1375); Joint::reset*/setControlMode/setPID
// also reset the joint PID (Joint.cpp:148-151).
template <int N>
__device__ __forceinline__ void joint_resets(const SimDev& S, int W, int w, float (&q)[N], float (&qd)[N]) {
#pragma unroll
    for (int d = 0; d < N; ++d) {
        const uint8_t f = S.rflag[d * W + w];
        if (f) {
            if (f & 2u) qd[d] = S.rqd[d * W + w];
            if (f & 1u) { q[d] = S.rq[d * W + w]; S.qlo[d * W + w] = 0.f; }
            if (f & 4u) { S.pid_e[d * W + w] = 0.f; S.pid_i[d * W + w] = 0.f; S.pid_u[d * W + w] = 0.f; }
            S.rflag[d * W + w] = 0;
        }
    }
}

template <int N, bool DUAL, bool CONS, Topo TOPO, int BAKED = 0>
__global__ void __launch_bounds__(256) scenario_run_kernel(const ChainF* __restrict__ Pin, SimDev S, PidSet pid,
                                                           int W, RunArgs A) {
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= W) return;
    const ChainF* __restrict__ P = model_params<BAKED>(Pin);
    float q[N], qd[N], qlo[N];
    load_state<N>(S, W, w, q, qd);
    if (A.first) joint_resets<N>(S, W, w, q, qd);
#pragma unroll
    for (int d = 0; d < N; ++d) qlo[d] = S.qlo[d * W + w];
    if (!A.paused) {
        float cmd[N], vc[N], tau[N], qdd[N];
        uint8_t act[N];
        bool any_pid = false;
#pragma unroll
        for (int d = 0; d < N; ++d) {
            cmd[d] = A.first ? S.cmd[d * W + w] : 0.f;
            act[d] = S.act[d * W + w];
            vc[d] = S.vtgt[d * W + w];
            any_pid = any_pid || act[d] >= kActPidPos;
        }
        MW_DECLARE_STAGE(N, DUAL, BAKED, stage);
        for (int s = 0; s < A.substeps; ++s) {
            joint_forces<N>(P, S, pid, W, w, A, s, act, cmd, vc, q, qd, qlo, any_pid, tau);
            substep<N, DUAL, CONS, TOPO>(P, q, qd, tau, act, vc, A.dt, A.pgs_iters, qdd, stage, nominal_dyn<N>(P),
                                         qlo);
        }
#pragma unroll
        for (int d = 0; d < N; ++d) S.qdd[d * W + w] = qdd[d];
#pragma unroll
        for (int d = 0; d < N; ++d) S.qlo[d * W + w] = qlo[d];
    }
#pragma unroll
    for (int d = 0; d < N; ++d) S.cmd[d * W + w] = 0.f;  // JointForceCmd zero-fill (paused too)
    store_state<N>(S, W, w, q, qd);
    bool bad = false;
#pragma unroll
    for (int d = 0; d < N; ++d) bad = bad || nonfinite_bits(q[d]) || nonfinite_bits(qd[d]);
    if (bad) mark_diverged(S.div, S.ndiv, w);
}

template <int N, int KIND>
__global__ void __launch_bounds__(256) vecenv_reset_kernel(const ChainF* __restrict__ P, TaskF T, SimDev S,
                                                           VecDev V, float* __restrict__ obs, int W) {
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= W) return;
    float q[N], qd[N], o[4];
    if (T.randomize) {
        const uint32_t gw = T.world_offset + static_cast<uint32_t>(w);
        float gz;
        const Dyn<N> D = sample_dyn<N>(P, T, gw, 0u, gz);
        store_dyn<N>(T, V, W, w, D, gz);
    }
    task_reset<N, KIND>(T, T.world_offset + static_cast<uint32_t>(w), 0u, q, qd);
    task_obs<N, KIND>(q, qd, o);
    constexpr int NO = (KIND == 3) ? 3 : 4;
    store_obs<NO>(obs + static_cast<size_t>(w) * NO, o);
    store_state<N>(S, W, w, q, qd);
    V.episode[w] = 0u;
    V.steps[w] = 0u;
}

// STEPS == 0: single step; otherwise loop over T_steps with [t, w] layouts.
template <int N, int KIND, bool DUAL, bool CONS, bool ROLLOUT, int BAKED, bool RAND = false>
__global__ void __launch_bounds__(256) vecenv_step_kernel(const ChainF* __restrict__ Pin, TaskF T, SimDev S,
                                                          VecDev V, const void* __restrict__ actions,
                                                          float* __restrict__ obs, float* __restrict__ reward,
                                                          uint8_t* __restrict__ done_out,
                                                          float* __restrict__ term_obs, int W, float dt,
                                                          int substeps, int pgs_iters, int T_steps) {
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= W) return;
    const ChainF* __restrict__ P = model_params<BAKED>(Pin);
    constexpr int NO = (KIND == 3) ? 3 : 4;
    float q[N], qd[N];
    load_state<N>(S, W, w, q, qd);
    const uint32_t episode0 = V.episode[w];
    uint32_t episode = episode0;
    uint32_t steps = V.steps[w];
    uint8_t act[N];
    float vc[N];
#pragma unroll
    for (int d = 0; d < N; ++d) { act[d] = kActForce; vc[d] = 0.f; }
    Dyn<N> D;
    if constexpr (RAND) D = load_dyn<N>(P, T, V, W, w);
    const int nsteps = ROLLOUT ? T_steps : 1;
    for (int t = 0; t < nsteps; ++t) {
        const size_t idx = static_cast<size_t>(t) * W + w;
        float force;
        if constexpr (KIND == 0) {
            const int a = static_cast<const int32_t*>(actions)[idx];
            force = (a == 1) ? T.force_mag : -T.force_mag;   // cartpole_discrete_balancing.py:70
        } else {
            force = static_cast<const float*>(actions)[idx];
        }
        // the driven joint ("linear" / "pivot") is dof 0; other joints are Idle
        const float e = P->b[0].effort;
        force = fminf(fmaxf(force, -e), e);
        float tau[N], qdd[N];
        for (int s = 0; s < substeps; ++s) {
#pragma unroll
            for (int d = 0; d < N; ++d) tau[d] = 0.f;
            tau[0] = (s == 0) ? force : 0.f;
            if constexpr (RAND) substep_dyn<N, DUAL, CONS>(P, q, qd, tau, act, vc, dt, pgs_iters, qdd, D);
            else substep<N, DUAL, CONS>(P, q, qd, tau, act, vc, dt, pgs_iters, qdd);
        }
        float o[4];
        task_obs<N, KIND>(q, qd, o);
        const bool tdone = task_done<KIND>(T, o);
        reward[idx] = task_reward<N, KIND>(T, q, qd, o, tdone);
        steps += 1u;
        const bool d_ = tdone || (T.max_steps > 0 && steps >= static_cast<uint32_t>(T.max_steps));
        done_out[idx] = d_ ? 1 : 0;
        if (d_) {
            store_obs<NO>(term_obs + idx * NO, o);
            episode += 1u;
            steps = 0u;
            if constexpr (RAND) {
                // GazeboEnvRandomizer.reset: new physics and model sample per episode
                float gz;
                D = sample_dyn<N>(P, T, T.world_offset + static_cast<uint32_t>(w), episode, gz);
                store_dyn<N>(T, V, W, w, D, gz);
            }
            task_reset<N, KIND>(T, T.world_offset + static_cast<uint32_t>(w), episode, q, qd);
            task_obs<N, KIND>(q, qd, o);
        }
        store_obs<NO>(obs + idx * NO, o);
    }
    store_state<N>(S, W, w, q, qd);
    if (episode != episode0) V.episode[w] = episode;  // changes only on auto-reset
    V.steps[w] = steps;
}

// ------------------------------------------------- floating free body ----
// Base pose / twist of world w, with the pending resets of a run's first
// launch applied (UpdatePhysics: World pose / velocity resets of the model's
// base link, Physics.cpp:1330-1375).
__device__ __forceinline__ FreeState load_base(const FreeDev& D, int W, int w, bool first) {
    auto at = [&](int f) -> float { return D.base[f * W + w]; };
    FreeState S;
    S.p = {at(0), at(1), at(2)};
    S.qw = at(3); S.qx = at(4); S.qy = at(5); S.qz = at(6);
    S.V = {{at(7), at(8), at(9)}, {at(10), at(11), at(12)}};
    if (first) {
        // the reset values load together with their flag (one round trip,
        // not a flag load and then the values: both buffers always exist)
        const uint8_t fl = D.rflag[w];
        float rp[7], rv[6];
#pragma unroll
        for (int f = 0; f < 7; ++f) rp[f] = D.rpose[f * W + w];
#pragma unroll
        for (int f = 0; f < 6; ++f) rv[f] = D.rvel[f * W + w];
        if (fl & 1u) {
            S.p = {rp[0], rp[1], rp[2]};
            const float inv = 1.f / sqrtf(rp[3] * rp[3] + rp[4] * rp[4] + rp[5] * rp[5] + rp[6] * rp[6]);
            S.qw = rp[3] * inv; S.qx = rp[4] * inv; S.qy = rp[5] * inv; S.qz = rp[6] * inv;
        }
        if (fl & 2u) {
            // world velocities of the base origin -> body-frame twist
            const M3 R = quat_to_R(S.qw, S.qx, S.qy, S.qz);
            const f3 lin = {rv[0], rv[1], rv[2]};
            const f3 ang = {rv[3], rv[4], rv[5]};
            S.V = {mulT(R, ang), mulT(R, lin)};
        }
        if (fl) D.rflag[w] = 0;
    }
    return S;
}

__device__ __forceinline__ void store_base(const FreeDev& D, int W, int w, const FreeState& S) {
    auto at = [&](int f) -> float& { return D.base[f * W + w]; };
    at(0) = S.p.x; at(1) = S.p.y; at(2) = S.p.z;
    at(3) = S.qw; at(4) = S.qx; at(5) = S.qy; at(6) = S.qz;
    at(7) = S.V.w.x; at(8) = S.V.w.y; at(9) = S.V.w.z;
    at(10) = S.V.v.x; at(11) = S.V.v.y; at(12) = S.V.v.z;
}

// contact force on the body, world frame: (n x_n + t1 x_t1 + t2 x_t2) / dt
// with n = (0, 0, 1), t1 = (0, -1, 0), t2 = (1, 0, 0)
__device__ __forceinline__ void store_contact(const FreeDev& D, int W, int w, int slot, f3 xw, float xn, float x1,
                                              float x2, float depth, float inv_dt) {
    float* o = D.cdata + static_cast<size_t>(slot) * 7 * W + w;
    o[0 * W] = xw.x; o[1 * W] = xw.y; o[2 * W] = xw.z;
    o[3 * W] = x2 * inv_dt;
    o[4 * W] = -x1 * inv_dt;
    o[5 * W] = xn * inv_dt;
    o[6 * W] = depth;
}

// GazeboSimulator::run() for a floating single-body model: pending base pose /
// velocity resets (WorldPoseCmd / WorldVelocityCmd, Model.cpp:256-360 ->
// Physics.cpp:1535-1590), the substeps, and the contacts of the last substep
// (Physics.cpp:2351-2540: point, force on the body = impulse / dt, depth).
template <bool MESH>
__global__ void __launch_bounds__(256) free_run_kernel(const FreeF* __restrict__ F, FreeDev D, int W, RunArgs A,
                                                       int want_contacts) {
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= W) return;
    FreeState S = load_base(D, W, w, A.first);
    __shared__ SlotRec slots[kMaxFreeSlots * kFreeLanes];
    Contacts C;
    C.active = 0u;
    C.rec = slots + threadIdx.x;
    if (!A.paused) {
        for (int s = 0; s < A.substeps; ++s) free_step<MESH>(F, A.dt, A.pgs_iters, S, C);
    }
    store_base(D, W, w, S);
    if (base_nonfinite(S)) mark_diverged(D.div, D.ndiv, w);
    if (want_contacts && !A.paused) {
        D.cmask[w] = C.active;
        const float inv_dt = 1.f / A.dt;
        for (uint32_t m = C.active; m; m &= m - 1u) {
            const int slot = __builtin_ctz(m);
            const SlotRec& r = C.at(slot);
            store_contact(D, W, w, slot, r.xw, r.x[0], r.x[1], r.x[2], r.depth, inv_dt);
        }
    }
}

// Articulated model on a floating base (float_tree.hpp): the scenario run of
// scenario_run_kernel (joint resets, commands, PID) plus the base state of
// free_run_kernel.  ws: the per-world row workspace, FloatWs<N>::words(n_slots)
// floats per world, [word][W].
template <int N, Topo TOPO, bool CONS>
__global__ void __launch_bounds__(64) float_run_kernel(const ChainF* __restrict__ P, const FloatF* __restrict__ F,
                                                       SimDev S, FreeDev D, PidSet pid, float* __restrict__ ws,
                                                       int W, RunArgs A, int want_contacts) {
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= W) return;
    FloatBody<N> X;
    X.base = load_base(D, W, w, A.first);
    load_state<N>(S, W, w, X.q, X.qd);
    if (A.first) joint_resets<N>(S, W, w, X.q, X.qd);
    uint32_t active = 0u;
    const WsRef wr = {ws + w, W};
    if (!A.paused) {
        float cmd[N], vc[N], tau[N], qdd[N];
        uint8_t act[N];
        bool any_pid = false;
#pragma unroll
        for (int d = 0; d < N; ++d) {
            cmd[d] = A.first ? S.cmd[d * W + w] : 0.f;
            act[d] = S.act[d * W + w];
            vc[d] = S.vtgt[d * W + w];
            any_pid = any_pid || act[d] >= kActPidPos;
        }
        __shared__ BodyState sh_bs[N * kLdsLanes];
        __shared__ SV7 sh_own[N * kLdsLanes];
        __shared__ float sh_rows[kRowsLdsWords * kLdsLanes];
        LdsStage<N, false> stage{sh_bs + threadIdx.x, nullptr, sh_own + threadIdx.x, nullptr};
        const RowsLds rows{sh_rows + threadIdx.x};
        const float no_lo[N] = {};  // the floating-tree kernel integrates q uncompensated
        for (int s = 0; s < A.substeps; ++s) {
            joint_forces<N>(P, S, pid, W, w, A, s, act, cmd, vc, X.q, X.qd, no_lo, any_pid, tau);
            active = float_step<N, TOPO, CONS>(P, F, X, tau, act, vc, A.dt, A.pgs_iters, qdd, stage, wr, rows);
        }
#pragma unroll
        for (int d = 0; d < N; ++d) S.qdd[d * W + w] = qdd[d];
    }
#pragma unroll
    for (int d = 0; d < N; ++d) S.cmd[d * W + w] = 0.f;
    store_state<N>(S, W, w, X.q, X.qd);
    store_base(D, W, w, X.base);
    bool bad = base_nonfinite(X.base);
#pragma unroll
    for (int d = 0; d < N; ++d) bad = bad || nonfinite_bits(X.q[d]) || nonfinite_bits(X.qd[d]);
    if (bad) mark_diverged(D.div, D.ndiv, w);
    if (want_contacts && !A.paused) {
        D.cmask[w] = active;
        const float inv_dt = 1.f / A.dt;
        using L = FloatWs<N>;
        for (uint32_t m = active; m; m &= m - 1u) {
            const int slot = __builtin_ctz(m);
            const int o = slot * L::kSlotWords;
            store_contact(D, W, w, slot, mk(wr.at(o + 3), wr.at(o + 4), wr.at(o + 5)), wr.at(o + 16), wr.at(o + 17),
                          wr.at(o + 18), wr.at(o + 6), inv_dt);
        }
    }
}

// Large articulated models on a floating base, one world per wavefront
// (wave_tree.hpp).  Same run semantics as float_run_kernel; the PID gains
// come from a device array (any dof count).  blockIdx.x = world.
// The first substep's PID inputs of dof d, loaded with the kernel's prologue
// (the wave kernel: otherwise the PID phase waits on them, two dependent
// round trips after the prologue's own).
struct PidPre {
    float effort, u, tgt, e, i;
    PidF g;
};

__device__ __forceinline__ PidPre pid_preload(const ChainF* __restrict__ P, const SimDev& S,
                                              const PidF* __restrict__ pid, int W, int w, int d) {
    const size_t k = static_cast<size_t>(d) * W + w;
    return PidPre{P->b[d].effort, S.pid_u[k], S.ptgt[k], S.pid_e[k], S.pid_i[k], pid[d]};
}

__device__ __forceinline__ float dof_force(const ChainF* __restrict__ P, const SimDev& S, const PidF* __restrict__ pid,
                                           int W, int w, const RunArgs& A, int s, int d, uint32_t act, float cmd,
                                           float vc, float q, float qd, const PidPre* pre = nullptr) {
    const float e = pre ? pre->effort : P->b[d].effort;
    float tau = (act == kActForce && s == 0) ? fminf(fmaxf(cmd, -e), e) : 0.f;
    if (act >= kActPidPos) {
        const size_t k = static_cast<size_t>(d) * W + w;
        float u = pre ? pre->u : S.pid_u[k];
        if ((A.pid_gate >> s) & 1u) {
            const float err = (act == kActPidPos) ? (q - (pre ? pre->tgt : S.ptgt[k])) : (qd - vc);
            float el = pre ? pre->e : S.pid_e[k], ie = pre ? pre->i : S.pid_i[k];
            if (pid_update(pre ? pre->g : pid[d], err, A.inv_dt, A.dt, el, ie, u)) {
                S.pid_e[k] = el; S.pid_i[k] = ie; S.pid_u[k] = u;
            } else {
                u = 0.f;
            }
        }
        tau = fminf(fmaxf(u, -e), e);
    }
    return tau;
}

template <int MAXN, bool CONS>
__global__ void __launch_bounds__(64, 1) wave_run_kernel(const ChainF* __restrict__ P, const FloatF* __restrict__ F,
                                                      int N, SimDev S, FreeDev D, const PidF* __restrict__ pid,
                                                      int W, RunArgs A, int want_contacts, int* __restrict__ overflow) {
    MW_PROF_T(tk0);
    const int w = xcd_block();  // XCD-aware (xcd.hpp): neighbouring worlds share state lines
    const int lane = lane_id();
    __shared__ WaveWorld<MAXN> L;
    // Every load of the prologue is issued before any is used: the reset flags
    // used to gate the warm-record and reset-value loads, two dependent round
    // trips (the prologue measured 11.1k cycles per launch, profiles/r05y)
    constexpr int kXwPerLane = (kWaveWarmRecord + kWaveLanes - 1) / kWaveLanes;
    float xwv[kXwPerLane];
    if (A.warm) {
#pragma unroll
        for (int j = 0; j < kXwPerLane; ++j) {
            const int e = lane + j * kWaveLanes;
            xwv[j] = (e < kWaveWarmRecord) ? D.warm[static_cast<size_t>(e) * W + w] : 0.f;
        }
    }
    const bool base_reset = A.first && D.rflag[w] != 0;
    uint32_t act = 0u;
    float cmd = 0.f, vc = 0.f, q = 0.f, qd = 0.f, rq = 0.f, rqd = 0.f;
    uint8_t jflag = 0;
    const size_t kq = static_cast<size_t>(lane) * W + w;
    if (lane < N) {
        q = S.q[kq];
        qd = S.qd[kq];
        if (A.first) {
            jflag = S.rflag[kq];
            rq = S.rq[kq];
            rqd = S.rqd[kq];
            cmd = S.cmd[kq];
        }
        act = S.act[kq];
        vc = S.vtgt[kq];
    }
    PidPre pre0 = {};
    if (lane < N) pre0 = pid_preload(P, S, pid, W, w, lane);
    FreeState base = load_base(D, W, w, A.first);
    // warm start: a world whose base or joints were reset starts cold
    if (A.warm) {
        const bool warm_reset = __ballot(base_reset || jflag != 0) != 0;
#pragma unroll
        for (int j = 0; j < kXwPerLane; ++j) {
            const int e = lane + j * kWaveLanes;
            if (e < kWaveWarmRecord) L.xw[e] = warm_reset ? 0.f : xwv[j];
        }
    }
    if (lane < N) {
        if (jflag) {
            if (jflag & 2u) qd = rqd;
            if (jflag & 1u) q = rq;
            if (jflag & 4u) {
                // Joint::resetPosition resets the PID (Joint.cpp:132-180): the
                // preloaded first-substep inputs must see the reset too
                S.pid_e[kq] = 0.f; S.pid_i[kq] = 0.f; S.pid_u[kq] = 0.f;
                pre0.e = 0.f; pre0.i = 0.f; pre0.u = 0.f;
            }
            S.rflag[kq] = 0;
        }
        L.q[lane] = q;
        L.qd[lane] = qd;
        L.act[lane] = act;
        L.vc[lane] = vc;
    }
    uint32_t active = 0u;
    int ovf = 0, unconv = 0;
    unsigned long long prof[kWaveProfPhases] = {};
    if (A.wrenches && lane <= N) {
        // the world wrenches of this launch's substeps (lane = node: 0 the base)
#pragma unroll
        for (int e = 0; e < 6; ++e) L.ext[lane][e] = D.wrench[(static_cast<size_t>(e) * D.wnodes + lane) * W + w];
    }
#ifdef MW_WAVE_PROF
    {
        // the prologue's loads have landed once the first substep reads them
        // (q / qd through LDS): time to here is issue + the first waits
        wave_lds_sync();
        MW_PROF_T(tk1);
        MW_PROF_ACC(20, tk0, tk1);
    }
#endif
    // the first substep's joint forces from the preloaded PID inputs (pre0
    // dies here instead of living through the substep loop)
    float tau0 = 0.f;
    if (!A.paused && lane < N) tau0 = dof_force(P, S, pid, W, w, A, 0, lane, act, cmd, vc, q, qd, &pre0);
    if (!A.paused) {
        for (int s = 0; s < A.substeps; ++s) {
            MW_PROF_T(ta);
            if (lane < N)
                L.tau[lane] = (s == 0) ? tau0 : dof_force(P, S, pid, W, w, A, s, lane, act, cmd, vc, L.q[lane], L.qd[lane]);
            MW_PROF_T(tb);
            MW_PROF_ACC(0, ta, tb);
            active = wave_step<MAXN, CONS>(P, F, N, base, L, A.dt, A.pgs_iters, A.pgs_tol, A.warm != 0,
                                           A.lcp_solves, L.qdd, &ovf, &unconv, prof, A.wrenches != 0);
            MW_PROF_T(tc);
            MW_PROF_ACC(7, ta, tc);
        }
    }
#ifdef MW_WAVE_PROF
    if (lane == 0)
        for (int k = 0; k < kWaveProfPhases; ++k) {
            if (k == 11 || k == 12)
                atomicMax(&g_wave_prof[k], prof[k]);
            else
                atomicAdd(&g_wave_prof[k], prof[k]);
        }
#else
    (void)prof;
#endif
    bool bad = false;
    if (lane < N) {
        const size_t k = static_cast<size_t>(lane) * W + w;
        S.q[k] = L.q[lane];
        S.qd[k] = L.qd[lane];
        if (!A.paused) S.qdd[k] = L.qdd[lane];
        S.cmd[k] = 0.f;
        bad = nonfinite_bits(L.q[lane]) || nonfinite_bits(L.qd[lane]);
    }
    if (lane == 0) bad = bad || base_nonfinite(base);
    bad = __ballot(bad) != 0;
    if (lane == 0) {
        if (bad) mark_diverged(D.div, D.ndiv, w);
        store_base(D, W, w, base);
        if (ovf) atomicAdd(overflow, ovf);
        // exact LCP solves that ran out of budget: a 64-bit counter at words 2-3
        if (unconv) atomicAdd(reinterpret_cast<unsigned long long*>(overflow + 2), static_cast<unsigned long long>(unconv));
    }
    if (A.warm)  // also after a paused run: it may have consumed a reset
        for (int e = lane; e < kWaveWarmRecord; e += kWaveLanes) D.warm[static_cast<size_t>(e) * W + w] = L.xw[e];
    if (want_contacts && !A.paused) {
        if (lane == 0) D.cmask[w] = active;
        if (lane < 32 && ((active >> lane) & 1u)) {
            const float inv_dt = 1.f / A.dt;
            store_contact(D, W, w, lane, mk(L.s_xw[lane][0], L.s_xw[lane][1], L.s_xw[lane][2]), L.s_x[lane][0],
                          L.s_x[lane][1], L.s_x[lane][2], L.s_depth[lane], inv_dt);
        }
    }
}

// ------------------------------------------------ position-target task ----
// kind 4 (BASELINE config 4, Panda): every joint in Position mode, the
// JointController PID runs every substep (controller period = step size,
// test_pid_controllers.py:69) on error = q - target (JointController.cpp:308).
// obs = [q, qd] (2n), reward = -sum (q - target)^2, done = TimeLimit only;
// reset: home pose + U(-noise, noise) per joint (Philox block k = 4-dof group),
// clipped into the position limits, qd = 0, PID reset.
template <int N>
__device__ __forceinline__ void pid_task_reset(const ChainF* __restrict__ P, const TaskF& T, uint32_t w,
                                               uint32_t episode, float (&q)[N], float (&qd)[N]) {
#pragma unroll
    for (int b = 0; b < (N + 3) / 4; ++b) {
        uint32_t r[4];
        philox(T.seed_lo, T.seed_hi, w, episode, r, static_cast<uint32_t>(b));
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int d = 4 * b + k;
            if (d < N) {
                const float x = T.home[d] + unif(r[k], -T.home_noise, T.home_noise);
                q[d] = P->b[d].limited ? fminf(fmaxf(x, P->b[d].lower), P->b[d].upper) : x;
                qd[d] = 0.f;
            }
        }
    }
}

template <int N>
__device__ __forceinline__ void store_pid_obs(float* __restrict__ dst, const float (&q)[N], const float (&qd)[N]) {
#pragma unroll
    for (int d = 0; d < N; ++d) { dst[d] = q[d]; dst[N + d] = qd[d]; }
}

template <int N, Topo TOPO, bool DUAL, bool CONS, int BAKED = 0>
__global__ void __launch_bounds__(256) vecenv_pid_step_kernel(const ChainF* __restrict__ Pin, TaskF T, SimDev S,
                                                              VecDev V, PidSet pid,
                                                              const float* __restrict__ targets,
                                                              float* __restrict__ obs, float* __restrict__ reward,
                                                              uint8_t* __restrict__ done_out,
                                                              float* __restrict__ term_obs, int W, float dt,
                                                              float inv_dt, int substeps, int pgs_iters) {
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= W) return;
    const ChainF* __restrict__ P = model_params<BAKED>(Pin);
    float q[N], qd[N], qlo[N], tgt[N], pe[N], pi[N], pu[N];
    load_state<N>(S, W, w, q, qd);
#pragma unroll
    for (int d = 0; d < N; ++d) {
        qlo[d] = S.qlo[d * W + w];
        tgt[d] = targets[static_cast<size_t>(w) * N + d];
        pe[d] = S.pid_e[d * W + w];
        pi[d] = S.pid_i[d * W + w];
        pu[d] = S.pid_u[d * W + w];
    }
    uint8_t act[N];
    float vc[N];
#pragma unroll
    for (int d = 0; d < N; ++d) { act[d] = kActPidPos; vc[d] = 0.f; }
    float tau[N], qdd[N];
    MW_DECLARE_STAGE(N, DUAL, BAKED, stage);
    for (int s = 0; s < substeps; ++s) {
#pragma unroll
        for (int d = 0; d < N; ++d) {
            float u = pu[d];
            if (!pid_update(pid.g[d], (q[d] - tgt[d]) + qlo[d], inv_dt, dt, pe[d], pi[d], u)) u = 0.f;
            else pu[d] = u;
            const float e = P->b[d].effort;
            tau[d] = fminf(fmaxf(u, -e), e);
        }
        substep<N, DUAL, CONS, TOPO>(P, q, qd, tau, act, vc, dt, pgs_iters, qdd, stage, nominal_dyn<N>(P), qlo);
    }
    float r = 0.f;
#pragma unroll
    for (int d = 0; d < N; ++d) r -= (q[d] - tgt[d]) * (q[d] - tgt[d]);
    reward[w] = r;
    const uint32_t episode0 = V.episode[w];
    uint32_t steps = V.steps[w] + 1u;
    const bool d_ = (T.max_steps > 0 && steps >= static_cast<uint32_t>(T.max_steps));
    done_out[w] = d_ ? 1 : 0;
    if (d_) {
        store_pid_obs<N>(term_obs + static_cast<size_t>(w) * 2 * N, q, qd);
        steps = 0u;
        V.episode[w] = episode0 + 1u;
        pid_task_reset<N>(P, T, T.world_offset + static_cast<uint32_t>(w), episode0 + 1u, q, qd);
#pragma unroll
        for (int d = 0; d < N; ++d) { pe[d] = 0.f; pi[d] = 0.f; pu[d] = 0.f; qlo[d] = 0.f; }
    }
    store_pid_obs<N>(obs + static_cast<size_t>(w) * 2 * N, q, qd);
    store_state<N>(S, W, w, q, qd);
#pragma unroll
    for (int d = 0; d < N; ++d) {
        S.qlo[d * W + w] = qlo[d];
        S.pid_e[d * W + w] = pe[d];
        S.pid_i[d * W + w] = pi[d];
        S.pid_u[d * W + w] = pu[d];
    }
    V.steps[w] = steps;
}

template <int N>
__global__ void __launch_bounds__(256) vecenv_pid_reset_kernel(const ChainF* __restrict__ P, TaskF T, SimDev S,
                                                               VecDev V, float* __restrict__ obs, int W) {
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= W) return;
    float q[N], qd[N];
    pid_task_reset<N>(P, T, T.world_offset + static_cast<uint32_t>(w), 0u, q, qd);
    store_pid_obs<N>(obs + static_cast<size_t>(w) * 2 * N, q, qd);
    store_state<N>(S, W, w, q, qd);
#pragma unroll
    for (int d = 0; d < N; ++d) {
        S.pid_e[d * W + w] = 0.f; S.pid_i[d * W + w] = 0.f; S.pid_u[d * W + w] = 0.f; S.qlo[d * W + w] = 0.f;
    }
    V.episode[w] = 0u;
    V.steps[w] = 0u;
}

}  // namespace dev

// ------------------------------------------------------- launchers ------
namespace {

dim3 grid_for(int W, int block) { return dim3(static_cast<unsigned>((W + block - 1) / block)); }

// 64-thread blocks spread a small world count over as many CUs as possible
// (each wave runs a long dependent chain); 256 once there is work for all.
int block_for(int W) { return (W <= 64 * 256) ? 64 : 256; }
// LDS-staged kernels (>= kLdsMinDofs dofs) always run one wave per workgroup
int block_for(int W, int n) { return (n >= dev::kLdsMinDofs) ? dev::kLdsLanes : block_for(W); }

template <int N, Topo TOPO>
hipError_t scenario_n(const ChainF* P, bool cons, bool dual, int baked, const SimDev& S, const PidSet& pid, int W,
                      const RunArgs& a, hipStream_t st) {
    const int B = block_for(W, N);
    if constexpr (N == 9 && TOPO == kPandaTopo) {
        // the shipped Panda, constant-folded (it has limits and no damping)
        if (baked == baked::kPandaId && cons && !dual) {
            hipLaunchKernelGGL((dev::scenario_run_kernel<N, false, true, TOPO, baked::kPandaId>), grid_for(W, B),
                               dim3(B), 0, st, P, S, pid, W, a);
            return hipGetLastError();
        }
    }
    if (!cons)
        hipLaunchKernelGGL((dev::scenario_run_kernel<N, false, false, TOPO>), grid_for(W, B), dim3(B), 0, st, P,
                           S, pid, W, a);
    else if (!dual)
        hipLaunchKernelGGL((dev::scenario_run_kernel<N, false, true, TOPO>), grid_for(W, B), dim3(B), 0, st, P,
                           S, pid, W, a);
    else
        hipLaunchKernelGGL((dev::scenario_run_kernel<N, true, true, TOPO>), grid_for(W, B), dim3(B), 0, st, P,
                           S, pid, W, a);
    return hipGetLastError();
}

template <int N, int KIND, bool ROLLOUT, bool RAND>
hipError_t vec_nk(const ChainF* P, bool cons, bool dual, int baked, const TaskF& T, const SimDev& S,
                  const VecDev& V, const void* a, float* o, float* r, uint8_t* d, float* to, int W,
                  float dt, int substeps, int pgs, int Ts, hipStream_t st) {
    const int B = block_for(W);
    // constant-folded instantiations for the shipped models (their flags fix cons/dual)
    if constexpr (N == 2 && KIND <= 2) {
        if (baked == baked::kCartpoleId && cons && !dual) {
            hipLaunchKernelGGL((dev::vecenv_step_kernel<N, KIND, false, true, ROLLOUT, baked::kCartpoleId, RAND>),
                               grid_for(W, B), dim3(B), 0, st, P, T, S, V, a, o, r, d, to, W, dt, substeps, pgs, Ts);
            return hipGetLastError();
        }
    }
    if constexpr (N == 1 && KIND == 3) {
        if (baked == baked::kPendulumId && !cons) {
            hipLaunchKernelGGL((dev::vecenv_step_kernel<N, KIND, false, false, ROLLOUT, baked::kPendulumId, RAND>),
                               grid_for(W, B), dim3(B), 0, st, P, T, S, V, a, o, r, d, to, W, dt, substeps, pgs, Ts);
            return hipGetLastError();
        }
    }
    if (!cons)
        hipLaunchKernelGGL((dev::vecenv_step_kernel<N, KIND, false, false, ROLLOUT, 0, RAND>), grid_for(W, B), dim3(B),
                           0, st, P, T, S, V, a, o, r, d, to, W, dt, substeps, pgs, Ts);
    else if (!dual)
        hipLaunchKernelGGL((dev::vecenv_step_kernel<N, KIND, false, true, ROLLOUT, 0, RAND>), grid_for(W, B), dim3(B),
                           0, st, P, T, S, V, a, o, r, d, to, W, dt, substeps, pgs, Ts);
    else
        hipLaunchKernelGGL((dev::vecenv_step_kernel<N, KIND, true, true, ROLLOUT, 0, RAND>), grid_for(W, B), dim3(B),
                           0, st, P, T, S, V, a, o, r, d, to, W, dt, substeps, pgs, Ts);
    return hipGetLastError();
}

}  // namespace

int kernel_topology(const int* parents, int n) {
    bool chain = true, panda = (n == 9), quad = (n == 8);
    for (int i = 0; i < n; ++i) {
        chain = chain && parents[i] == i - 1;
        panda = panda && parents[i] == parent_of(kPandaTopo, i);
        quad = quad && parents[i] == parent_of(kQuadrupedTopo, i);
    }
    if (chain && n >= 1 && n <= 9) return 0;
    if (panda) return 1;
    if (quad) return 2;
    return -1;
}

int float_workspace_words(int n, int n_slots) {
    switch (n) {
    case 1: return dev::FloatWs<1>::words(n_slots);
    case 2: return dev::FloatWs<2>::words(n_slots);
    case 3: return dev::FloatWs<3>::words(n_slots);
    case 8: return dev::FloatWs<8>::words(n_slots);
    default: return -1;
    }
}

namespace {
template <int N, Topo TOPO>
hipError_t float_n(const ChainF* P, bool cons, const FloatF* F, const SimDev& S, const FreeDev& D, const PidSet& pid,
                   float* ws, int W, const RunArgs& a, int contacts, hipStream_t st) {
    const int B = dev::kLdsLanes;  // LDS stage: one wave per workgroup
    if (cons)
        hipLaunchKernelGGL((dev::float_run_kernel<N, TOPO, true>), grid_for(W, B), dim3(B), 0, st, P, F, S, D, pid, ws,
                           W, a, contacts);
    else
        hipLaunchKernelGGL((dev::float_run_kernel<N, TOPO, false>), grid_for(W, B), dim3(B), 0, st, P, F, S, D, pid,
                           ws, W, a, contacts);
    return hipGetLastError();
}
}  // namespace

#ifdef MW_WAVE_PROF
// debug builds only: read and clear the wave kernel's phase counters
// debug builds: the dumped hard exact LCP of the wave kernel (wave_tree.hpp), then re-armed
extern "C" int mw_debug_wave_dump(float* out, int n) {
#ifdef MW_WAVE_PROF
    if (n < static_cast<int>(sizeof(dev::g_wave_dump) / sizeof(float))) return 2;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(dev::g_wave_dump), sizeof(dev::g_wave_dump)) != hipSuccess) return 1;
    const unsigned int z = 0u;
    return hipMemcpyToSymbol(HIP_SYMBOL(dev::g_wave_dump_claim), &z, sizeof(z)) == hipSuccess ? 0 : 1;
#else
    (void)out;
    (void)n;
    return 1;
#endif
}

extern "C" int mw_debug_wave_prof(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(dev::g_wave_prof), sizeof(dev::g_wave_prof)) != hipSuccess) return 1;
    const unsigned long long z[dev::kWaveProfPhases] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(dev::g_wave_prof), z, sizeof(z)) == hipSuccess ? 0 : 1;
}
#endif

hipError_t launch_wave_run(const ChainF* P, int n, int depth, bool cons, const FloatF* F, const SimDev& S,
                           const FreeDev& D, const PidF* pid, int W, const RunArgs& a, int contacts, int* overflow,
                           hipStream_t st) {
    const dim3 grid(static_cast<unsigned>(W)), block(dev::kWaveLanes);
    if (depth > dev::kWaveMaxDepth) return hipErrorInvalidValue;
    if (n <= 16 && depth <= dev::WaveWorld<16>::kDepth) {
        if (cons)
            hipLaunchKernelGGL((dev::wave_run_kernel<16, true>), grid, block, 0, st, P, F, n, S, D, pid, W, a,
                               contacts, overflow);
        else
            hipLaunchKernelGGL((dev::wave_run_kernel<16, false>), grid, block, 0, st, P, F, n, S, D, pid, W, a,
                               contacts, overflow);
    } else if (n <= 32) {
        if (cons)
            hipLaunchKernelGGL((dev::wave_run_kernel<32, true>), grid, block, 0, st, P, F, n, S, D, pid, W, a,
                               contacts, overflow);
        else
            hipLaunchKernelGGL((dev::wave_run_kernel<32, false>), grid, block, 0, st, P, F, n, S, D, pid, W, a,
                               contacts, overflow);
    } else if (n <= kMaxBodies) {
        if (cons)
            hipLaunchKernelGGL((dev::wave_run_kernel<kMaxBodies, true>), grid, block, 0, st, P, F, n, S, D, pid, W,
                               a, contacts, overflow);
        else
            hipLaunchKernelGGL((dev::wave_run_kernel<kMaxBodies, false>), grid, block, 0, st, P, F, n, S, D, pid, W,
                               a, contacts, overflow);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_float_run(const ChainF* P, int n, int topo, bool cons, const FloatF* F, const SimDev& S,
                            const FreeDev& D, const PidSet& pid, float* ws, int W, const RunArgs& a, int contacts,
                            hipStream_t st) {
    if (topo == 2 && n == 8) return float_n<8, kQuadrupedTopo>(P, cons, F, S, D, pid, ws, W, a, contacts, st);
    if (topo != 0) return hipErrorInvalidValue;
    switch (n) {
    case 1: return float_n<1, chain_topo(1)>(P, cons, F, S, D, pid, ws, W, a, contacts, st);
    case 2: return float_n<2, chain_topo(2)>(P, cons, F, S, D, pid, ws, W, a, contacts, st);
    case 3: return float_n<3, chain_topo(3)>(P, cons, F, S, D, pid, ws, W, a, contacts, st);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_scenario_run(const ChainF* P, int n, int topo, bool cons, bool dual, int baked, const SimDev& S,
                               const PidSet& pid, int W, const RunArgs& a, hipStream_t st) {
    if (topo == 1) return scenario_n<9, kPandaTopo>(P, cons, dual, baked, S, pid, W, a, st);
    if (topo != 0) return hipErrorInvalidValue;
    switch (n) {
    case 1: return scenario_n<1, chain_topo(1)>(P, cons, dual, baked, S, pid, W, a, st);
    case 2: return scenario_n<2, chain_topo(2)>(P, cons, dual, baked, S, pid, W, a, st);
    case 3: return scenario_n<3, chain_topo(3)>(P, cons, dual, baked, S, pid, W, a, st);
    case 4: return scenario_n<4, chain_topo(4)>(P, cons, dual, baked, S, pid, W, a, st);
    case 5: return scenario_n<5, chain_topo(5)>(P, cons, dual, baked, S, pid, W, a, st);
    case 6: return scenario_n<6, chain_topo(6)>(P, cons, dual, baked, S, pid, W, a, st);
    case 7: return scenario_n<7, chain_topo(7)>(P, cons, dual, baked, S, pid, W, a, st);
    case 8: return scenario_n<8, chain_topo(8)>(P, cons, dual, baked, S, pid, W, a, st);
    case 9: return scenario_n<9, chain_topo(9)>(P, cons, dual, baked, S, pid, W, a, st);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_free_run(const FreeF* F, const FreeDev& D, int W, const RunArgs& a, int contacts, int mesh,
                           hipStream_t st) {
    const int B = dev::kFreeLanes;  // the contact slot records in LDS assume 64-thread blocks
    if (mesh)
        hipLaunchKernelGGL(dev::free_run_kernel<true>, grid_for(W, B), dim3(B), 0, st, F, D, W, a, contacts);
    else
        hipLaunchKernelGGL(dev::free_run_kernel<false>, grid_for(W, B), dim3(B), 0, st, F, D, W, a, contacts);
    return hipGetLastError();
}

hipError_t launch_vecenv_reset(const ChainF* P, int n, const TaskF& T, const SimDev& S,
                               const VecDev& V, float* obs, int W, hipStream_t st) {
    const int B = block_for(W);
    if (T.kind == 4 && n == 9)
        hipLaunchKernelGGL((dev::vecenv_pid_reset_kernel<9>), grid_for(W, B), dim3(B), 0, st, P, T, S, V, obs, W);
    else if (T.kind == 3 && n == 1)
        hipLaunchKernelGGL((dev::vecenv_reset_kernel<1, 3>), grid_for(W, B), dim3(B), 0, st, P, T, S, V, obs, W);
    else if (T.kind == 0 && n == 2)
        hipLaunchKernelGGL((dev::vecenv_reset_kernel<2, 0>), grid_for(W, B), dim3(B), 0, st, P, T, S, V, obs, W);
    else if (T.kind == 1 && n == 2)
        hipLaunchKernelGGL((dev::vecenv_reset_kernel<2, 1>), grid_for(W, B), dim3(B), 0, st, P, T, S, V, obs, W);
    else if (T.kind == 2 && n == 2)
        hipLaunchKernelGGL((dev::vecenv_reset_kernel<2, 2>), grid_for(W, B), dim3(B), 0, st, P, T, S, V, obs, W);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t launch_vecenv_pid_step(const ChainF* P, int n, int topo, bool cons, bool dual, int baked, const TaskF& T,
                                  const SimDev& S, const VecDev& V, const PidSet& pid, const float* targets,
                                  float* obs, float* reward, uint8_t* done, float* term_obs, int W,
                                  float dt, int substeps, int pgs_iters, hipStream_t st) {
    if (n != 9 || topo != 1) return hipErrorInvalidValue;
    const int B = block_for(W, 9);
    const float inv_dt = 1.f / dt;
    if (baked == baked::kPandaId && cons && !dual)
        hipLaunchKernelGGL((dev::vecenv_pid_step_kernel<9, kPandaTopo, false, true, baked::kPandaId>), grid_for(W, B),
                           dim3(B), 0, st, P, T, S, V, pid, targets, obs, reward, done, term_obs, W, dt, inv_dt,
                           substeps, pgs_iters);
    else if (!cons)
        hipLaunchKernelGGL((dev::vecenv_pid_step_kernel<9, kPandaTopo, false, false>), grid_for(W, B), dim3(B), 0,
                           st, P, T, S, V, pid, targets, obs, reward, done, term_obs, W, dt, inv_dt, substeps,
                           pgs_iters);
    else if (!dual)
        hipLaunchKernelGGL((dev::vecenv_pid_step_kernel<9, kPandaTopo, false, true>), grid_for(W, B), dim3(B), 0,
                           st, P, T, S, V, pid, targets, obs, reward, done, term_obs, W, dt, inv_dt, substeps,
                           pgs_iters);
    else
        hipLaunchKernelGGL((dev::vecenv_pid_step_kernel<9, kPandaTopo, true, true>), grid_for(W, B), dim3(B), 0,
                           st, P, T, S, V, pid, targets, obs, reward, done, term_obs, W, dt, inv_dt, substeps,
                           pgs_iters);
    return hipGetLastError();
}

hipError_t launch_vecenv_step(const ChainF* P, int n, bool cons, bool dual, int baked, const TaskF& T,
                              const SimDev& S, const VecDev& V, const void* actions, float* obs,
                              float* reward, uint8_t* done, float* term_obs, int W, float dt,
                              int substeps, int pgs_iters, int T_steps, hipStream_t st) {
#define MW_VEC_R(NN, KK, RR)                                                                                 \
    return (T_steps > 0)                                                                                     \
               ? vec_nk<NN, KK, true, RR>(P, cons, dual, baked, T, S, V, actions, obs, reward, done, term_obs, W, \
                                          dt, substeps, pgs_iters, T_steps, st)                              \
               : vec_nk<NN, KK, false, RR>(P, cons, dual, baked, T, S, V, actions, obs, reward, done, term_obs,   \
                                           W, dt, substeps, pgs_iters, 1, st)
#define MW_VEC(NN, KK)              \
    if (T.randomize) MW_VEC_R(NN, KK, true); \
    MW_VEC_R(NN, KK, false)
    if (T.kind == 3 && n == 1) { MW_VEC(1, 3); }
    if (T.kind == 0 && n == 2) { MW_VEC(2, 0); }
    if (T.kind == 1 && n == 2) { MW_VEC(2, 1); }
    if (T.kind == 2 && n == 2) { MW_VEC(2, 2); }
#undef MW_VEC
#undef MW_VEC_R
    return hipErrorInvalidValue;
}

}  // namespace mw

// ---- test hook: one linear solve of the exact LCP's active-set method -------
// (include/mwstep_testhooks.h mw_debug_lcp_solve; tests/test_gpu_lcp_solve.py checks both
// paths against numpy on random SPD systems with held rows)
namespace mw {
namespace dev {
__global__ void __launch_bounds__(64) debug_lcp_solve_kernel(const float* __restrict__ A, const float* __restrict__ rhs,
                                                             uint64_t freeM, int n, int method, float* __restrict__ d) {
    __shared__ float Uw[kLcpWorkFloats];
    const int lane = lane_id();
    float a[kWaveMaxRows];
#pragma unroll
    for (int r = 0; r < kWaveMaxRows; ++r) a[r] = (r < n && lane < n) ? A[r * n + lane] : 0.f;
    const float rh = (lane < n) ? rhs[lane] : 0.f;
    float out;
    if (method == 0) {
        out = (n <= 32) ? lcp_mfma_solve<32>(a, rh, freeM, Uw) : lcp_mfma_solve<64>(a, rh, freeM, Uw);
    } else {
        const bool fr = mask_bit(freeM, lane);
        float k[kWaveMaxRows];
#pragma unroll
        for (int c = 0; c < kWaveMaxRows; ++c) k[c] = (fr && mask_bit(freeM, c)) ? a[c] : ((!fr && c == lane) ? 1.f : 0.f);
        out = lcp_ge_solve<kWaveMaxRows>(k, fr ? rh : 0.f, n, Uw, false, freeM);
    }
    d[lane] = out;
}
}  // namespace dev
}  // namespace mw

extern "C" int mw_debug_lcp_solve(const float* A, const float* rhs, uint64_t free_mask, int32_t n, int32_t method,
                                  float* d) {
    // include/mwstep_testhooks.h: a test hook, not for a running simulator --
    // its own buffers and its own stream, and it waits on that stream only
    if (!A || !rhs || !d || n < 1 || n > mw::dev::kWaveMaxRows || method < 0 || method > 1) return 2;
    float *dA = nullptr, *dr = nullptr, *dd = nullptr;
    hipStream_t st = nullptr;
    const size_t nn = static_cast<size_t>(n) * n;
    int rc = 1;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess &&
        hipMalloc(reinterpret_cast<void**>(&dA), nn * sizeof(float)) == hipSuccess &&
        hipMalloc(reinterpret_cast<void**>(&dr), 64 * sizeof(float)) == hipSuccess &&
        hipMalloc(reinterpret_cast<void**>(&dd), 64 * sizeof(float)) == hipSuccess &&
        hipMemcpyAsync(dA, A, nn * sizeof(float), hipMemcpyHostToDevice, st) == hipSuccess &&
        hipMemcpyAsync(dr, rhs, n * sizeof(float), hipMemcpyHostToDevice, st) == hipSuccess) {
        const uint64_t live = (n >= 64) ? ~0ull : ((1ull << n) - 1ull);
        hipLaunchKernelGGL(mw::dev::debug_lcp_solve_kernel, dim3(1), dim3(64), 0, st, dA, dr, free_mask & live, n,
                           method, dd);
        if (hipGetLastError() == hipSuccess &&
            hipMemcpyAsync(d, dd, n * sizeof(float), hipMemcpyDeviceToHost, st) == hipSuccess &&
            hipStreamSynchronize(st) == hipSuccess)
            rc = 0;
    }
    if (st) (void)hipStreamSynchronize(st);
    (void)hipFree(dA);
    (void)hipFree(dr);
    (void)hipFree(dd);
    if (st) (void)hipStreamDestroy(st);
    return rc;
}
