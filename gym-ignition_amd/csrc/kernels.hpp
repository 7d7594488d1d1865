// kernels.hpp -- host-callable launchers of the HIP kernels (kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "chain_params.hpp"

namespace mw {

// SoA device state of a simulator: every array is [n_dofs][n_worlds].
struct SimDev {
    float* q = nullptr;
    float* qd = nullptr;
    float* qdd = nullptr;
    float* cmd = nullptr;     // JointForceCmd (consumed by the next substep)
    float* vtgt = nullptr;   // JointVelocityTarget (VelocityFollowerDart)
    float* rq = nullptr;     // JointPositionReset values
    float* rqd = nullptr;    // JointVelocityReset values
    float* ptgt = nullptr;   // JointPositionTarget (Position mode)
    uint8_t* act = nullptr;  // kActForce / kActServo / kActPidPos / kActPidVel
    uint8_t* rflag = nullptr;  // bit0 position reset, bit1 velocity reset, bit2 PID reset pending
    // JointPID state (ignition::math::PID pErrLast, iErr, cmd), device only
    float* pid_e = nullptr;
    float* pid_i = nullptr;
    float* pid_u = nullptr;
    // low word of the joint positions (q = q_hi + qlo, compensated position
    // integration): the PID error q - target is formed from both, so its
    // derivative term (gain d / dt on the position error) does not amplify
    // the float32 rounding of q += dt qd (kernels with a JointController)
    float* qlo = nullptr;
    // divergence detection (mw_diverged): [W] sticky per-world flag set by the
    // run kernels when a world's stored joint or base state is not finite,
    // and the count of worlds flagged since initialisation
    uint8_t* div = nullptr;
    unsigned long long* ndiv = nullptr;
};

// Device arrays of a floating single-body model (free_body.hpp).
struct FreeDev {
    float* base = nullptr;     // [13][W]: p xyz, q wxyz, twist (body frame) w xyz, v xyz
    float* rpose = nullptr;    // [7][W] pending base pose reset (p, q wxyz)
    float* rvel = nullptr;     // [6][W] pending base velocity reset (world linear, world angular)
    uint8_t* rflag = nullptr;  // [W] bit0 pose reset, bit1 velocity reset
    float* cdata = nullptr;    // [kMaxFreeSlots][7][W] contact point xyz, force xyz, depth
    uint32_t* cmask = nullptr; // [W] active contact slots
    float* warm = nullptr;     // [kWaveWarmWords][W] previous step's PGS impulses (wave kernel, warm start)
    // world wrenches of the launch's substeps (wave kernel, mw_apply_link_wrench):
    // [6][node][W], world force at the link origin and world torque, node 0 the
    // base, 1 + i body i (the host splits launches where a wrench expires)
    float* wrench = nullptr;
    int32_t wnodes = 0;
    uint8_t* div = nullptr;               // as SimDev::div / ndiv
    unsigned long long* ndiv = nullptr;
};
constexpr int kSimWrenchSlots = 4;  // concurrent wrenches (distinct expiries) per link

// One launch of the scenario kernel covers up to 64 substeps of a run.
struct RunArgs {
    float dt, inv_dt;
    int substeps;         // substeps of this launch (<= 64)
    int paused;
    int pgs_iters;
    int first;            // first launch of the run: resets + force commands apply
    uint64_t pid_gate;    // bit s: the JointController computes a new PID force at substep s
    float pgs_tol;        // > 0: a PGS sweep that moved no impulse by more than pgs_tol max|x| ends the solve
    int warm;             // PGS starts from the previous step's impulses (wave kernel)
    int lcp_solves;       // > 0: the wave kernel solves its boxed LCP exactly within that many linear solves
    int wrenches;         // FreeDev::wrench holds this launch's world wrenches
};

// Task description for the device-side env (see sim.cpp for the sources).
struct TaskF {
    int32_t kind;
    int32_t max_steps;
    int32_t reward_cart_at_center;
    int32_t n_obs;
    uint32_t seed_lo, seed_hi;
    uint32_t world_offset;
    uint32_t pad_;
    float force_mag;
    float x_factor;   // reward rail factor (0.9 / 1.0 / 0.8)
    float hi[4];      // float32 bounds of the done-space (reset_space / observation_space)
    // position-target tasks (kind 4): reset pose and half-width of its uniform noise
    float home[kMaxKernelDofs];
    float home_noise;
    // per-world physics randomisation, resampled at every reset
    // (gym_ignition_environments/randomizers/cartpole.py:51-56, 100-135)
    int32_t randomize;     // bit 0: body masses, bit 1: gravity
    float mass_lo, mass_hi;  // additive mass sample U(lo, hi), clipped at 0 (force_positive)
    float g_mean, g_std;     // world gravity z ~ N(mean, std)
    float gdir[3];           // the world z axis in the base frame (gravity = gz * gdir)
};
enum : int32_t { kRandMass = 1, kRandGravity = 2 };

struct VecDev {
    uint32_t* episode = nullptr;
    uint32_t* steps = nullptr;
    float* rmass = nullptr;  // [n_dofs][W] per-world body masses (randomised tasks)
    float* rgz = nullptr;    // [W] per-world gravity z
};

// Returns hipSuccess or the launch error.
// topology id of a model's parent list: 0 = serial chain, 1 = Panda tree,
// 2 = quadruped (floating base), -1 = not compiled into this build
int kernel_topology(const int* parents, int n);

hipError_t launch_scenario_run(const ChainF* P, int n, int topo, bool cons, bool dual, int baked, const SimDev& S,
                               const PidSet& pid, int W, const RunArgs& a, hipStream_t st);

// F: the model's FreeF block in device memory (free_body.hpp)
hipError_t launch_free_run(const struct FreeF* F, const FreeDev& D, int W, const RunArgs& a, int contacts, int mesh,
                           hipStream_t st);

// Articulated model on a floating base (float_tree.hpp); F: its FloatF block
// in device memory, ws: FloatWs words per world x W floats (device).
hipError_t launch_float_run(const ChainF* P, int n, int topo, bool cons, const struct FloatF* F, const SimDev& S,
                            const FreeDev& D, const PidSet& pid, float* ws, int W, const RunArgs& a, int contacts,
                            hipStream_t st);
// Large floating-base trees, one world per wavefront (wave_tree.hpp): any
// topology of <= kMaxBodies bodies and depth <= 12; pid: n PidF in device
// memory; overflow: device counter of constraint rows dropped (> 64 per step).
// depth: the tree's depth in joints (the <= 16-body instance takes <= 10)
hipError_t launch_wave_run(const ChainF* P, int n, int depth, bool cons, const struct FloatF* F, const SimDev& S,
                           const FreeDev& D, const PidF* pid, int W, const RunArgs& a, int contacts, int* overflow,
                           hipStream_t st);
constexpr int kWaveMaxDepthHost = 12;
// words of the wave kernel's warm-start record per world (wave_tree.hpp
// kWaveWarmRecord: the final impulses, then the exact solve's stage-1 impulses)
constexpr int kWaveWarmWordsHost = 2 * (3 * 32 + 3 * kMaxBodies);
// workspace words per world of a floating-tree model, -1 if n is not compiled in
int float_workspace_words(int n, int n_slots);

hipError_t launch_vecenv_reset(const ChainF* P, int n, const TaskF& T, const SimDev& S,
                               const VecDev& V, float* obs, int W, hipStream_t st);

// Position-target task (kind 4, Panda): actions float32 [W, n] are the
// JointController position targets; PID every substep (period = step size).
hipError_t launch_vecenv_pid_step(const ChainF* P, int n, int topo, bool cons, bool dual, int baked, const TaskF& T,
                                  const SimDev& S, const VecDev& V, const PidSet& pid, const float* targets,
                                  float* obs, float* reward, uint8_t* done, float* term_obs, int W,
                                  float dt, int substeps, int pgs_iters, hipStream_t st);

// The same task with one world per 16-lane row (group_kernel.hip): any
// fixed-base tree of <= kMaxKernelDofs bodies numbered depth-first, with the
// row topology words of the parameter block filled (group_topology_words).
// lt: per-dof PID gains and reset pose in device memory (one record per lane).
struct GLaneTask {
    PidF pid;
    float home;
    float pad_[3];
};
hipError_t launch_vecenv_pid_group(const ChainF* P, int n, bool cons, bool dual, const TaskF& T, const SimDev& S,
                                   const VecDev& V, const GLaneTask* lt, const float* targets, float* obs,
                                   float* reward, uint8_t* done, float* term_obs, int W, float dt, int substeps,
                                   int pgs_iters, hipStream_t st);

// T_steps == 0: one step with the per-step output layout; otherwise a fused
// open-loop rollout of T_steps steps ([T, W] inputs and outputs).
// baked: id of a bit-identical shipped model (baked_models.hpp) or 0 (generic)
hipError_t launch_vecenv_step(const ChainF* P, int n, bool cons, bool dual, int baked, const TaskF& T,
                              const SimDev& S, const VecDev& V, const void* actions, float* obs,
                              float* reward, uint8_t* done, float* term_obs, int W, float dt,
                              int substeps, int pgs_iters, int T_steps, hipStream_t st);

}  // namespace mw
