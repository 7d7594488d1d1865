/*
 * mwstep.h -- C ABI of the MI355X many-worlds articulated-body stepper.
 *
 * This is the drop-in boundary that replaces the reference's ScenarI/O Gazebo
 * backend on the env-step hot path:
 *   GazeboRuntime.step()            python/gym_ignition/runtimes/gazebo_runtime.py:91-120
 *   -> scenario.GazeboSimulator.run cpp/scenario/gazebo/src/GazeboSimulator.cpp:202-251
 *   -> Physics system Update        cpp/scenario/plugins/Physics/Physics.cpp:646-685
 *   -> DART World::step             [EXT]
 * Every world of a simulator is one slot of structure-of-arrays device state;
 * one mw_run() steps all of them (the reference steps one ECM per world,
 * GazeboSimulator.cpp:435-488 / Physics.cpp:1832-1834).
 *
 * Conventions
 *   - every function returns MW_OK (0) or an MW_E* status; the message of the
 *     last failure on the calling thread is mw_last_error().  Bool-returning
 *     ScenarI/O calls map MW_OK -> true; getters that throw in the reference
 *     (exceptions::DOFMismatch etc., cpp/scenario/gazebo/include/scenario/
 *     gazebo/exceptions.h) map a failure to RuntimeError in the Python shim.
 *   - host buffers are double precision, row-major [n_worlds_in_range, n_dofs];
 *     device buffers are float32 and owned by the caller unless stated.
 *   - no torch or HIP types appear in these signatures; a HIP stream is passed
 *     as void*.
 */
#ifndef MWSTEP_H
#define MWSTEP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MW_OK 0
#define MW_EINVAL 1      /* bad argument (dof/world out of range, bad mode) */
#define MW_ESTATE 2      /* wrong lifecycle state (not initialized, ...)    */
#define MW_EPARSE 3      /* model file could not be parsed / unsupported    */
#define MW_EHIP 4        /* HIP runtime failure                            */
#define MW_ENOTFOUND 5   /* unknown joint / model / field name             */
#define MW_ECAPACITY 6   /* a per-step capacity was exceeded: contact points /
                            constraint rows were dropped (the step ran without
                            them; DART would have kept them)                */
#define MW_EDIVERGED 7   /* a world's state became non-finite in this run (the
                            run advanced every world; mw_diverged lists the
                            flagged ones) -- failure detection, SURVEY.md §5 */

/* JointControlMode, same numbering as scenario::core::JointControlMode
 * (cpp/scenario/core/include/scenario/core/Joint.h:37-75). */
#define MW_MODE_INVALID 0
#define MW_MODE_IDLE 1
#define MW_MODE_FORCE 2
#define MW_MODE_VELOCITY 3
#define MW_MODE_VELOCITY_FOLLOWER_DART 4
#define MW_MODE_POSITION 5
#define MW_MODE_POSITION_INTERPOLATED 6

/* JointType, same numbering as scenario::core::JointType (Joint.h:25-31). */
#define MW_JOINT_INVALID 0
#define MW_JOINT_FIXED 1
#define MW_JOINT_REVOLUTE 2
#define MW_JOINT_PRISMATIC 3
#define MW_JOINT_BALL 4
/* An SDF ball joint (3 dofs) is compiled as three revolute dofs named
 * <joint>#x, <joint>#y, <joint>#z: rotations about the x, y, z axes of the
 * joint frame at one point (intrinsic X-Y-Z angles), the first two on
 * massless links <joint>#x, <joint>#y; mw_joint_type reports MW_JOINT_BALL
 * for all three.  The ScenarI/O mirror (scenario/gazebo.py BallJoint)
 * presents them in DART's BallJoint coordinates (rotation vector, child-frame
 * angular velocity and torque). */

/* per-joint parameters that the reference lets a just-created model change
 * (Joint::setCoulombFriction / setViscousFriction / setMaxGeneralizedForce,
 * cpp/scenario/gazebo/src/Joint.cpp:258-318,622-640) */
#define MW_PARAM_COULOMB_FRICTION 0
#define MW_PARAM_VISCOUS_FRICTION 1
#define MW_PARAM_MAX_GENERALIZED_FORCE 2
#define MW_PARAM_POSITION_LIMIT_MIN 3
#define MW_PARAM_POSITION_LIMIT_MAX 4

typedef struct mw_sim mw_sim;
typedef struct mw_vecenv mw_vecenv;

typedef struct {
    double step_size;        /* GazeboSimulator(step_size, rtf, steps_per_run) */
    double rtf;              /* validated (> 0) like helpers.cpp:391-400;       */
                             /* no wall-clock throttling is performed           */
    int32_t steps_per_run;   /* physics substeps per mw_run (> 0)              */
    int32_t n_worlds;        /* parallel worlds on this device (>= 1)          */
    int32_t device;          /* HIP device ordinal                             */
    int32_t pgs_iters;       /* boxed-LCP sweeps per substep (0 -> 20)          */
} mw_config;

/* ---- lifecycle (GazeboSimulator ctor / initialize / close) ---- */
const char* mw_last_error(void);
const char* mw_version(void);
int mw_create(const mw_config* cfg, mw_sim** out);
void mw_destroy(mw_sim* sim);
/* Load the articulated model replicated into every world.  `urdf` is a file
 * path or an inline string holding a URDF <robot> or an SDF <model>; pose =
 * {x, y, z, qw, qx, qy, qz} (World::insertModel,
 * cpp/scenario/gazebo/src/World.cpp:70-180; for SDF the identity pose keeps
 * the model's own <pose>, any other replaces it, World.cpp:169-177). */
int mw_load_model(mw_sim* sim, const char* urdf, const double pose[7], const char* name);
int mw_initialize(mw_sim* sim);
int mw_initialized(const mw_sim* sim);
/* Optional: launch on an external stream (e.g. torch's current stream);
 * NULL selects the default stream.  Without this call the simulator creates
 * its own non-blocking stream at mw_initialize. */
int mw_set_stream(mw_sim* sim, void* hip_stream);

/* ---- stepping (GazeboSimulator::run) ---- */
/* Applies pending resets and commands, executes steps_per_run substeps unless
 * paused, refreshes the host-side readback, and blocks until done. */
int mw_run(mw_sim* sim, int paused);
/* `runs` x mw_run(sim, 0) with the state kept on the device: no readback and
 * no host synchronisation (graph-capturable; the getters read back lazily). */
int mw_run_device(mw_sim* sim, int32_t runs);
/* Simulated time in seconds after the last run (World::time, World.cpp:326-332). */
int mw_time(const mw_sim* sim, double* seconds);
int mw_set_gravity(mw_sim* sim, const double g[3]);
int mw_gravity(const mw_sim* sim, double g[3]);

/* ---- model / joint introspection ---- */
int mw_n_worlds(const mw_sim* sim, int32_t* n);
int mw_dofs(const mw_sim* sim, int32_t* n);
int mw_joint_name(const mw_sim* sim, int32_t dof, char* buf, int32_t buflen);
/* the (lumped) link moved by joint dof (Model::linkNames, Model.cpp:479-520) */
int mw_link_name(const mw_sim* sim, int32_t dof, char* buf, int32_t buflen);
int mw_joint_index(const mw_sim* sim, const char* name, int32_t* dof);
int mw_joint_type(const mw_sim* sim, int32_t dof, int32_t* type);
int mw_model_name(const mw_sim* sim, char* buf, int32_t buflen);
int mw_base_frame(const mw_sim* sim, char* buf, int32_t buflen);
int mw_set_joint_param(mw_sim* sim, int32_t dof, int32_t which, double value);
int mw_joint_param(const mw_sim* sim, int32_t dof, int32_t which, double* value);
/* Export the compiled tree (fp64) for cross-checks: per dof, in depth-first
 * body order, {jtype, limited, E[9], r[3], axis[3], mass, com[3], Ic[6],
 * damping, friction, lower, upper, effort, vel_limit, parent} = 34 doubles,
 * then gravity_base[3]. */
int mw_model_export(const mw_sim* sim, double* out, int32_t len);
/* The base of the compiled tree: {floating, base_R[9], base_p[3] (the model
 * frame in the world), base_mass, base_com[3], base_Ic[6]} = 23 doubles (the
 * inertia is zero for a fixed base). */
int mw_model_export_base(const mw_sim* sim, double out[23]);
/* Collision shapes of body `body` (-1 = the base), in its frame: per shape
 * {type (0 box, 1 sphere), size[3] (half extents / radius), R[9], p[3]} = 16
 * doubles; *count receives the number of shapes, at most `max_shapes` are
 * written (Physics.cpp:687-1219 creates one collision per <collision>). */
int mw_model_export_shapes(const mw_sim* sim, int32_t body, double* out, int32_t max_shapes, int32_t* count);
/* Compile a model (URDF / SDF file path or string; no simulator, no GPU) and
 * export every collision it holds, base first then by body, as the scene
 * kernel sees them (Physics.cpp:687-1219 builds one shape per <collision>;
 * meshes :897-931): per shape MW_COLLISION_WORDS doubles {body (-1 = base),
 * type (0 box, 1 sphere, 2 cylinder, 3 mesh), size[3], R[9], p[3], npts,
 * points[16][3]} -- a mesh's size is its bounding box half extents, p the box
 * centre, points its ground-contact support points in the shape frame
 * (gym-ignition_amd/csrc/mesh.cpp).  mw_sim: a floating model's mesh
 * contacts the ground at its support points (articulated: zero-radius
 * spheres; joint-less: free-body shape entries of <= 8 points), fixed-base
 * models drop mesh shapes. */
#define MW_COLLISION_WORDS 66
int mw_compile_collisions(const char* model, const double pose[7], double* out, int32_t max_shapes,
                          int32_t* count);

/* Copy of the float32 parameter block the kernels read (struct ChainF of
 * gym-ignition_amd/csrc/chain_params.hpp), for tests and tools. */
int mw_device_params(const mw_sim* sim, void* out, int32_t bytes);
/* the FloatF block (base inertia, shapes, contact slots) of an articulated
 * floating-base model, for the same test harness */
int mw_device_float_params(const mw_sim* sim, void* out, int32_t bytes);
/* Id of the shipped model whose parameter block the loaded model matches bit
 * for bit (1 cartpole, 2 pendulum): the batched env then runs a kernel with the
 * model constant-folded.  0 = generic kernel.  MWSTEP_DISABLE_BAKED=1 forces 0. */
int mw_baked_model(const mw_sim* sim, int32_t* id);

/* ---- batched ScenarI/O accessors over worlds [w0, w0 + nw) ----
 * dofs == NULL selects all dofs in model order (ndofs ignored). */
int mw_get_joint_positions(const mw_sim* sim, int32_t w0, int32_t nw, const int32_t* dofs, int32_t ndofs, double* out);
int mw_get_joint_velocities(const mw_sim* sim, int32_t w0, int32_t nw, const int32_t* dofs, int32_t ndofs, double* out);
int mw_get_joint_accelerations(const mw_sim* sim, int32_t w0, int32_t nw, const int32_t* dofs, int32_t ndofs, double* out);
int mw_get_joint_forces(const mw_sim* sim, int32_t w0, int32_t nw, const int32_t* dofs, int32_t ndofs, double* out);
int mw_get_joint_force_targets(const mw_sim* sim, int32_t w0, int32_t nw, const int32_t* dofs, int32_t ndofs, double* out);
int mw_get_joint_velocity_targets(const mw_sim* sim, int32_t w0, int32_t nw, const int32_t* dofs, int32_t ndofs, double* out);
int mw_get_joint_position_targets(const mw_sim* sim, int32_t w0, int32_t nw, const int32_t* dofs, int32_t ndofs, double* out);
int mw_set_joint_force_targets(mw_sim* sim, int32_t w0, int32_t nw, const int32_t* dofs, int32_t ndofs, const double* v);
int mw_set_joint_velocity_targets(mw_sim* sim, int32_t w0, int32_t nw, const int32_t* dofs, int32_t ndofs, const double* v);
int mw_set_joint_position_targets(mw_sim* sim, int32_t w0, int32_t nw, const int32_t* dofs, int32_t ndofs, const double* v);
int mw_reset_joint_positions(mw_sim* sim, int32_t w0, int32_t nw, const int32_t* dofs, int32_t ndofs, const double* v);
int mw_reset_joint_velocities(mw_sim* sim, int32_t w0, int32_t nw, const int32_t* dofs, int32_t ndofs, const double* v);
int mw_set_joint_control_mode(mw_sim* sim, int32_t w0, int32_t nw, const int32_t* dofs, int32_t ndofs, int32_t mode);
int mw_joint_control_mode(const mw_sim* sim, int32_t w, int32_t dof, int32_t* mode);

/* JointController PID of one dof, shared by all worlds of the simulator.
 * gains = {p, i, d, cmd_min, cmd_max, cmd_offset, i_min, i_max}, the field
 * order of scenario::core::PID (cpp/scenario/core/include/scenario/core/
 * Joint.h:505-523).  Replaces Joint::setPID / Joint::pid (Joint.cpp:466-525):
 * output limits less limiting than +-max generalized force are replaced by
 * them; the new PID starts from a reset state.  Default: Joint.cpp:63. */
int mw_set_joint_pid(mw_sim* sim, int32_t dof, const double gains[8]);
int mw_joint_pid(const mw_sim* sim, int32_t dof, double gains[8]);
/* Model::setControllerPeriod / controllerPeriod (Model.cpp:589-602, default
 * the maximum duration, Model.cpp:181-185): the PID force of Position /
 * Velocity joints is recomputed when at least one period of simulated time
 * has elapsed (JointController.cpp:130-169), else the last force is reused. */
int mw_set_controller_period(mw_sim* sim, double period);
int mw_controller_period(const mw_sim* sim, double* period);

/* ---- floating bases (root link not attached to "world": a DART FreeJoint
 * root).  This build steps single floating bodies and articulated models on
 * a floating base (any tree of <= 48 bodies), with box / sphere / cylinder
 * collision shapes on any link against a ground plane z = 0 and a contact LCP
 * with friction.  Fixed-base trees outside the compiled chain topologies run
 * on the same world-per-wavefront kernel with a welded base; for every
 * fixed-base model the base getters return the model frame at rest ---- */
int mw_is_floating(const mw_sim* sim, int32_t* floating);
/* Model::basePosition / baseOrientation: out [nw][7] = x y z qw qx qy qz. */
int mw_get_base_pose(const mw_sim* sim, int32_t w0, int32_t nw, double* out);
/* Model::baseWorldLinearVelocity / baseWorldAngularVelocity: out [nw][6] =
 * linear xyz (base origin), angular xyz, world frame. */
int mw_get_base_velocity(const mw_sim* sim, int32_t w0, int32_t nw, double* out);
/* Model::resetBasePose / resetBaseWorldVelocity (Model.cpp:256-400): applied by
 * the next run (pose first, then the velocity). */
int mw_reset_base_pose(mw_sim* sim, int32_t w0, int32_t nw, const double* pose);
int mw_reset_base_velocity(mw_sim* sim, int32_t w0, int32_t nw, const double* lin_ang);
/* Contact / joint-row solver options of the world-per-wavefront kernel
 * (articulated floating bases, generic fixed trees).  DART's primary boxed-LCP
 * solver is Dantzig's exact pivoting method [EXT]; the kernel runs projected
 * Gauss-Seidel sweeps (mw_config.pgs_iters).  tol > 0 ends the sweeps once a
 * sweep changed no row's constraint velocity (J dqd, m/s or rad/s) by more
 * than tol -- velocity space, where the redundant contact corners' null
 * directions do not count; warm_start != 0 starts
 * every row from the previous step's impulse of the same contact slot / joint
 * row (cold after a reset of the world).  Defaults: 0, 0 (a fixed sweep
 * count from zero).  Other kernels ignore the tolerance; warm_start != 0
 * fails with MW_ESTATE once an initialized simulator runs on another kernel
 * (they have no warm-start record). */
int mw_set_pgs_options(mw_sim* sim, double tol, int32_t warm_start);
int mw_pgs_options(const mw_sim* sim, double* tol, int32_t* warm_start);
/* The boxed-LCP solver of floating models.  MW_LCP_EXACT (default,
 * max_solves 48) solves the LCP as DART does: DART's primary solver is ODE's
 * Dantzig pivoting LCP [EXT], reached from ForwardStep (Physics.cpp:1824-1835),
 * whose friction index boxes every friction row once, by mu x the normal
 * impulses of the frictionless problem -- two strictly convex box QPs
 * (wave_lcp.hpp), each from the previous step's solution, PGS sweeps on the
 * stage's box problem (at most min(mw_config.pgs_iters, 4), ending once a
 * sweep moves no constraint velocity by more than 1e-6), then the primal
 * active-set method from the previous step's working set, with at most
 * max_solves dense linear solves (elimination over the wave's lanes) per
 * world-step.  It runs on the world-per-wavefront
 * kernel, which then steps every floating model (joint-less bodies, small
 * trees at any world count).  MW_LCP_PGS: the coupled PGS sweeps alone (cold
 * unless mw_set_pgs_options asks for the warm start); chosen before
 * mw_load_model it lets a joint-less body / small compiled tree take the
 * PGS-only lane kernels.  Selecting MW_LCP_EXACT for a model already loaded
 * onto a lane kernel fails with MW_ESTATE; mw_lcp_solver reports the solver
 * the model's kernel runs. */
#define MW_LCP_PGS 0
#define MW_LCP_EXACT 1
int mw_set_lcp_solver(mw_sim* sim, int32_t mode, int32_t max_solves);

/* Link::applyWorldWrench / applyWorldForce / applyWorldTorque
 * (cpp/scenario/gazebo/src/Link.cpp:484-560) on the worlds [w0, w0 + nw):
 * wrench[6 * nw] = world force at the link origin (xyz) and world torque
 * (xyz) per world, applied from the next physics step for
 * max(1, ceil(duration / dt)) steps; wrenches on one link add up (at most 4
 * distinct expiries at once).  link -1 = the base.  Carried by the
 * world-per-wavefront kernel (articulated floating bases, generic fixed-base
 * trees); other models fail with MW_ESTATE (use a scene).  Not seen by graphs
 * captured before the call. */
int mw_apply_link_wrench(mw_sim* sim, int32_t link, int32_t w0, int32_t nw, const double* wrench, double duration);
int mw_lcp_solver(const mw_sim* sim, int32_t* mode, int32_t* max_solves);
/* World-steps whose exact LCP solve ran out of budget since mw_initialize
 * (they keep their last impulses projected onto the friction boxes of their
 * normals and the joint rows' bounds: feasible, not optimal; 0 = every solve
 * converged).  64-bit device counters. */
int mw_lcp_unconverged(const mw_sim* sim, int64_t* world_steps);
/* The world's ground plane (z = 0, normal +z) and its friction coefficient. */
int mw_set_ground_plane(mw_sim* sim, int32_t enabled, double mu);
/* Model::enableContacts / contactsEnabled (Model.cpp:674-700). */
int mw_enable_contacts(mw_sim* sim, int32_t enable);
int mw_contacts_enabled(const mw_sim* sim, int32_t* enabled);
/* Contacts of world w after the last run (Physics.cpp:2351-2540): up to cap
 * rows of 10 doubles = point xyz, normal xyz (into the body), force on the
 * body xyz (N), penetration depth; *n = number of contact points. */
int mw_get_contacts(const mw_sim* sim, int32_t w, double* out, int32_t cap, int32_t* n);
/* The body of every contact point of mw_get_contacts, same order: -1 = the
 * base link, i >= 0 = the link moved by joint i (Link::contacts,
 * Link.cpp:365-440, collects the contacts of one link). */
int mw_get_contact_bodies(const mw_sim* sim, int32_t w, int32_t* bodies, int32_t cap, int32_t* n);
/* Articulated floating-base models: which kernel steps them -- 0 none (not
 * such a model), 1 one world per lane (small compiled trees), 2 one world per
 * wavefront (any tree of <= 48 bodies; MWSTEP_WAVE_TREE=1 forces it) -- and the
 * number of constraint rows the wave kernel dropped so far (its per-step
 * capacity is 64 active rows; 0 in every test and bench configuration).
 * mw_run returns MW_ECAPACITY when its run dropped rows (the state has
 * advanced without them); mw_run_device, which does not synchronise, leaves
 * the check to mw_constraint_overflow. */
int mw_float_kernel(const mw_sim* sim, int32_t* kind);
int mw_constraint_overflow(const mw_sim* sim, int64_t* rows);

/* Zero-copy device views, float32 [n_dofs][n_worlds] (world index fastest):
 * the SoA state "q", "qd", "qdd", and "position_target" (the Position-mode
 * targets; after the view is taken, writes through it drive the next runs
 * and the host getters/setters re-read the device copy). */
int mw_device_ptr(mw_sim* sim, const char* field, void** dptr, int64_t* world_stride);
/* Device-to-device copy of the SoA state ([n_dofs][n_worlds] float32 each) to
 * (to_sim = 0) or from (to_sim = 1) caller buffers, on the sim's stream. */
int mw_copy_state(mw_sim* sim, float* q_dev, float* qd_dev, int to_sim);

/* ---- failure detection and per-world snapshots ----
 * The run kernels flag a world (sticky) when the joint or base state they
 * store is not finite -- tested on the exponent bits, the kernels being
 * built finite-math-only -- and count the flagged worlds.  mw_run reads the
 * count back with its state and returns MW_EDIVERGED when new worlds were
 * flagged (the reference has no such check: GazeboSimulator::run,
 * GazeboSimulator.cpp:202-251, only reports a failed server step);
 * mw_run_device leaves the check to mw_diverged.  mw_diverged: flags[nw] of
 * worlds [w0, w0 + nw) (flags may be NULL) and the number of flag events
 * since mw_initialize (a world counts again each time it is flagged after
 * its flag was re-armed); mw_clear_diverged re-arms the flags of a range.
 * Any reset of a world's state re-arms its flag too: mw_reset_joint_positions
 * / _velocities, mw_reset_base_pose / _velocity and mw_set_state, so a world
 * that diverges, is reset and diverges again is reported again. */
int mw_diverged(mw_sim* sim, int32_t w0, int32_t nw, uint8_t* flags, int64_t* count);
int mw_clear_diverged(mw_sim* sim, int32_t w0, int32_t nw);
/* The full per-world record as float32 words, [nw][words] in host memory, in
 * this order: q, qd, qdd, then the JointController PID state pErrLast, iErr,
 * cmd, then qlo (the low word of the compensated joint positions) -- n_dofs
 * words each, absent for joint-less bodies -- then the base pose (x y z, qw qx
 * qy qz) and body-frame twist (w, v) (13 words, floating and welded-tree
 * models), then the previous step's constraint impulses that the wave
 * kernel's warm start / exact LCP starts from (its models only: the final
 * impulses, then the stage-1 impulses, per contact slot and joint row).
 * mw_set_state writes the record back (bit-exact: a restored world steps
 * exactly as it did from the saved state), drops the worlds' pending resets
 * and clears their divergence flags.  The simulator time, the controller
 * period gate and the commands / targets are not per-world state and are not
 * part of the record. */
int mw_state_words(const mw_sim* sim, int32_t* words);
int mw_get_state(mw_sim* sim, int32_t w0, int32_t nw, float* out);
int mw_set_state(mw_sim* sim, int32_t w0, int32_t nw, const float* in);

/* ---- batched environment (device-side Task logic) ----
 * Tasks mirror python/gym_ignition_environments/tasks/ (CartPole x3,
 * Pendulum); the TimeLimit of
 * the gym registration (max_episode_steps, __init__.py:14-52) and
 * auto-reset of done worlds (Philox4x32-10 keyed by seed) run in-kernel. */
#define MW_TASK_CARTPOLE_DISCRETE 0
#define MW_TASK_CARTPOLE_CONTINUOUS_BALANCING 1
#define MW_TASK_CARTPOLE_CONTINUOUS_SWINGUP 2
#define MW_TASK_PENDULUM_SWINGUP 3
/* Position-target control of the 9-dof Panda (BASELINE config 4): actions
 * float32 [n_worlds, 9] are the Position-mode targets of every joint, the
 * JointController PID (gains: mw_set_joint_pid) runs every physics step;
 * obs = [q, qd] (18), reward = -|q - target|^2, done = TimeLimit only; reset
 * to the Panda wrapper's pose (python/gym_ignition_environments/models/
 * panda.py:41-44) with joints 1 and 6 at mid-range (test_pid_controllers.py:
 * 49-59) and the fingers half open, + U(-0.05, 0.05) per joint. */
#define MW_TASK_PANDA_POSITION_TRACKING 4

typedef struct {
    int32_t kind;
    int32_t max_episode_steps;       /* 0 = no time limit                   */
    int32_t reward_cart_at_center;   /* CartPole balancing tasks            */
    int32_t world_offset;            /* global index of world 0 (sharding):  */
                                     /* reset streams do not depend on P     */
    uint64_t seed;
    /* Per-world physics randomisation, resampled at every (auto-)reset like
     * GazeboEnvRandomizer.reset (python/gym_ignition/randomizers/
     * gazebo_env_randomizer.py): MW_RAND_MASS adds max(U(mass_low, mass_high), 0)
     * to every moving body's mass (randomizers/cartpole.py:100-135 with
     * SDFRandomizer's force_positive, randomizers/model/sdf.py:294-295; COM and
     * rotational inertia unchanged), MW_RAND_GRAVITY sets the world gravity to
     * (0, 0, N(gravity_mean, gravity_std)) (randomizers/cartpole.py:51-56). */
    int32_t randomize;
    float mass_low, mass_high;
    float gravity_mean, gravity_std;
    int32_t pad_;
} mw_task_config;
#define MW_RAND_MASS 1
#define MW_RAND_GRAVITY 2

int mw_vecenv_create(mw_sim* sim, const mw_task_config* cfg, mw_vecenv** out);
void mw_vecenv_destroy(mw_vecenv* env);
int mw_vecenv_obs_dim(const mw_vecenv* env, int32_t* n);
/* Reset every world (episode 0); obs_dev float32 [n_worlds, obs_dim]. */
int mw_vecenv_reset(mw_vecenv* env, float* obs_dev);
/* One env step of every world, asynchronous on the sim's stream.
 *   actions_dev: int32 [n_worlds] (discrete), float32 [n_worlds], or
 *                float32 [n_worlds, dofs] (position-target tasks)
 *   obs_dev float32 [n_worlds, obs_dim]  (reset obs where done)
 *   reward_dev float32 [n_worlds], done_dev uint8 [n_worlds]
 *   terminal_obs_dev float32 [n_worlds, obs_dim] (written only where done) */
int mw_vecenv_step(mw_vecenv* env, const void* actions_dev, float* obs_dev, float* reward_dev,
                   uint8_t* done_dev, float* terminal_obs_dev);
/* T env steps fused in one launch (open loop: actions [T, n_worlds]); outputs
 * [T, ...]. */
int mw_vecenv_rollout(mw_vecenv* env, int32_t T, const void* actions_dev, float* obs_dev,
                      float* reward_dev, uint8_t* done_dev, float* terminal_obs_dev);
/* Copy the per-world episode / step counters (uint32 [n_worlds]) into caller
 * device buffers (async, on the sim's stream). */
int mw_vecenv_counters(mw_vecenv* env, uint32_t* episode_dev, uint32_t* steps_dev);
/* Copy the per-world randomised physics (body masses float32 [n_dofs][n_worlds],
 * gravity z float32 [n_worlds]) into caller device buffers; MW_ESTATE when the
 * env was created without randomisation. */
int mw_vecenv_physics(mw_vecenv* env, float* mass_dev, float* gravity_z_dev);

#ifdef __cplusplus
}
#endif
#endif /* MWSTEP_H */
