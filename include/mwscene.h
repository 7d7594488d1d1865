/*
 * mwscene.h -- C ABI of SCENES: several models in one world, batched over
 * many worlds (the scene kernel, gym-ignition_amd/csrc/scene.hip).
 *
 * Replaces, on the ScenarI/O path, what the reference does with one ECM per
 * world and one DART world per ECM:
 *   World::insertModel / removeModel    cpp/scenario/gazebo/src/World.cpp:394-464
 *   GazeboSimulator::insertWorldsFromSDF (N worlds per server)
 *                                       cpp/scenario/gazebo/src/GazeboSimulator.cpp:435-488
 *   Physics::CreatePhysicsEntities      cpp/scenario/plugins/Physics/Physics.cpp:687-1219
 *   Physics::UpdatePhysics / Step / UpdateSim / UpdateCollisions
 *                                       Physics.cpp:1299-1835, 1871-2540
 *   Link::applyWorldForce / Torque / Wrench, ExternalWorldWrenchCmdWithDuration
 *                                       Link.cpp:484-560, Physics.cpp:1446-1525
 *   JointController (PID, period gating) JointController.cpp:114-331
 * Models are trees on a fixed or floating base (URDF or SDF) with box /
 * sphere / cylinder collision shapes; they touch the ground plane, and the
 * box-box, box-sphere, sphere-sphere and cylinder-sphere pairs of different
 * models of a world touch each other (DART + ODE collision detector [EXT];
 * cylinder-box and cylinder-cylinder pairs are not collided in this build).  A model inserted into
 * some worlds of a scene is absent from the others.
 *
 * Indexing: models in insertion order; joints ("dofs") numbered globally,
 * model by model (mw_scene_model_info gives each model's first dof); links of
 * a model: -1 = the base link, i = the link moved by the model's joint i.
 * Conventions as mwstep.h: status codes + mw_last_error(), host buffers
 * double, row-major [worlds][items].
 */
#ifndef MWSCENE_H
#define MWSCENE_H

#include <stdint.h>

#include "mwstep.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mw_scene mw_scene;

/* joint data fields of mw_scene_get_joints / mw_scene_set_joints */
#define MW_SC_POSITION 0          /* get                                      */
#define MW_SC_VELOCITY 1          /* get                                      */
#define MW_SC_ACCELERATION 2      /* get                                      */
#define MW_SC_FORCE_TARGET 3      /* get / set (Joint::setGeneralizedForceTarget) */
#define MW_SC_VELOCITY_TARGET 4   /* get / set                                */
#define MW_SC_POSITION_TARGET 5   /* get / set                                */
#define MW_SC_RESET_POSITION 6    /* set (Joint::resetPosition)               */
#define MW_SC_RESET_VELOCITY 7    /* set                                      */
#define MW_SC_FORCE 8             /* get: joint force readback (0 after DART's step) */

/* cfg: step_size, rtf, steps_per_run, n_worlds, device, pgs_iters (as mw_create) */
int mw_scene_create(const mw_config* cfg, mw_scene** out);
void mw_scene_destroy(mw_scene* sc);
int mw_scene_set_stream(mw_scene* sc, void* hip_stream);
/* World::insertModel into worlds [w0, w0 + nw): compile `urdf` (path or
 * inline string) at pose {x, y, z, qw, qx, qy, qz}; the model is absent from
 * the other worlds.  Allowed before and after runs; the state of the models
 * already in the scene is kept.  *model = its index. */
int mw_scene_insert_model(mw_scene* sc, const char* urdf, const double pose[7], const char* name, int32_t w0,
                          int32_t nw, int32_t* model);
/* In worlds [w0, w0 + nw): World::removeModel (present = 0), re-insertion at
 * the insertion pose with zero joint state (present = 1), or resuming a
 * removed model with its state kept (present = 2; e.g. a world whose physics
 * system is inserted late). */
int mw_scene_set_present(mw_scene* sc, int32_t model, int32_t w0, int32_t nw, int32_t present);
int mw_scene_present(const mw_scene* sc, int32_t model, int32_t w, int32_t* present);
/* Swap the definition of a model that is in no world for another URDF with
 * the same tree and collision shapes (inertias, joint parameters, pose and
 * name may differ): the per-episode model of an env randomizer
 * (python/gym_ignition/randomizers/gazebo_env_randomizer.py) reuses its slot. */
int mw_scene_replace_model(mw_scene* sc, int32_t model, const char* urdf, const double pose[7], const char* name);
/* the ground plane (a static model with a plane collision) of worlds [w0, w0 + nw) */
int mw_scene_set_world_ground(mw_scene* sc, int32_t w0, int32_t nw, int32_t enabled);
int mw_scene_n_worlds(const mw_scene* sc, int32_t* n);
int mw_scene_n_models(const mw_scene* sc, int32_t* n);
/* first global dof, dof count, floating base (1) or welded (0) */
int mw_scene_model_info(const mw_scene* sc, int32_t model, int32_t* first_dof, int32_t* n_dofs, int32_t* floating);
int mw_scene_model_name(const mw_scene* sc, int32_t model, char* buf, int32_t len);
int mw_scene_base_frame(const mw_scene* sc, int32_t model, char* buf, int32_t len);
int mw_scene_joint_name(const mw_scene* sc, int32_t dof, char* buf, int32_t len);
int mw_scene_link_name(const mw_scene* sc, int32_t dof, char* buf, int32_t len);
int mw_scene_joint_type(const mw_scene* sc, int32_t dof, int32_t* type);
/* per body of the model, 34 doubles (the layout of mw_model_export, parent
 * = model-local index), then gravity in the base frame (3); with len >=
 * 34 n + 7 also the base link's mass and COM (base frame) */
int mw_scene_model_export(const mw_scene* sc, int32_t model, double* out, int32_t len);

/* GazeboSimulator::run: pending resets and commands, steps_per_run physics
 * steps of every world (unless paused); getters read back lazily. */
int mw_scene_run(mw_scene* sc, int32_t paused);
/* `runs` unpaused runs without host synchronisation (graph-capturable when
 * no command is pending) */
int mw_scene_run_device(mw_scene* sc, int32_t runs);
int mw_scene_time(const mw_scene* sc, double* seconds);
int mw_scene_set_gravity(mw_scene* sc, const double g[3]);
/* World::setGravity / gravity of single worlds (World.cpp:301-319: each world
 * keeps its own Gravity component); mw_scene_set_gravity sets every world. */
int mw_scene_set_world_gravity(mw_scene* sc, int32_t w0, int32_t nw, const double g[3]);
int mw_scene_world_gravity(const mw_scene* sc, int32_t w, double g[3]);
/* Friction coefficient of the ground plane of single worlds (every contact of
 * those worlds uses it); mw_scene_set_ground_plane sets every world's. */
int mw_scene_set_world_friction(mw_scene* sc, int32_t w0, int32_t nw, double mu);
/* Boxed-LCP solver of the scene kernel (as mw_set_lcp_solver): MW_LCP_EXACT
 * (default, 48 linear solves per world-step) solves the contact / joint LCP
 * exactly after the PGS sweeps when a world has <= 64 rows (worlds with more
 * rows keep the sweeps and are counted); MW_LCP_PGS: the sweeps alone. */
int mw_scene_set_lcp_solver(mw_scene* sc, int32_t mode, int32_t max_solves);
int mw_scene_lcp_solver(const mw_scene* sc, int32_t* mode, int32_t* max_solves);
/* World-steps whose exact solve ran out of budget (or had > 64 rows). */
int mw_scene_lcp_unconverged(const mw_scene* sc, int64_t* world_steps);
/* Failure detection (as mw_diverged): the scene kernel flags a world whose
 * stored joint or base state is not finite; mw_scene_run returns MW_EDIVERGED
 * when the run flagged new worlds (ScenarI/O run() -> false).  A joint or
 * base reset (mw_scene_set_joints with a reset field, mw_scene_reset_base_*),
 * inserting a model into a world or removing it re-arms the world's flag, so
 * a world that diverges again after a reset is reported again; the count is
 * of flag events. */
int mw_scene_diverged(mw_scene* sc, int32_t w0, int32_t nw, uint8_t* flags, int64_t* count);
int mw_scene_clear_diverged(mw_scene* sc, int32_t w0, int32_t nw);
int mw_scene_gravity(const mw_scene* sc, double g[3]);
/* the ground plane's friction, and the plane in (enabled) or out of every world */
int mw_scene_set_ground_plane(mw_scene* sc, int32_t enabled, double mu);

/* joints over worlds [w0, w0 + nw), dofs == NULL: every dof */
int mw_scene_get_joints(const mw_scene* sc, int32_t field, int32_t w0, int32_t nw, const int32_t* dofs, int32_t ndofs,
                        double* out);
int mw_scene_set_joints(mw_scene* sc, int32_t field, int32_t w0, int32_t nw, const int32_t* dofs, int32_t ndofs,
                        const double* v);
int mw_scene_set_control_mode(mw_scene* sc, int32_t w0, int32_t nw, const int32_t* dofs, int32_t ndofs, int32_t mode);
int mw_scene_control_mode(const mw_scene* sc, int32_t w, int32_t dof, int32_t* mode);
int mw_scene_set_joint_pid(mw_scene* sc, int32_t dof, const double gains[8]);
int mw_scene_joint_pid(const mw_scene* sc, int32_t dof, double gains[8]);
int mw_scene_set_joint_param(mw_scene* sc, int32_t dof, int32_t which, double value);
int mw_scene_joint_param(const mw_scene* sc, int32_t dof, int32_t which, double* value);
int mw_scene_set_controller_period(mw_scene* sc, int32_t model, double period);
int mw_scene_controller_period(const mw_scene* sc, int32_t model, double* period);

/* bases: pose [nw][7] x y z qw qx qy qz; velocity [nw][6] world linear (of
 * the base origin), world angular.  Resets are applied by the next run. */
int mw_scene_get_base_pose(const mw_scene* sc, int32_t model, int32_t w0, int32_t nw, double* out);
int mw_scene_get_base_velocity(const mw_scene* sc, int32_t model, int32_t w0, int32_t nw, double* out);
int mw_scene_reset_base_pose(mw_scene* sc, int32_t model, int32_t w0, int32_t nw, const double* pose);
int mw_scene_reset_base_velocity(mw_scene* sc, int32_t model, int32_t w0, int32_t nw, const double* lin_ang);

/* Contacts of world w after the last unpaused run, rows of 14 doubles:
 * point xyz, normal xyz (from body B into body A), force on A xyz (N),
 * depth, model A, link A, model B (-1: the ground plane), link B. */
int mw_scene_get_contacts(const mw_scene* sc, int32_t w, double* out, int32_t cap, int32_t* n);
/* Link::applyWorldWrench for worlds [w0, w0 + nw): wrench [nw][6] = world
 * force (applied at the link origin) and world torque, active for
 * max(1, ceil(duration / step_size)) physics steps from the next one. */
int mw_scene_apply_world_wrench(mw_scene* sc, int32_t model, int32_t link, int32_t w0, int32_t nw,
                                const double* wrench, double duration);
/* contact points / constraint rows dropped so far (per-step capacity).
 * mw_scene_run returns MW_ECAPACITY when its run dropped any (the state has
 * advanced; the error says how many were dropped); mw_scene_run_device, which
 * does not synchronise, leaves the check to this counter. */
int mw_scene_overflow(const mw_scene* sc, int64_t* dropped);

#ifdef __cplusplus
}
#endif
#endif /* MWSCENE_H */
