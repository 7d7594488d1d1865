/*
 * oracle.h -- fp64 CPU restatement of the reference's physics step.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the
 * checker.  The product (gym-ignition_amd/) never links or calls it.
 *
 * What it restates (see oracle.c for line-level citations):
 *   - ScenarI/O Physics system step order: resets -> commands -> engine step ->
 *     readback -> zero-fill of force commands
 *     (/root/reference/cpp/scenario/plugins/Physics/Physics.cpp:646-685,
 *      :1330-1440, :2226-2345).
 *   - DART 6.x World::step [EXT, not vendored in the reference]: articulated
 *     body algorithm with implicit joint damping, semi-implicit Euler,
 *     joint-space constraint impulses (position limits, Coulomb friction,
 *     servo = VelocityFollowerDart) solved as a boxed LCP.
 *
 * Parity status: pinned against the reference's analytic pendulum
 * (tests/.python/test_pendulum_wrt_ground_truth.py:53-67) and the reference
 * KATs listed in DESIGN.md; trajectory-level parity vs DART itself is
 * "parity unpinned" (DART/Ignition are absent from this image).
 */
#ifndef MW_ORACLE_H
#define MW_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OR_MAXB 48

/* Fixed-base kinematic tree, one dof per body.  parent[i] < i (bodies in
 * depth-first order, -1 = the fixed base body); a serial chain has
 * parent[i] == i - 1. */
typedef struct {
    int32_t n;                   /* moving bodies == dofs                      */
    int32_t jtype[OR_MAXB];      /* 0 revolute, 1 prismatic                    */
    int32_t limited[OR_MAXB];    /* position limits enforced                   */
    int32_t parent[OR_MAXB];     /* parent body index, -1 = base               */
    int32_t pad_;
    double gravity_base[3];      /* gravity expressed in the base link frame   */
    double E[OR_MAXB][9];        /* joint origin rotation in parent (row-major) */
    double r[OR_MAXB][3];        /* joint origin translation in parent         */
    double axis[OR_MAXB][3];     /* joint axis in child frame (unit)           */
    double mass[OR_MAXB];
    double com[OR_MAXB][3];      /* COM in body frame                          */
    double Ic[OR_MAXB][6];       /* inertia about COM: xx yy zz xy xz yz       */
    double damping[OR_MAXB];
    double friction[OR_MAXB];    /* Coulomb                                    */
    double lower[OR_MAXB];
    double upper[OR_MAXB];
    double effort[OR_MAXB];
    double vel_limit[OR_MAXB];
} or_model;

/* joint actuation as seen by the engine (DART actuator types) */
enum { OR_PASSIVE = 0, OR_FORCE = 1, OR_SERVO = 2 };

/* ABA forward dynamics with DART's implicit damping term (dt_implicit = 0
 * gives the plain ABA).  tau is the total applied generalized force. */
void or_aba(const or_model* m, const double* q, const double* qd,
            const double* tau, double dt_implicit, double* qdd);

/* Composite-rigid-body mass matrix (independent algorithm; test cross-check). */
void or_crba(const or_model* m, const double* q, double* M /* n*n */);

/* Recursive Newton-Euler inverse dynamics: tau = M qdd + C(q,qd) + g(q). */
void or_rnea(const or_model* m, const double* q, const double* qd,
             const double* qdd, double* tau);

/* One engine step (DART World::step restated).
 *   mode[i]      OR_PASSIVE / OR_FORCE / OR_SERVO
 *   cmd[i]       force command (FORCE) or velocity command (SERVO)
 *   qdd_out[i]   joint acceleration readback (includes impulse/dt)
 *   force_out[i] joint force readback (applied + constraint impulse/dt)
 * q and qd are updated in place.  Returns the number of active LCP rows. */
int or_step(const or_model* m, double dt, double* q, double* qd,
            const int32_t* mode, const double* cmd, int pgs_iters,
            double* qdd_out, double* force_out);

/* Boxed LCP by projected Gauss-Seidel (A row-major n*n).  Every solver of
 * this oracle takes a sweep budget: iters >= 0 runs exactly that many sweeps
 * (the GPU kernels' count); iters < 0 (OR_PGS_CONVERGED) sweeps to the fixed
 * point (largest change of a sweep <= 1e-13 (1 + max|x|)).  or_pgs_stats():
 * sweeps and last change of the latest solve. */
#define OR_PGS_CONVERGED (-1)
void or_pgs(int n, const double* A, const double* b, const double* lo,
            const double* hi, double* x, int iters);
void or_pgs_stats(int* sweeps, double* last_delta);
/* test hook: the latest floating-tree LCP and its solution (n rows, or -n if cap < n) */
int or_lcp_last(int cap, double* A, double* b, double* lo, double* hi, int* kind, double* x, double* mu);
/* Row identities of the same capture (the kernels' warm-record index: contact
 * slot rows 3 slot + d, joint rows OR_WARM_JOINT0 + 3 dof + type; -1 when the
 * step has none), the converged mode's stage-1 impulses (DART's frictionless
 * stage; 0 on friction rows, 0 everywhere after a PGS-only solve) and per row
 * the magnitude of the terms b_r is formed from (sum_e |J_re nu_e| plus the
 * bias velocity).  A step without rows leaves no capture (count 0).  Returns
 * the row count (-count when cap is too small). */
int or_lcp_last_rows(int cap, int32_t* wid, double* x1, double* bscale);
/* tests: perturb the Delassus matrix of every exact LCP solve (0 = off) */
void or_set_lcp_perturbation(double eps, uint64_t seed);

/* Joint PID of the ScenarI/O JointController (Position / Velocity modes,
 * cpp/scenario/plugins/JointController/JointController.cpp:129-190). */
typedef struct {
    double p, i, d, imax, imin, cmdmax, cmdmin, offset;
} or_pid_gains;
typedef struct {
    double perr_last, ierr, cmd;
} or_pid_state;
double or_pid_update(const or_pid_gains* g, or_pid_state* s, double err, double dt);

/* ------------------------------------------------------------------ */
/* Floating rigid body with ground-plane contacts (DART FreeJoint +     */
/* ContactConstraint [EXT], Physics.cpp:2351-2540 contact readback).    */
/* ------------------------------------------------------------------ */
#define OR_MAXSHAPES 8
#define OR_MAXCONTACTS (8 * OR_MAXSHAPES)

typedef struct {
    double mass;
    double com[3];              /* body frame                                */
    double Ic[6];               /* about the COM: xx yy zz xy xz yz          */
    int32_t n_shapes;
    int32_t ground;             /* 1: ground plane z = 0, normal +z           */
    int32_t shape_type[OR_MAXSHAPES];   /* 0 box (size = half extents), 1 sphere */
    double shape_size[OR_MAXSHAPES][3];
    double shape_R[OR_MAXSHAPES][9];    /* shape pose in the body frame          */
    double shape_p[OR_MAXSHAPES][3];
    double gravity[3];          /* world frame                                */
    double mu;                  /* Coulomb friction with the ground           */
    /* type 3: mesh support points of the shape entry (<= 8, shape frame) */
    int32_t mesh_npts[OR_MAXSHAPES];
    double mesh_pt[OR_MAXSHAPES][8][3];
} or_free_model;

typedef struct {
    double p[3];                /* body origin, world frame                   */
    double R[9];                /* body orientation (row-major)               */
    double w[3];                /* angular velocity, BODY frame (FreeJoint)   */
    double v[3];                /* linear velocity of the origin, BODY frame  */
} or_free_state;

/* One engine step of a free body.  Contacts (world frame, force acting on
 * the body, impulse / dt) are written to c_* (capacity OR_MAXCONTACTS);
 * returns their number. */
int or_free_step(const or_free_model* m, double dt, or_free_state* s, int pgs_iters,
                 double* c_pos, double* c_normal, double* c_force, double* c_depth);

/* ------------------------------------------------------------------ */
/* Articulated floating base (DART FreeJoint root + tree) with ground   */
/* contacts: dense formulation (CRBA + RNEA + dense LCP), independent   */
/* of the device's recursive one.                                       */
/* ------------------------------------------------------------------ */
#define OR_MAXFS 16
#define OR_MAXFC (8 * OR_MAXFS)
#define OR_MESH_MAXP 16
#define OR_HULL_MAXF 32   /* faces of a hull of <= OR_MESH_MAXP points (<= 2 n - 4 triangles) */
#define OR_HULL_MAXE 48   /* edges (<= 3 n - 6) */

typedef struct {
    or_model tree;               /* moving bodies; parent -1 = the base body  */
    double base_mass;
    double base_com[3];
    double base_Ic[6];
    int32_t n_shapes;
    int32_t ground;
    int32_t shape_body[OR_MAXFS];        /* -1 = base                        */
    int32_t shape_type[OR_MAXFS];        /* 0 box (half extents), 1 sphere,  */
                                         /* 2 cylinder, 3 mesh               */
    double shape_size[OR_MAXFS][3];
    double shape_R[OR_MAXFS][9];
    double shape_p[OR_MAXFS][3];
    double gravity[3];           /* world frame                               */
    double mu;
    /* type 3 mesh (scenes only): size = half extents of its bounding box (the
     * shape frame sits at the box centre), ground-contact support points in
     * the shape frame */
    int32_t shape_npts[OR_MAXFS];
    double shape_pts[OR_MAXFS][OR_MESH_MAXP][3];
} or_float_model;

typedef struct {
    double p[3];
    double R[9];
    double V[6];                 /* base twist, body frame [w; v]             */
    double q[OR_MAXB];
    double qd[OR_MAXB];
} or_float_state;

/* One engine step; mode / cmd as or_step (joint actuation).  Contacts as
 * or_free_step (point, normal +z, force on the body, depth) plus the body
 * index (-1 = base) in c_body.  Returns the number of contact points. */
int or_float_step(const or_float_model* m, double dt, or_float_state* s, const int32_t* mode,
                  const double* cmd, int pgs_iters, double* c_pos, double* c_force, double* c_depth,
                  int32_t* c_body);
/* or_float_step with the kernels' solver options: pgs_tol > 0 ends the sweeps
 * once a sweep changed no row's constraint velocity (A x)_r by more than
 * pgs_tol; warm (NULL:
 * cold) holds the previous step's impulses by row identity (3 slot + d for
 * contact slots, OR_WARM_JOINT0 + 3 dof + t for joint rows) and receives this
 * step's. */
#define OR_WARM_SLOTS OR_MAXFC
#define OR_WARM_JOINT0 (3 * OR_WARM_SLOTS)
#define OR_WARM_WORDS (OR_WARM_JOINT0 + 3 * OR_MAXB)
int or_float_step_warm(const or_float_model* m, double dt, or_float_state* s, const int32_t* mode,
                       const double* cmd, int pgs_iters, double pgs_tol, double* warm, double* c_pos,
                       double* c_force, double* c_depth, int32_t* c_body);

/* CPU-baseline rollouts under the JointController PID hold (bench.py):
 * W fixed-base worlds (q, qd, q0, PID states [W][n]; targets
 * q0 + amp sin(2 pi freq t)), or one floating-base world (fixed targets). */
void or_pid_rollout(const or_model* m, double dt, int W, int T, double* q, double* qd, const double* q0,
                    const double* amp, double freq, const or_pid_gains* g, or_pid_state* st, int pgs_iters);
void or_float_pid_rollout(const or_float_model* m, double dt, int T, or_float_state* s, const double* target,
                          const or_pid_gains* g, or_pid_state* st, int pgs_iters);

/* Floating-base mass matrix ((6+n)^2, row-major) and bias h (gravity +
 * velocity products) at a state (test cross-checks). */
void or_float_dynamics(const or_float_model* m, const or_float_state* s, double* M, double* h);

/* ------------------------------------------------------------------ */
/* Batched environment (task logic of the reference's CartPole /      */
/* Pendulum tasks + gym TimeLimit + auto-reset with Philox4x32-10).   */
/* ------------------------------------------------------------------ */
enum {
    OR_TASK_CARTPOLE_DISCRETE = 0,
    OR_TASK_CARTPOLE_CONTINUOUS_BALANCING = 1,
    OR_TASK_CARTPOLE_CONTINUOUS_SWINGUP = 2,
    OR_TASK_PENDULUM_SWINGUP = 3,
};

typedef struct {
    int32_t kind;
    int32_t steps_per_run;
    int32_t max_episode_steps;      /* 0 = no TimeLimit                        */
    int32_t reward_cart_at_center;
    double dt;
    uint64_t seed;
    /* per-world physics randomisation (bit 0 masses, bit 1 gravity), sampled
     * from (world, episode): randomizers/cartpole.py:51-56, 100-135 */
    int32_t randomize;
    /* global index of world 0 of this env (a rank's shard: its Philox
     * streams are keyed by the global world index, mwstep/shard.py) */
    int32_t world0;
    double mass_low, mass_high;     /* additive mass sample, clipped at 0     */
    double gravity_mean, gravity_std;
    double gdir[3];                 /* world z axis in the base frame          */
} or_task;

/* Per-world physics of (world, episode): masses[n] and gravity z. */
void or_task_sample_physics(const or_model* m, const or_task* t, uint32_t world,
                            uint32_t episode, double* masses, double* gz);

/* Philox4x32-10 (Salmon et al. 2011), key = seed, counter = (world, episode, 0, 0). */
void or_philox(uint64_t seed, uint32_t world, uint32_t episode, uint32_t out[4]);
/* raw Philox4x32-10 on (ctr[4], key[2]) for the published known-answer vectors */
void or_philox_raw(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

/* Sample the initial state of world w for its given episode index. */
void or_task_reset_state(const or_task* t, uint32_t world, uint32_t episode,
                         double* q, double* qd);

/* Observation of one world (returns n_obs). */
int or_task_obs(const or_task* t, const double* q, const double* qd, double* obs);

/* One vectorised env step over W worlds, state SoA q[d*W + w].
 * actions: int32 (discrete) or double (continuous) per world.
 * Writes obs[W*n_obs] (reset obs where done), reward[W], done[W],
 * terminal_obs[W*n_obs] (only where done), and advances episode/steps. */
void or_vec_step(const or_model* m, const or_task* t, int W,
                 double* q, double* qd, const void* actions,
                 uint32_t* episode, uint32_t* steps,
                 double* obs, double* reward, uint8_t* done,
                 double* terminal_obs, int pgs_iters);

/* Initial reset of all worlds (episode index 0). */
void or_vec_reset(const or_model* m, const or_task* t, int W, double* q,
                  double* qd, uint32_t* episode, uint32_t* steps, double* obs);

/* CPU baseline: T vec steps, actions[T*W] (int32 for discrete, double else). */
void or_vec_rollout(const or_model* m, const or_task* t, int W, int T,
                    double* q, double* qd, const void* actions,
                    uint32_t* episode, uint32_t* steps, double* obs,
                    double* reward, uint8_t* done, double* terminal_obs,
                    int pgs_iters);

/* ------------------------------------------------------------------ */
/* Scene: several models in one world (World::insertModel,             */
/* cpp/scenario/gazebo/src/World.cpp:394-420), each a tree on a fixed  */
/* or floating base, colliding with the ground plane and with each     */
/* other (box / sphere shapes; DART + ODE collision detector [EXT]),   */
/* external world wrenches on links (Link::applyWorldWrench,           */
/* Link.cpp:484-560; Physics.cpp:1446-1525).  Dense formulation: block */
/* diagonal mass matrix of the models' or_float_dynamics, one boxed    */
/* LCP over every contact and joint row.                               */
/* ------------------------------------------------------------------ */
#define OR_SC_MAXM 8
#define OR_SC_MAXC 160           /* contact points per step (above the GPU large-contact capacity, 128) */
#define OR_SC_MAXNV (6 * OR_SC_MAXM + OR_MAXB)

typedef struct {
    int32_t n_models;
    int32_t ground;              /* ground plane z = 0, normal +z             */
    double mu;                   /* Coulomb friction of every contact         */
    double gravity[3];
    int32_t floating[OR_SC_MAXM];/* 0: the base link is welded at its pose    */
    int32_t pad_;
    or_float_model model[OR_SC_MAXM];  /* trees, base inertias, shapes        */
} or_scene_model;

typedef struct {
    or_float_state s[OR_SC_MAXM];      /* fixed models: p, R constant, V = 0  */
} or_scene_state;

/* One engine step of the scene.
 *   mode / cmd   [OR_SC_MAXM][OR_MAXB] joint actuation of every model
 *   wrench       [OR_SC_MAXM][1 + OR_MAXB][6] world force (at the link
 *                origin) and world torque per link, index 0 = the base link;
 *                may be NULL
 * Contacts (capacity OR_SC_MAXC): c_out rows of 10 = point xyz, normal xyz
 * (from body B into body A), force on A xyz (impulse / dt), depth; c_who
 * rows of 4 = model A, link A, model B, link B (link -1 = base; model B -1 =
 * the ground plane).  Order: ground contacts model by model, shape by shape
 * (box corners, then spheres); then shape pairs of different models in
 * (model a, shape, model b, shape) order, at most 4 points per pair.  Shapes
 * on the base link of a welded (fixed-base) model do not touch the ground,
 * nor each other.
 * Returns the number of contacts. */
int or_scene_step(const or_scene_model* m, double dt, or_scene_state* st, const int32_t* mode,
                  const double* cmd, const double* wrench, int pgs_iters, double* c_out, int32_t* c_who);

/* Narrow phase used by or_scene_step (exposed for tests): box-box (SAT over
 * the 15 axes, face clipping or edge-edge), box-sphere, sphere-sphere.  Shape
 * type 0 box (size = half extents), 1 sphere (size[0] = radius); pose (c, R
 * row-major, columns = shape axes in the world).  Writes up to 4 points and
 * depths and the unit normal from B into A; returns the point count. */
/* shape-frame point of ground-contact slot c (box corner, sphere centre,
 * cylinder rim point); RS = the shape's world rotation */
void or_slot_point(int type, const double* h, const double* RS, int c, double l[3]);
/* Convex hull of a mesh shape's support points (np <= OR_MESH_MAXP, fp64,
 * brute force; coplanar points share one face, counter-clockwise seen from
 * outside): outward unit normals n, offsets d (inside n . x <= d), the face
 * polygons and the edges.  Returns the face count, 0 for a flat point set. */
typedef struct {
    int32_t nv, nf, ne;
    double n[OR_HULL_MAXF][3];
    double d[OR_HULL_MAXF];
    int32_t fnv[OR_HULL_MAXF];
    int32_t fv[OR_HULL_MAXF][OR_MESH_MAXP];
    int32_t e[OR_HULL_MAXE][2];
    int32_t ef[OR_HULL_MAXE][2];   /* the two faces meeting at each edge */
} or_hull_info;
int or_hull_build(int np, const double* pts, or_hull_info* info);
/* The hull narrow phase of a mesh shape (type 3) against a box (0) or
 * another mesh: SAT over face normals and edge pairs, reference-face
 * clipping (same outputs as or_collide: normal from B into A, <= 4 points
 * with their depths); a mesh's npts / pts are its support points. */
int or_collide_hull(int type_a, const double* size_a, int npts_a, const double* pts_a, const double* c_a,
                    const double* R_a, int type_b, const double* size_b, int npts_b, const double* pts_b,
                    const double* c_b, const double* R_b, double normal[3], double* points, double* depths);
int or_collide(int type_a, const double* size_a, const double* c_a, const double* R_a, int type_b,
               const double* size_b, const double* c_b, const double* R_b, double normal[3], double* points,
               double* depths);

#ifdef __cplusplus
}
#endif
#endif
