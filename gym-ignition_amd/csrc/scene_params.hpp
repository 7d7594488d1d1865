// scene_params.hpp -- device parameter block of a scene: several models in
// one world (World::insertModel, cpp/scenario/gazebo/src/World.cpp:394-420),
// each a kinematic tree on a fixed or floating base, with box / sphere
// collision shapes that touch the ground plane and the shapes of the other
// models.  Shared by every world of a scene (read-only, uniform per wave).
//
// Node numbering of the scene kernel (scene_kernel.hip), one node per lane, model by
// model in insertion order (stable when models are added): model m owns nodes
// [node0, node0 + 1 + n_bodies): its base link, then its bodies (the links
// moved by its joints) depth-first (parent index < own index).  Bodies (=
// dofs) are numbered globally in the same order.
// Generalized velocity nu: model by model, [6 base coordinates if floating]
// then the model's joint coordinates.
#pragma once

#include <cstdint>

#include "chain_params.hpp"

namespace mw {

constexpr int kScMaxModels = 8;
constexpr int kScMaxBodies = 48;
constexpr int kScMaxNodes = kScMaxModels + kScMaxBodies;   // <= 64 lanes
constexpr int kScMaxNv = 6 * kScMaxModels + kScMaxBodies;   // 96 coordinates
constexpr int kScMaxShapes = 48;
constexpr int kScMaxPairs = 128;        // shape pairs of different models (2 lane passes)
constexpr int kScMaxGroundSlots = 128;  // 8 per box / cylinder, 1 per sphere, <= 16 per mesh (2 lane passes)
constexpr int kScMaxContacts = 32;      // contact points per step (3 rows each)
constexpr int kScMaxRows = 64;         // rows of the compact path (the register LCP); more: the large-contact path
constexpr int kScWrenchSlots = 4;       // concurrent wrenches (distinct expiries) per link
constexpr int kScMaxDepth = 12;         // tree depth of the response passes' stacks
constexpr uint32_t kScGroundBit = 1u << 31;  // present mask: the world has a ground plane
constexpr int kScMaxHulls = 8;          // mesh shapes with a collision hull (hull.hpp)
// Large-contact world-steps (scene_kernel.hip sc_big_constraints): a step with
// more than kScMaxContacts contact points, or more constraint rows than the
// 64-lane register LCP holds, keeps its contacts, Jacobian / response rows and
// Delassus matrix in a per-world workspace in HBM (SceneDev::big) of up to
// this capacity, and solves DART's two stages by block Gauss-Seidel over
// 64-row blocks, each block an exact box QP (wave_lcp.hpp wave_boxqp)
constexpr int kScBigContacts = 128;
constexpr int kScBigRows = 512;         // 8 blocks of 64: contact rows 3 c + d, then joint rows
constexpr int kScBigContactWords = 20;  // p[3] n[3] t1[3] t2[3] depth, node A, node B, key, x[3], pad
constexpr int kScPairMaxPoints = 4;     // contact points of one shape pair (every pair reduces to <= 4; worst-case sizing)

// A mesh shape's collision hull (hull.hpp build_hull, float32, shape frame):
// vertices, outward face planes (n, d: inside n . x <= d), face polygons
// counter-clockwise seen from outside, edges, the vertex centroid.
struct ScHull {
    int32_t nv, nf, ne, pad_;
    float ctr[4];
    float v[16][4];
    float plane[32][4];
    int8_t fnv[32];
    int8_t fv[32][16];
    int8_t e[48][2];
    int8_t ef[48][2];   // the two faces meeting at each edge
};

struct SceneModelF {
    int32_t floating;   // 1: DART FreeJoint root; 0: welded at (p0, R0)
    int32_t body0;      // first body of the model
    int32_t n_bodies;
    int32_t coff;       // first coordinate of the model in nu
    int32_t node0;      // the base link's node
    float mass;         // base link inertial
    float com[3];
    float Io[6];        // rotational inertia about the base ORIGIN: xx yy zz xy xz yz
    float p0[3];        // pose of a welded base (world)
    float R0[9];
    float pad_[5];
};
static_assert(sizeof(SceneModelF) == 32 * 4, "SceneModelF layout");

struct SceneF {
    int32_t n_models;
    int32_t n_bodies;
    int32_t nv;             // coordinates
    int32_t n_shapes;
    int32_t n_pairs;
    int32_t n_slots;        // ground slots
    int32_t n_nodes;
    int32_t levels;         // node depth levels (bases are level 0)
    int32_t fanout;         // most children of one node
    int32_t dual;           // some joint has damping
    int32_t ground;         // ground plane z = 0
    float mu;               // Coulomb friction of every contact
    float g[3];             // world gravity
    int32_t pad_;
    SceneModelF model[kScMaxModels];
    BodyF b[kScMaxBodies];  // parent: global body index, -1 = the model's base
    int8_t body_model[kScMaxBodies];
    int8_t body_node[kScMaxBodies];
    int8_t node_model[kScMaxNodes];
    int8_t node_body[kScMaxNodes];      // -1: the node is its model's base link
    int8_t node_depth[kScMaxNodes];     // bases 0, bodies 1 + depth below the base
    int8_t node_srank[kScMaxNodes];     // rank among the parent node's children (highest index first)
    int16_t body_coord[kScMaxBodies];   // coordinate of the body's joint in nu
    uint64_t body_path[kScMaxBodies];   // bit k: body k is the body or one of its ancestors
    // collision shapes, model by model (base first, then by body)
    int32_t shape_node[kScMaxShapes];   // node owning the shape
    int32_t shape_model[kScMaxShapes];
    int32_t shape_type[kScMaxShapes];   // 0 box (half extents), 1 sphere (radius), 2 cylinder, 3 mesh
                                        // (bounding box half extents; ground slots at slot_pt)
    int32_t shape_slot0[kScMaxShapes];  // first ground slot
    float shape_size[kScMaxShapes][3];
    float shape_R[kScMaxShapes][9];     // shape pose in the node frame
    float shape_p[kScMaxShapes][3];
    int16_t pair_a[kScMaxPairs];        // shape indices, model(a) < model(b)
    int16_t pair_b[kScMaxPairs];
    int16_t slot_shape[kScMaxGroundSlots];
    float slot_pt[kScMaxGroundSlots][3];  // mesh slots: support point in the shape frame
    // mesh shapes against boxes and meshes of other models: the hull narrow
    // phase (-1: a box-shaped or flat mesh, which collides as its bounding box)
    int8_t shape_hull[kScMaxShapes];
    int32_t n_hulls;
    ScHull hull[kScMaxHulls];
    ScHull box_hull;   // the unit box (half extents 1) as a hull: a box's topology for the hull narrow phase
};

// per-model JointController period gates of one launch (bit s: the PID of the
// model's Position / Velocity joints is recomputed on substep s)
struct SceneGates {
    uint64_t gate[kScMaxModels];
};

// device arrays of a scene, world index fastest
struct SceneDev {
    // joints [n_bodies][W] (same meaning as SimDev)
    float *q, *qd, *qdd, *cmd, *vtgt, *rq, *rqd, *ptgt, *pid_e, *pid_i, *pid_u;
    uint8_t *act, *rflag;
    // bases [13 * n_models][W] (p xyz, q wxyz, twist body frame [w; v]); pending
    // pose / velocity resets [7 * K][W], [6 * K][W] and their flags [K][W]
    float *base, *rpose, *rvel;
    uint8_t* bflag;
    uint32_t* present;   // [W] bit m: model m is in world w
    // wrenches [slot][6][node][W] (world force at the link origin, world
    // torque) and the last iteration of each slot [slot][node][W]
    float* wrench;
    int32_t* wlast;
    // contacts of the last step: [c][12][W] (point, normal B->A, force on A,
    // depth, node A, node B (-1 ground)) and their count [W]
    float* contact;
    int32_t* ncontact;
    int32_t* overflow;   // [0] contact points / rows dropped (capacity), [2..3] exact LCP solves out of
                         // budget (uint64), [4..5] worlds flagged diverged (uint64)
    uint8_t* diverged;   // [W] sticky: the world's stored joint / base state was not finite
    float* wphys;        // [4][W] per-world physics: gravity xyz (World::setGravity), ground friction
    // exact-LCP warm start, the previous step's impulses by row identity:
    // [0] contact count [W], [1 .. kScMaxContacts] contact keys (ground slot,
    // or n_slots + 4 pair + point) [c][W], then kScWarmRows impulses [row][W]
    // (contact c rows 3 c + d, joint rows kScWarmJoint0 + 3 body + type)
    int32_t* warm;
    // direct runs (mw_scene_run of small scenes): the host-mapped q / qd / qdd
    // planes of the pinned mirror, [3][rb_plane], written beside the device
    // state so the run needs no readback copy; nullptr otherwise
    float* rb;
    int32_t rb_plane;
    // large-contact workspace (nullptr: the scene cannot exceed the compact
    // capacity, or has no shapes): big_stride floats per world -- contacts
    // [big_cmax][kScBigContactWords], row fields [11][big_rows]
    // (scene_kernel.hip ScBigWs), J^T and MJ^T [MAXNV][big_rows], A
    // [big_rows][big_rows] (symmetric, CFM on the diagonal), its LDL^T
    float* big;
    int64_t big_stride;
    int32_t big_cmax, big_rows;
    int32_t contact_cap;  // contact points per world the contact output holds
};

// floats of one world's large-contact workspace (host sizing and device views agree)
inline constexpr int64_t sc_big_world_floats(int cmax, int rows, int maxnv) {
    return static_cast<int64_t>(kScBigContactWords) * cmax + 11LL * rows + 2LL * maxnv * rows +
           2 * static_cast<int64_t>(rows) * rows;   // row fields, J^T / MJ^T, A and its LDL^T
}

constexpr int kScWarmJoint0 = 3 * kScMaxContacts;
constexpr int kScWarmRows = kScWarmJoint0 + 3 * kScMaxBodies;
// the impulse block twice: the final impulses, then the exact solve's stage-1
// (frictionless) impulses (wave_lcp.hpp: DART's two stages)
constexpr int kScWarmWords = 1 + kScMaxContacts + 2 * kScWarmRows;

// per-launch arguments
struct SceneArgs {
    float dt, inv_dt;
    int32_t substeps;
    int32_t pgs_iters;
    int32_t first;       // first launch of a run: apply resets and commands
    int32_t paused;
    int32_t iter0;       // simulator iterations before this launch (wrench expiry)
    int32_t want_contacts;
    int32_t lcp_solves;  // > 0: exact boxed LCP (wave_lcp.hpp) within that many linear solves per step
};

}  // namespace mw
