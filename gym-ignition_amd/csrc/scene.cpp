// scene.cpp -- C ABI of scenes (include/mwscene.h): several models per world,
// many worlds per launch (scene_kernel.hip).
//
// Host counterpart of the reference's World / Model / Joint / Link component
// plumbing (cpp/scenario/gazebo/src/World.cpp, Model.cpp, Joint.cpp,
// Link.cpp) for a multi-model world: models are appended (node, body and
// coordinate numbering stay stable), device arrays are sized for the scene
// capacity up front (no reallocation when a model is inserted mid-run), and a
// model's presence in each world is a bit of a per-world mask.
#include "mwscene.h"
#include "mwstep_testhooks.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>
#include <limits>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "errors.hpp"
#include "hull.hpp"
#include "model.hpp"
#include "scene_params.hpp"

namespace mw {
hipError_t launch_scene_run(const SceneF* P, int nv, const SceneDev& D, const PidF* pid, const SceneGates& G, int W,
                            const SceneArgs& a, hipStream_t st);
}

namespace {

// a hull (hull.hpp, fp64) as the scene kernel reads it (float32)
void fill_hull(mw::ScHull& H, const mw::HostHull& h) {
    H.nv = h.nv;
    H.nf = h.nf;
    H.ne = h.ne;
    for (int k = 0; k < 3; ++k) H.ctr[k] = static_cast<float>(h.ctr[k]);
    for (int i = 0; i < h.nv; ++i)
        for (int k = 0; k < 3; ++k) H.v[i][k] = static_cast<float>(h.v[i][k]);
    for (int f = 0; f < h.nf; ++f) {
        for (int k = 0; k < 3; ++k) H.plane[f][k] = static_cast<float>(h.n[f][k]);
        H.plane[f][3] = static_cast<float>(h.d[f]);
        H.fnv[f] = static_cast<int8_t>(h.fnv[f]);
        for (int t = 0; t < h.fnv[f]; ++t) H.fv[f][t] = static_cast<int8_t>(h.fv[f][t]);
    }
    for (int e = 0; e < h.ne; ++e)
        for (int k = 0; k < 2; ++k) {
            H.e[e][k] = static_cast<int8_t>(h.e[e][k]);
            H.ef[e][k] = static_cast<int8_t>(h.ef[e][k]);
        }
}

int fail(int code, const std::string& msg) {
    mw::set_last_error(msg);
    return code;
}

#define SC_HIP(call)                                                                      \
    do {                                                                                  \
        hipError_t e_ = (call);                                                           \
        if (e_ != hipSuccess)                                                             \
            return fail(MW_EHIP, std::string(#call " failed: ") + hipGetErrorString(e_)); \
    } while (0)

constexpr int NBMAX = mw::kScMaxBodies;
constexpr int KMAX = mw::kScMaxModels;
constexpr int NNMAX = mw::kScMaxNodes;
constexpr int CMAX = mw::kScMaxContacts;
constexpr int SLOTS = mw::kScWrenchSlots;
// ignition::math::PID(1, 0.1, 0.01, -1, 0, -1, 0, 0) (Joint.cpp:63)
constexpr std::array<double, 8> kDefaultPid = {1.0, 0.1, 0.01, 0.0, -1.0, 0.0, 0.0, -1.0};

float to_f32(double v) {
    const double big = static_cast<double>(std::numeric_limits<float>::max());
    return static_cast<float>(v > big ? big : (v < -big ? -big : v));
}

struct SceneModel {
    mw::ChainModel m;
    std::string name;
    std::array<double, 7> pose{};
    int body0 = 0, node0 = 0, coff = 0;
    bool controller = false;   // a Position / Velocity / servo joint inserted the JointController
    int64_t period_ns = std::numeric_limits<int64_t>::max();
    int64_t prev_ns = 0;
    bool stepped = false;
};

}  // namespace

struct mw_scene {
    mw_config cfg{};
    int W = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    std::vector<SceneModel> models;
    int NB = 0;                    // bodies (= dofs)
    int nv = 0;
    double gravity[3] = {0.0, 0.0, -9.8};
    bool ground = false;
    double mu = 1.0;
    int64_t iterations = 0, dt_ns = 0;
    mw::SceneF hp{};
    mw::SceneF* dp = nullptr;
    mw::SceneDev dev{};
    // device blocks
    void* d_joint = nullptr;       // [q qd qdd | cmd vtgt rq rqd ptgt | act rflag | pid_e pid_i pid_u]
    void* d_base = nullptr;        // [base 13K | rpose 7K | rvel 6K][W] f32 + bflag [K][W]
    void* d_misc = nullptr;        // present [W] | ncontact [W] | overflow | wlast [S][NN][W]
    float* d_wrench = nullptr;     // [S][6][NN][W]
    float* d_contact = nullptr;    // [contact_cap][12][W]
    int contact_cap = CMAX;        // contact points per world of the contact output
    float* d_big = nullptr;        // large-contact workspace (SceneDev::big), big_bytes long
    size_t big_bytes = 0;
    float* d_wphys = nullptr;      // [4][W]: gravity xyz, ground friction per world
    int32_t* d_warm = nullptr;     // [kScWarmWords][W]: exact-LCP warm-start record (SceneDev::warm)
    mw::PidF* d_pid = nullptr;
    // pinned host mirrors with the device layouts
    uint8_t* h_joint = nullptr;
    uint8_t* h_base = nullptr;
    uint32_t* h_present = nullptr;
    int32_t* h_wlast = nullptr;
    float* h_wrench = nullptr;
    float* h_contact = nullptr;
    int32_t* h_ncontact = nullptr;
    int32_t* h_overflow = nullptr;  // pinned copy of the device drop counter
    uint64_t* h_ndiv = nullptr;     // pinned copy of the count of worlds flagged diverged
    int64_t div_seen = 0;           // flagged worlds already reported
    float* h_wphys = nullptr;       // pinned mirror of d_wphys (uploaded with the presence words)
    int64_t overflow_seen = 0;      // drops already reported
    int32_t lcp_mode = MW_LCP_EXACT;  // mw_scene_set_lcp_solver
    int32_t lcp_solves = 48;        // linear solves per world-step (scene leg: 24 -> 724 unconverged, 48 -> 0; profiles/r05t)
    mw::PidF* h_pid = nullptr;
    size_t jrows = 0;              // NBMAX * W
    // host-only component data
    std::vector<int32_t> mode;     // [dof][W]
    std::vector<double> cmd64, ptgt64;
    std::vector<std::array<double, 8>> pid;   // per dof
    // dirty / stale flags
    bool cmd_dirty = false, base_dirty = false, present_dirty = true, wrench_dirty = false, pid_dirty = true;
    bool params_dirty = true;
    bool joints_stale = false, base_stale = false, contacts_stale = false;
    bool ran = false;              // an unpaused run produced contacts
    bool idle = true;              // nothing of ours is queued on the stream
    bool clear_cmd = false, clear_base = false;  // consumed mirrors to clear after the next sync
    // direct runs: the kernel reads the command block out of the pinned mirror
    // (h_joint_dev: its device address) and writes q / qd / qdd into it; the
    // device copy of the command block is then stale until the next upload
    float* h_joint_dev = nullptr;
    bool dev_cmd_stale = false;

    size_t jidx(int d, int w) const { return static_cast<size_t>(d) * W + w; }
    float* hq() { return reinterpret_cast<float*>(h_joint); }
    float* hqd() { return hq() + jrows; }
    float* hqdd() { return hq() + 2 * jrows; }
    float* hcmd() { return hq() + 3 * jrows; }
    float* hvt() { return hq() + 4 * jrows; }
    float* hrq() { return hq() + 5 * jrows; }
    float* hrqd() { return hq() + 6 * jrows; }
    float* hptgt() { return hq() + 7 * jrows; }
    uint8_t* hact() { return h_joint + 8 * jrows * sizeof(float); }
    uint8_t* hrflag() { return hact() + jrows; }
    size_t state_bytes() const { return 3 * jrows * sizeof(float); }
    size_t cmd_off() const { return state_bytes(); }
    size_t cmd_bytes() const { return 5 * jrows * sizeof(float) + 2 * jrows; }
    size_t joint_bytes() const { return cmd_off() + cmd_bytes() + 3 * jrows * sizeof(float); }
    size_t krows() const { return static_cast<size_t>(KMAX) * W; }
    float* hbase(int m, int f, int w) { return reinterpret_cast<float*>(h_base) + (static_cast<size_t>(13 * m + f)) * W + w; }
    float* hrpose(int m, int f, int w) {
        return reinterpret_cast<float*>(h_base) + 13 * krows() + static_cast<size_t>(7 * m + f) * W + w;
    }
    float* hrvel(int m, int f, int w) {
        return reinterpret_cast<float*>(h_base) + 20 * krows() + static_cast<size_t>(6 * m + f) * W + w;
    }
    uint8_t* hbflag() { return h_base + 26 * krows() * sizeof(float); }
    size_t base_bytes() const { return 26 * krows() * sizeof(float) + krows(); }
    int model_of_dof(int d) const {
        for (size_t m = 0; m < models.size(); ++m)
            if (d >= models[m].body0 && d < models[m].body0 + models[m].m.dofs()) return static_cast<int>(m);
        return -1;
    }
};

namespace {

int check(const mw_scene* s) {
    if (!s) return fail(MW_EINVAL, "null scene handle");
    return MW_OK;
}

int check_model(const mw_scene* s, int32_t m) {
    if (int rc = check(s)) return rc;
    if (m < 0 || m >= static_cast<int32_t>(s->models.size()))
        return fail(MW_ENOTFOUND, "model index " + std::to_string(m) + " out of range");
    return MW_OK;
}

int check_worlds(const mw_scene* s, int32_t w0, int32_t nw) {
    if (w0 < 0 || nw < 0 || w0 + nw > s->W)
        return fail(MW_EINVAL, "world range [" + std::to_string(w0) + ", " + std::to_string(w0 + nw) +
                                   ") out of [0, " + std::to_string(s->W) + ")");
    return MW_OK;
}

// parameter block of the current model list; throws on capacity overflow
void build_params(mw_scene* s) {
    mw::SceneF& P = s->hp;
    std::memset(&P, 0, sizeof(P));
    {
        // the unit box's hull: every box's topology in the hull narrow phase
        // (corners in the box slot order; oracle.c hull_box builds the same)
        std::vector<std::array<double, 3>> corners;
        for (int c = 0; c < 8; ++c)
            corners.push_back({(c & 4) ? 1.0 : -1.0, (c & 2) ? 1.0 : -1.0, (c & 1) ? 1.0 : -1.0});
        mw::HostHull h;
        mw::build_hull(corners, h);
        fill_hull(P.box_hull, h);
    }
    const int K = static_cast<int>(s->models.size());
    P.n_models = K;
    P.ground = s->ground ? 1 : 0;
    P.mu = static_cast<float>(s->mu);
    for (int k = 0; k < 3; ++k) P.g[k] = static_cast<float>(s->gravity[k]);
    int body = 0, node = 0, coff = 0, shape = 0, slot = 0, dual = 0;
    std::vector<int> children(NNMAX, 0), depth(NNMAX, 0);
    auto snap = [](double v) { return std::fabs(v) < 1e-12 ? 0.0 : v; };
    for (int m = 0; m < K; ++m) {
        SceneModel& sm = s->models[m];
        const mw::ChainModel& cm = sm.m;
        const int n = cm.dofs();
        if (body + n > NBMAX) throw std::runtime_error("a scene holds at most " + std::to_string(NBMAX) + " joints");
        if (node + 1 + n > NNMAX) throw std::runtime_error("too many links in the scene");
        sm.body0 = body;
        sm.node0 = node;
        sm.coff = coff;
        mw::SceneModelF& md = P.model[m];
        md.floating = cm.floating ? 1 : 0;
        md.body0 = body;
        md.n_bodies = n;
        md.coff = coff;
        md.node0 = node;
        const double ms = cm.base_mass, *c = cm.base_com.data(), *ic = cm.base_Ic.data();
        const double c2 = c[0] * c[0] + c[1] * c[1] + c[2] * c[2];
        md.mass = static_cast<float>(ms);
        for (int k = 0; k < 3; ++k) md.com[k] = static_cast<float>(c[k]);
        const double Io[6] = {ic[0] + ms * (c2 - c[0] * c[0]), ic[1] + ms * (c2 - c[1] * c[1]),
                              ic[2] + ms * (c2 - c[2] * c[2]), ic[3] - ms * c[0] * c[1], ic[4] - ms * c[0] * c[2],
                              ic[5] - ms * c[1] * c[2]};
        for (int k = 0; k < 6; ++k) md.Io[k] = static_cast<float>(Io[k]);
        for (int k = 0; k < 3; ++k) md.p0[k] = static_cast<float>(cm.base_p[k]);
        for (int k = 0; k < 9; ++k) md.R0[k] = static_cast<float>(snap(cm.base_R[k]));
        P.node_model[node] = static_cast<int8_t>(m);
        P.node_body[node] = -1;
        P.node_depth[node] = 0;
        coff += cm.floating ? 6 : 0;
        for (int i = 0; i < n; ++i) {
            const mw::ChainBody& b = cm.bodies[i];
            const int g = body + i;
            mw::BodyF& f = P.b[g];
            for (int k = 0; k < 9; ++k) f.E[k] = static_cast<float>(snap(b.E[k]));
            for (int k = 0; k < 3; ++k) {
                f.r[k] = static_cast<float>(b.r[k]);
                f.axis[k] = static_cast<float>(b.axis[k]);
                f.com[k] = static_cast<float>(b.com[k]);
                f.Ea[k] = static_cast<float>(snap(b.E[k * 3] * b.axis[0] + b.E[k * 3 + 1] * b.axis[1] +
                                                  b.E[k * 3 + 2] * b.axis[2]));
            }
            f.jtype = ((b.type == mw::JType::Prismatic) ? 1 : 0) | (b.ball << 4);  // chain_dyn.hpp ball_part
            f.mass = static_cast<float>(b.mass);
            const double bc2 = b.com[0] * b.com[0] + b.com[1] * b.com[1] + b.com[2] * b.com[2];
            f.Io[0] = static_cast<float>(b.Ic[0] + b.mass * (bc2 - b.com[0] * b.com[0]));
            f.Io[1] = static_cast<float>(b.Ic[1] + b.mass * (bc2 - b.com[1] * b.com[1]));
            f.Io[2] = static_cast<float>(b.Ic[2] + b.mass * (bc2 - b.com[2] * b.com[2]));
            f.Io[3] = static_cast<float>(b.Ic[3] - b.mass * b.com[0] * b.com[1]);
            f.Io[4] = static_cast<float>(b.Ic[4] - b.mass * b.com[0] * b.com[2]);
            f.Io[5] = static_cast<float>(b.Ic[5] - b.mass * b.com[1] * b.com[2]);
            f.damping = static_cast<float>(b.damping);
            f.friction = static_cast<float>(b.friction);
            f.lower = to_f32(b.lower);
            f.upper = to_f32(b.upper);
            f.effort = to_f32(b.effort);
            f.vel_limit = to_f32(b.vel_limit);
            f.limited = b.limited ? 1 : 0;
            f.parent = b.parent >= 0 ? body + b.parent : -1;
            if (b.damping != 0.0) dual = 1;
            const int nd = node + 1 + i;
            P.body_model[g] = static_cast<int8_t>(m);
            P.body_node[g] = static_cast<int8_t>(nd);
            P.node_model[nd] = static_cast<int8_t>(m);
            P.node_body[nd] = static_cast<int8_t>(g);
            const int pnode = b.parent >= 0 ? node + 1 + b.parent : node;
            depth[nd] = depth[pnode] + 1;
            P.node_depth[nd] = static_cast<int8_t>(depth[nd]);
            if (depth[nd] > mw::kScMaxDepth) throw std::runtime_error("a model's tree is deeper than 12 joints");
            P.body_coord[g] = static_cast<int16_t>(coff + i);
            P.body_path[g] = (uint64_t{1} << g) | (b.parent >= 0 ? P.body_path[body + b.parent] : uint64_t{0});
        }
        // sibling ranks, highest index first (the serial inward pass order)
        for (int i = n - 1; i >= 0; --i) {
            const int nd = node + 1 + i;
            const int pnode = cm.bodies[i].parent >= 0 ? node + 1 + cm.bodies[i].parent : node;
            P.node_srank[nd] = static_cast<int8_t>(children[pnode]++);
        }
        // shapes: base first, then by body
        auto add_shape = [&](const mw::Shape& sh, int nd) {
            if (shape >= mw::kScMaxShapes) throw std::runtime_error("a scene holds at most 48 collision shapes");
            P.shape_node[shape] = nd;
            P.shape_model[shape] = m;
            P.shape_type[shape] = sh.type;
            for (int k = 0; k < 3; ++k) {
                P.shape_size[shape][k] = static_cast<float>(sh.size[k]);
                P.shape_p[shape][k] = static_cast<float>(sh.p[k]);
            }
            for (int k = 0; k < 9; ++k) P.shape_R[shape][k] = static_cast<float>(snap(sh.R[k]));
            // a welded base link never touches the ground (it does not move)
            const bool movable = !(nd == node && !cm.floating);
            P.shape_slot0[shape] = slot;
            P.shape_hull[shape] = -1;
            if (sh.type == mw::Shape::Mesh && !mw::mesh_is_box(sh.points, sh.size)) {
                mw::HostHull h;
                if (mw::build_hull(sh.points, h)) {
                    if (P.n_hulls >= mw::kScMaxHulls) throw std::runtime_error("a scene holds at most 8 mesh hulls");
                    mw::ScHull& H = P.hull[P.n_hulls];
                    fill_hull(H, h);
                    P.shape_hull[shape] = static_cast<int8_t>(P.n_hulls++);
                }
            }
            if (movable) {
                const int ns = (sh.type == mw::Shape::Sphere) ? 1
                               : (sh.type == mw::Shape::Mesh) ? static_cast<int>(sh.points.size())
                                                              : 8;
                if (slot + ns > mw::kScMaxGroundSlots) throw std::runtime_error("too many ground contact slots");
                for (int k = 0; k < ns; ++k) {
                    P.slot_shape[slot + k] = static_cast<int16_t>(shape);
                    if (sh.type == mw::Shape::Mesh)
                        for (int e = 0; e < 3; ++e) P.slot_pt[slot + k][e] = static_cast<float>(sh.points[k][e]);
                }
                slot += ns;
            }
            ++shape;
        };
        for (const auto& sh : cm.base_shapes) add_shape(sh, node);
        for (int i = 0; i < n; ++i)
            for (const auto& sh : cm.bodies[i].shapes) add_shape(sh, node + 1 + i);
        body += n;
        node += 1 + n;
        coff += n;
    }
    if (coff > 64) throw std::runtime_error("a scene holds at most 64 generalized coordinates in this build");
    P.n_bodies = body;
    P.n_nodes = node;
    P.nv = coff;
    P.n_shapes = shape;
    P.n_slots = slot;
    P.dual = dual;
    int levels = 1, fanout = 0;
    for (int k = 0; k < node; ++k) {
        levels = std::max(levels, depth[k] + 1);
        fanout = std::max(fanout, children[k]);
    }
    P.levels = levels;
    P.fanout = fanout;
    // shape pairs of different models (not both on welded base links)
    int np = 0;
    for (int a = 0; a < shape; ++a)
        for (int b = a + 1; b < shape; ++b) {
            if (P.shape_model[a] == P.shape_model[b]) continue;
            const auto welded = [&](int sh) {
                const mw::SceneModelF& md = P.model[P.shape_model[sh]];
                return !md.floating && P.shape_node[sh] == md.node0;
            };
            if (welded(a) && welded(b)) continue;
            if (np >= mw::kScMaxPairs) throw std::runtime_error("too many collision shape pairs in the scene");
            P.pair_a[np] = static_cast<int16_t>(a);
            P.pair_b[np] = static_cast<int16_t>(b);
            ++np;
        }
    P.n_pairs = np;
    s->NB = body;
    s->nv = coff;
}

int sync(mw_scene* s) {
    SC_HIP(hipStreamSynchronize(s->stream));
    s->idle = true;
    return MW_OK;
}

// the kernel consumes force commands and resets (UpdateSim zero-fill,
// Physics.cpp:2226-2254): mirror that on the host copy once the uploads
// out of it have completed
void clear_consumed(mw_scene* s) {
    if (s->clear_cmd) {
        std::memset(s->hcmd(), 0, s->jrows * sizeof(float));
        std::memset(s->hrflag(), 0, s->jrows);
        std::fill(s->cmd64.begin(), s->cmd64.end(), 0.0);
    }
    if (s->clear_base) std::memset(s->hbflag(), 0, s->krows());
    s->clear_cmd = s->clear_base = false;
}

int ensure_big(mw_scene* s);

// Upload pending parameters, commands, resets, presence, wrenches and gains
// (asynchronous copies out of the pinned mirrors).  defer: the caller
// synchronises later and then calls clear_consumed(); otherwise this waits
// for the copies and clears the consumed mirrors itself.
int flush(mw_scene* s, bool defer, bool direct = false) {
    const bool any = s->params_dirty || s->cmd_dirty || s->base_dirty || s->present_dirty || s->wrench_dirty ||
                     s->pid_dirty || (s->dev_cmd_stale && !direct);
    if (!any) return MW_OK;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    SC_HIP(hipStreamIsCapturing(s->stream, &cap));
    if (cap != hipStreamCaptureStatusNone)
        return fail(MW_ESTATE, "pending commands, resets or model changes cannot be captured into a graph: "
                               "apply them with a run before capturing");
    // the mirrors were rewritten by the setters: an earlier copy out of them
    // must not still be queued
    if (!s->idle)
        if (int rc = sync(s)) return rc;
    if (s->params_dirty) {
        if (int rc = ensure_big(s)) return rc;
        SC_HIP(hipMemcpyAsync(s->dp, &s->hp, sizeof(mw::SceneF), hipMemcpyHostToDevice, s->stream));
        // new slots / pairs: the warm-start keys of the old layout mean nothing
        SC_HIP(hipMemsetAsync(s->d_warm, 0, s->W * sizeof(int32_t), s->stream));
        s->params_dirty = false;
    }
    if (direct) {
        // the launch reads the command block straight out of the mirror
        if (s->cmd_dirty) {
            s->clear_cmd = true;
            s->dev_cmd_stale = true;
        }
    } else if (s->cmd_dirty || s->dev_cmd_stale) {
        SC_HIP(hipMemcpyAsync(static_cast<uint8_t*>(s->d_joint) + s->cmd_off(), s->h_joint + s->cmd_off(),
                              s->cmd_bytes(), hipMemcpyHostToDevice, s->stream));
        s->clear_cmd = s->clear_cmd || s->cmd_dirty;
        s->dev_cmd_stale = false;
    }
    if (s->base_dirty) {
        const size_t off = 13 * s->krows() * sizeof(float);
        SC_HIP(hipMemcpyAsync(static_cast<uint8_t*>(s->d_base) + off, s->h_base + off, s->base_bytes() - off,
                              hipMemcpyHostToDevice, s->stream));
        s->clear_base = true;
    }
    if (s->present_dirty) {
        SC_HIP(hipMemcpyAsync(s->dev.present, s->h_present, s->W * sizeof(uint32_t), hipMemcpyHostToDevice,
                              s->stream));
        SC_HIP(hipMemcpyAsync(s->d_wphys, s->h_wphys, 4 * s->W * sizeof(float), hipMemcpyHostToDevice, s->stream));
    }
    if (s->wrench_dirty) {
        const size_t nn = static_cast<size_t>(SLOTS) * NNMAX * s->W;
        SC_HIP(hipMemcpyAsync(s->d_wrench, s->h_wrench, 6 * nn * sizeof(float), hipMemcpyHostToDevice, s->stream));
        SC_HIP(hipMemcpyAsync(s->dev.wlast, s->h_wlast, nn * sizeof(int32_t), hipMemcpyHostToDevice, s->stream));
    }
    if (s->pid_dirty) {
        for (int d = 0; d < s->NB; ++d) {
            const auto& g = s->pid[d];
            s->h_pid[d] = {to_f32(g[0]), to_f32(g[1]), to_f32(g[2]), to_f32(g[7]), to_f32(g[6]),
                           to_f32(g[4]), to_f32(g[3]), to_f32(g[5])};
        }
        SC_HIP(hipMemcpyAsync(s->d_pid, s->h_pid, NBMAX * sizeof(mw::PidF), hipMemcpyHostToDevice, s->stream));
    }
    s->idle = false;
    s->cmd_dirty = s->base_dirty = s->present_dirty = s->wrench_dirty = s->pid_dirty = false;
    if (!defer) {
        if (int rc = sync(s)) return rc;
        clear_consumed(s);
    }
    return MW_OK;
}

// queue the D2H copies of the joint state planes (q, qd, qdd: the rows of
// the scene's bodies) and of the base states
// what a synchronous run must read back: the base block only when some
// model has a floating base (a welded base never moves from its insertion
// pose, which the host mirror holds), the drop counter only when the scene can
// exceed a capacity (collision shapes, or more joint rows than the LCP holds)
bool needs_base_readback(const mw_scene* s) {
    for (const auto& sm : s->models)
        if (sm.m.floating) return true;
    return false;
}
bool can_overflow(const mw_scene* s) { return s->hp.n_shapes > 0 || 3 * s->NB > mw::kScMaxRows; }

// The large-contact workspace a scene needs (SceneDev::big; scene_kernel.hip
// sc_big_constraints), from its worst case: every ground slot touching,
// kScPairMaxPoints per shape pair, three joint rows per body.  None when that
// fits the compact path (<= kScMaxContacts points, <= 64 rows).
void size_big(const mw_scene* s, int& cmax, int& rows) {
    const mw::SceneF& P = s->hp;
    const int worst = (P.ground ? P.n_slots : 0) + mw::kScPairMaxPoints * P.n_pairs;
    const int jrows = 3 * s->NB;
    cmax = rows = 0;
    if (worst <= mw::kScMaxContacts && 3 * worst + jrows <= 64) return;
    cmax = std::min(worst, mw::kScBigContacts);
    rows = std::min(mw::kScBigRows, (3 * cmax + jrows + 63) / 64 * 64);
}

// (re)allocate the large-contact workspace and the contact output for the
// current parameters (the stream is idle: flush synchronised)
int ensure_big(mw_scene* s) {
    int cmax = 0, rows = 0;
    size_big(s, cmax, rows);
    const int maxnv = s->nv <= 32 ? 32 : 64;   // the kernel instance (launch_scene_run)
    const int64_t stride = rows ? mw::sc_big_world_floats(cmax, rows, maxnv) : 0;
    const size_t bytes = static_cast<size_t>(stride) * s->W * sizeof(float);
    if (bytes != s->big_bytes) {
        (void)hipFree(s->d_big);
        s->d_big = nullptr;
        s->big_bytes = 0;
        if (bytes) SC_HIP(hipMalloc(reinterpret_cast<void**>(&s->d_big), bytes));
        s->big_bytes = bytes;
    }
    mw::SceneDev& D = s->dev;
    D.big = rows ? s->d_big : nullptr;
    D.big_stride = stride;
    D.big_cmax = cmax;
    D.big_rows = rows;
    const int cap = std::max(CMAX, cmax);
    if (cap != s->contact_cap) {
        const size_t n = static_cast<size_t>(cap) * 12 * s->W * sizeof(float);
        (void)hipFree(s->d_contact);
        (void)hipHostFree(s->h_contact);
        s->d_contact = nullptr;
        s->h_contact = nullptr;
        SC_HIP(hipMalloc(reinterpret_cast<void**>(&s->d_contact), n));
        SC_HIP(hipHostMalloc(reinterpret_cast<void**>(&s->h_contact), n, hipHostMallocDefault));
        s->contact_cap = cap;
        D.contact = s->d_contact;
        SC_HIP(hipMemsetAsync(D.ncontact, 0, s->W * sizeof(int32_t), s->stream));
    }
    D.contact_cap = cap;
    return MW_OK;
}

int queue_readback(mw_scene* s, bool base = true) {
    const size_t plane = s->jrows * sizeof(float), rows = static_cast<size_t>(s->NB) * s->W * sizeof(float);
    if (rows && 3 * plane <= (size_t{1} << 20)) {
        // small scenes: one copy of the three planes beats three copies
        SC_HIP(hipMemcpyAsync(s->h_joint, s->d_joint, 3 * plane, hipMemcpyDeviceToHost, s->stream));
    } else if (rows) {
        for (int f = 0; f < 3; ++f)
            SC_HIP(hipMemcpyAsync(s->h_joint + f * plane, static_cast<uint8_t*>(s->d_joint) + f * plane, rows,
                                  hipMemcpyDeviceToHost, s->stream));
    }
    const size_t brows = static_cast<size_t>(13 * s->models.size()) * s->W * sizeof(float);
    if (brows && base) SC_HIP(hipMemcpyAsync(s->h_base, s->d_base, brows, hipMemcpyDeviceToHost, s->stream));
    s->idle = false;
    return MW_OK;
}

int pull_joints(mw_scene* s) {
    if (!s->joints_stale) return MW_OK;
    if (int rc = queue_readback(s)) return rc;
    if (int rc = sync(s)) return rc;
    s->joints_stale = s->base_stale = false;
    return MW_OK;
}

int pull_base(mw_scene* s) { return pull_joints(s); }

int pull_contacts(mw_scene* s) {
    if (!s->contacts_stale) return MW_OK;
    SC_HIP(hipMemcpyAsync(s->h_ncontact, s->dev.ncontact, s->W * sizeof(int32_t), hipMemcpyDeviceToHost, s->stream));
    SC_HIP(hipMemcpyAsync(s->h_contact, s->d_contact, static_cast<size_t>(s->contact_cap) * 12 * s->W * sizeof(float),
                          hipMemcpyDeviceToHost, s->stream));
    if (int rc = sync(s)) return rc;
    s->contacts_stale = false;
    return MW_OK;
}

int selection(const mw_scene* s, int32_t w0, int32_t nw, const int32_t* dofs, int32_t ndofs, std::vector<int32_t>& out) {
    if (int rc = check_worlds(s, w0, nw)) return rc;
    out.clear();
    if (!dofs) {
        for (int d = 0; d < s->NB; ++d) out.push_back(d);
        return MW_OK;
    }
    for (int k = 0; k < ndofs; ++k) {
        if (dofs[k] < 0 || dofs[k] >= s->NB) return fail(MW_EINVAL, "dof index " + std::to_string(dofs[k]) + " out of range");
        out.push_back(dofs[k]);
    }
    return MW_OK;
}

int copy_str(const std::string& v, char* buf, int32_t len) {
    if (!buf || len <= 0) return fail(MW_EINVAL, "invalid output buffer");
    if (static_cast<int32_t>(v.size()) + 1 > len) return fail(MW_EINVAL, "output buffer too small");
    std::memcpy(buf, v.c_str(), v.size() + 1);
    return MW_OK;
}

// quaternion wxyz of a row-major rotation
void quat_of(const std::array<double, 9>& R, double q[4]) {
    const double tr = R[0] + R[4] + R[8];
    if (tr > 0) {
        const double k = 0.5 / std::sqrt(tr + 1.0);
        q[0] = 0.25 / k; q[1] = (R[7] - R[5]) * k; q[2] = (R[2] - R[6]) * k; q[3] = (R[3] - R[1]) * k;
    } else if (R[0] > R[4] && R[0] > R[8]) {
        const double k = 2.0 * std::sqrt(1.0 + R[0] - R[4] - R[8]);
        q[0] = (R[7] - R[5]) / k; q[1] = 0.25 * k; q[2] = (R[1] + R[3]) / k; q[3] = (R[2] + R[6]) / k;
    } else if (R[4] > R[8]) {
        const double k = 2.0 * std::sqrt(1.0 + R[4] - R[0] - R[8]);
        q[0] = (R[2] - R[6]) / k; q[1] = (R[1] + R[3]) / k; q[2] = 0.25 * k; q[3] = (R[5] + R[7]) / k;
    } else {
        const double k = 2.0 * std::sqrt(1.0 + R[8] - R[0] - R[4]);
        q[0] = (R[3] - R[1]) / k; q[1] = (R[2] + R[6]) / k; q[2] = (R[5] + R[7]) / k; q[3] = 0.25 * k;
    }
}

// model m enters worlds [w0, w0 + nw) at its insertion pose, joints at rest
// A reset, insertion or removal of a world's models re-arms its divergence
// flag (mwscene.h): a world that diverged, was reset and diverges again is
// reported again.
int rearm_diverged(mw_scene* s, int32_t w0, int32_t nw) {
    if (s->dev.diverged && nw > 0) SC_HIP(hipMemsetAsync(s->dev.diverged + w0, 0, nw, s->stream));
    return MW_OK;
}

int place_model(mw_scene* s, int m, int32_t w0, int32_t nw) {
    if (int rc = pull_joints(s)) return rc;
    const SceneModel& sm = s->models[m];
    double q[4];
    quat_of(sm.m.base_R, q);
    const double init[13] = {sm.m.base_p[0], sm.m.base_p[1], sm.m.base_p[2], q[0], q[1], q[2], q[3], 0, 0, 0, 0, 0, 0};
    for (int w = w0; w < w0 + nw; ++w) {
        s->h_present[w] |= 1u << m;
        // the pose enters through a pending base reset (the kernel applies it
        // on the next run), the joints through joint resets
        for (int f = 0; f < 7; ++f) *s->hrpose(m, f, w) = static_cast<float>(init[f]);
        for (int f = 0; f < 6; ++f) *s->hrvel(m, f, w) = 0.f;
        s->hbflag()[static_cast<size_t>(m) * s->W + w] = 3u;
        for (int f = 0; f < 13; ++f) *s->hbase(m, f, w) = static_cast<float>(init[f]);
        for (int i = 0; i < sm.m.dofs(); ++i) {
            const size_t k = s->jidx(sm.body0 + i, w);
            s->hrq()[k] = 0.f;
            s->hrqd()[k] = 0.f;
            s->hrflag()[k] = 1u | 2u | 4u;
            s->hq()[k] = s->hqd()[k] = s->hqdd()[k] = 0.f;
            s->hcmd()[k] = s->hvt()[k] = s->hptgt()[k] = 0.f;
            s->hact()[k] = mw::kActForce;
            s->mode[k] = MW_MODE_IDLE;
            s->cmd64[k] = 0.0;
            s->ptgt64[k] = 0.0;
        }
        // wrenches of the model's links are dropped
        for (int sl = 0; sl < SLOTS; ++sl)
            for (int nd = sm.node0; nd < sm.node0 + 1 + sm.m.dofs(); ++nd)
                s->h_wlast[(static_cast<size_t>(sl) * NNMAX + nd) * s->W + w] = -1;
    }
    s->present_dirty = s->base_dirty = s->cmd_dirty = s->wrench_dirty = true;
    return rearm_diverged(s, w0, nw);
}

}  // namespace

extern "C" {

int mw_scene_create(const mw_config* cfg, mw_scene** out) {
    if (!cfg || !out) return fail(MW_EINVAL, "null argument");
    *out = nullptr;
    if (!(cfg->step_size > 0.0)) return fail(MW_EINVAL, "the step size must be positive");
    if (!(cfg->rtf > 0.0)) return fail(MW_EINVAL, "the real-time factor must be positive");
    if (cfg->steps_per_run <= 0) return fail(MW_EINVAL, "steps_per_run must be positive");
    if (cfg->n_worlds <= 0) return fail(MW_EINVAL, "n_worlds must be positive");
    auto s = std::make_unique<mw_scene>();
    s->cfg = *cfg;
    if (s->cfg.pgs_iters <= 0) s->cfg.pgs_iters = 50;
    s->W = cfg->n_worlds;
    s->dt_ns = static_cast<int64_t>(std::llround(cfg->step_size * 1e9));
    SC_HIP(hipSetDevice(cfg->device));
    SC_HIP(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
    s->own_stream = true;
    const size_t W = static_cast<size_t>(s->W);
    s->jrows = static_cast<size_t>(NBMAX) * W;
    SC_HIP(hipMalloc(&s->d_joint, s->joint_bytes()));
    SC_HIP(hipMemsetAsync(s->d_joint, 0, s->joint_bytes(), s->stream));
    // coherent: direct runs read the command block out of it and write the
    // joint planes into it (scene_run)
    SC_HIP(hipHostMalloc(reinterpret_cast<void**>(&s->h_joint), s->cmd_off() + s->cmd_bytes(),
                         hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(s->h_joint, 0, s->cmd_off() + s->cmd_bytes());
    {
        void* dptr = nullptr;
        if (hipHostGetDevicePointer(&dptr, s->h_joint, 0) == hipSuccess) s->h_joint_dev = static_cast<float*>(dptr);
        else (void)hipGetLastError();
    }
    SC_HIP(hipMalloc(&s->d_base, s->base_bytes()));
    SC_HIP(hipMemsetAsync(s->d_base, 0, s->base_bytes(), s->stream));
    SC_HIP(hipHostMalloc(reinterpret_cast<void**>(&s->h_base), s->base_bytes(), hipHostMallocDefault));
    std::memset(s->h_base, 0, s->base_bytes());
    const size_t nwl = static_cast<size_t>(SLOTS) * NNMAX * W;
    const size_t misc = W * sizeof(uint32_t) + W * sizeof(int32_t) + 64 + nwl * sizeof(int32_t) + W;
    SC_HIP(hipMalloc(&s->d_misc, misc));
    SC_HIP(hipMemsetAsync(s->d_misc, 0, misc, s->stream));
    SC_HIP(hipMalloc(reinterpret_cast<void**>(&s->d_wrench), 6 * nwl * sizeof(float)));
    SC_HIP(hipMemsetAsync(s->d_wrench, 0, 6 * nwl * sizeof(float), s->stream));
    SC_HIP(hipMalloc(reinterpret_cast<void**>(&s->d_contact), static_cast<size_t>(CMAX) * 12 * W * sizeof(float)));
    SC_HIP(hipMalloc(reinterpret_cast<void**>(&s->d_pid), NBMAX * sizeof(mw::PidF)));
    SC_HIP(hipMalloc(reinterpret_cast<void**>(&s->dp), sizeof(mw::SceneF)));
    SC_HIP(hipMalloc(reinterpret_cast<void**>(&s->d_wphys), 4 * W * sizeof(float)));
    SC_HIP(hipMalloc(reinterpret_cast<void**>(&s->d_warm), mw::kScWarmWords * W * sizeof(int32_t)));
    SC_HIP(hipMemsetAsync(s->d_warm, 0, mw::kScWarmWords * W * sizeof(int32_t), s->stream));
    SC_HIP(hipHostMalloc(reinterpret_cast<void**>(&s->h_wphys), 4 * W * sizeof(float), hipHostMallocDefault));
    for (size_t w = 0; w < W; ++w) {
        for (int k = 0; k < 3; ++k) s->h_wphys[k * W + w] = static_cast<float>(s->gravity[k]);
        s->h_wphys[3 * W + w] = static_cast<float>(s->mu);
    }
    SC_HIP(hipHostMalloc(reinterpret_cast<void**>(&s->h_present), W * sizeof(uint32_t), hipHostMallocDefault));
    std::memset(s->h_present, 0, W * sizeof(uint32_t));
    SC_HIP(hipHostMalloc(reinterpret_cast<void**>(&s->h_wlast), nwl * sizeof(int32_t), hipHostMallocDefault));
    std::fill(s->h_wlast, s->h_wlast + nwl, -1);
    SC_HIP(hipHostMalloc(reinterpret_cast<void**>(&s->h_wrench), 6 * nwl * sizeof(float), hipHostMallocDefault));
    std::memset(s->h_wrench, 0, 6 * nwl * sizeof(float));
    SC_HIP(hipHostMalloc(reinterpret_cast<void**>(&s->h_contact), static_cast<size_t>(CMAX) * 12 * W * sizeof(float),
                         hipHostMallocDefault));
    SC_HIP(hipHostMalloc(reinterpret_cast<void**>(&s->h_ncontact), W * sizeof(int32_t), hipHostMallocDefault));
    std::memset(s->h_ncontact, 0, W * sizeof(int32_t));
    if (!s->h_overflow) {
        SC_HIP(hipHostMalloc(reinterpret_cast<void**>(&s->h_overflow), sizeof(int32_t), hipHostMallocDefault));
        *s->h_overflow = 0;
    }
    if (!s->h_ndiv) {
        SC_HIP(hipHostMalloc(reinterpret_cast<void**>(&s->h_ndiv), sizeof(uint64_t), hipHostMallocDefault));
        *s->h_ndiv = 0;
    }
    SC_HIP(hipHostMalloc(reinterpret_cast<void**>(&s->h_pid), NBMAX * sizeof(mw::PidF), hipHostMallocDefault));
    // device views
    float* j = static_cast<float*>(s->d_joint);
    const size_t r = s->jrows;
    mw::SceneDev& D = s->dev;
    D.q = j; D.qd = j + r; D.qdd = j + 2 * r;
    D.cmd = j + 3 * r; D.vtgt = j + 4 * r; D.rq = j + 5 * r; D.rqd = j + 6 * r; D.ptgt = j + 7 * r;
    D.act = reinterpret_cast<uint8_t*>(j + 8 * r);
    D.rflag = D.act + r;
    float* tail = reinterpret_cast<float*>(D.rflag + r);
    D.pid_e = tail; D.pid_i = tail + r; D.pid_u = tail + 2 * r;
    float* b = static_cast<float*>(s->d_base);
    const size_t kr = s->krows();
    D.base = b; D.rpose = b + 13 * kr; D.rvel = b + 20 * kr;
    D.bflag = reinterpret_cast<uint8_t*>(b + 26 * kr);
    uint8_t* mp = static_cast<uint8_t*>(s->d_misc);
    D.present = reinterpret_cast<uint32_t*>(mp);
    D.ncontact = reinterpret_cast<int32_t*>(mp + W * sizeof(uint32_t));
    D.overflow = reinterpret_cast<int32_t*>(mp + W * sizeof(uint32_t) + W * sizeof(int32_t));
    D.wlast = reinterpret_cast<int32_t*>(mp + W * sizeof(uint32_t) + W * sizeof(int32_t) + 64);
    D.diverged = mp + W * sizeof(uint32_t) + W * sizeof(int32_t) + 64 + nwl * sizeof(int32_t);
    D.wrench = s->d_wrench;
    D.contact = s->d_contact;
    D.contact_cap = CMAX;
    D.big = nullptr;
    D.big_stride = 0;
    D.big_cmax = D.big_rows = 0;
    D.wphys = s->d_wphys;
    D.warm = s->d_warm;
    s->mode.assign(s->jrows, MW_MODE_IDLE);
    s->cmd64.assign(s->jrows, 0.0);
    s->ptgt64.assign(s->jrows, 0.0);
    s->wrench_dirty = true;
    SC_HIP(hipStreamSynchronize(s->stream));
    *out = s.release();
    return MW_OK;
}

void mw_scene_destroy(mw_scene* s) {
    if (!s) return;
    (void)hipSetDevice(s->cfg.device);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    (void)hipFree(s->d_joint);
    (void)hipFree(s->d_base);
    (void)hipFree(s->d_misc);
    (void)hipFree(s->d_wrench);
    (void)hipFree(s->d_contact);
    (void)hipFree(s->d_big);
    (void)hipFree(s->d_pid);
    (void)hipFree(s->dp);
    (void)hipFree(s->d_wphys);
    (void)hipFree(s->d_warm);
    (void)hipHostFree(s->h_wphys);
    (void)hipHostFree(s->h_joint);
    (void)hipHostFree(s->h_base);
    (void)hipHostFree(s->h_present);
    (void)hipHostFree(s->h_wlast);
    (void)hipHostFree(s->h_wrench);
    (void)hipHostFree(s->h_contact);
    (void)hipHostFree(s->h_ncontact);
    (void)hipHostFree(s->h_overflow);
    (void)hipHostFree(s->h_ndiv);
    (void)hipHostFree(s->h_pid);
    if (s->own_stream && s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
}

int mw_scene_set_stream(mw_scene* s, void* stream) {
    if (int rc = check(s)) return rc;
    SC_HIP(hipStreamSynchronize(s->stream));
    if (s->own_stream) (void)hipStreamDestroy(s->stream);
    s->stream = static_cast<hipStream_t>(stream);
    s->own_stream = false;
    return MW_OK;
}

int mw_scene_insert_model(mw_scene* s, const char* urdf, const double pose[7], const char* name, int32_t w0,
                          int32_t nw, int32_t* model) {
    if (int rc = check(s)) return rc;
    if (!urdf || !model) return fail(MW_EINVAL, "null argument");
    if (int rc = check_worlds(s, w0, nw)) return rc;
    if (static_cast<int>(s->models.size()) >= KMAX)
        return fail(MW_ESTATE, "a scene holds at most " + std::to_string(KMAX) + " models");
    const double ident[7] = {0, 0, 0, 1, 0, 0, 0};
    SceneModel sm;
    try {
        sm.m = mw::compile_urdf(urdf, pose ? pose : ident);
    } catch (const std::exception& e) {
        return fail(MW_EPARSE, e.what());
    }
    sm.name = (name && *name) ? name : sm.m.name;
    for (int k = 0; k < 7; ++k) sm.pose[k] = (pose ? pose : ident)[k];
    for (const auto& o : s->models)
        if (o.name == sm.name) return fail(MW_EINVAL, "a model named '" + sm.name + "' is already in the scene");
    s->models.push_back(sm);
    try {
        build_params(s);
    } catch (const std::exception& e) {
        s->models.pop_back();
        build_params(s);
        return fail(MW_EPARSE, e.what());
    }
    const int m = static_cast<int>(s->models.size()) - 1;
    const SceneModel& in = s->models[m];
    s->pid.resize(s->NB, kDefaultPid);
    for (int i = 0; i < in.m.dofs(); ++i) s->pid[in.body0 + i] = kDefaultPid;
    s->params_dirty = s->pid_dirty = true;
    if (int rc = place_model(s, m, w0, nw)) return rc;
    *model = m;
    return MW_OK;
}

int mw_scene_set_present(mw_scene* s, int32_t model, int32_t w0, int32_t nw, int32_t present) {
    if (int rc = check_model(s, model)) return rc;
    if (int rc = check_worlds(s, w0, nw)) return rc;
    if (present == 1) return place_model(s, model, w0, nw);
    for (int w = w0; w < w0 + nw; ++w) {
        if (present == 2) s->h_present[w] |= 1u << model;   // resume: the state is kept
        else s->h_present[w] &= ~(1u << model);
    }
    s->present_dirty = true;
    return present == 2 ? MW_OK : rearm_diverged(s, w0, nw);
}

int mw_scene_set_world_ground(mw_scene* s, int32_t w0, int32_t nw, int32_t enabled) {
    if (int rc = check(s)) return rc;
    if (int rc = check_worlds(s, w0, nw)) return rc;
    for (int w = w0; w < w0 + nw; ++w) {
        if (enabled) s->h_present[w] |= mw::kScGroundBit;
        else s->h_present[w] &= ~mw::kScGroundBit;
    }
    s->present_dirty = true;
    return MW_OK;
}

int mw_scene_replace_model(mw_scene* s, int32_t model, const char* urdf, const double pose[7], const char* name) {
    if (int rc = check_model(s, model)) return rc;
    if (!urdf) return fail(MW_EINVAL, "null argument");
    for (int w = 0; w < s->W; ++w)
        if ((s->h_present[w] >> model) & 1u)
            return fail(MW_ESTATE, "a model can be replaced only while it is in no world");
    const double ident[7] = {0, 0, 0, 1, 0, 0, 0};
    mw::ChainModel cm;
    try {
        cm = mw::compile_urdf(urdf, pose ? pose : ident);
    } catch (const std::exception& e) {
        return fail(MW_EPARSE, e.what());
    }
    SceneModel& old = s->models[model];
    auto n_shapes = [](const mw::ChainModel& c) {
        size_t k = c.base_shapes.size();
        for (const auto& b : c.bodies) k += b.shapes.size();
        return k;
    };
    bool same = cm.dofs() == old.m.dofs() && cm.floating == old.m.floating && n_shapes(cm) == n_shapes(old.m);
    for (int i = 0; same && i < cm.dofs(); ++i) {
        same = cm.bodies[i].parent == old.m.bodies[i].parent && cm.bodies[i].shapes.size() == old.m.bodies[i].shapes.size();
        for (size_t k = 0; same && k < cm.bodies[i].shapes.size(); ++k)
            same = cm.bodies[i].shapes[k].type == old.m.bodies[i].shapes[k].type &&
                   cm.bodies[i].shapes[k].points.size() == old.m.bodies[i].shapes[k].points.size();
    }
    for (size_t k = 0; same && k < cm.base_shapes.size(); ++k)
        same = cm.base_shapes[k].type == old.m.base_shapes[k].type &&
               cm.base_shapes[k].points.size() == old.m.base_shapes[k].points.size();
    if (!same) return fail(MW_EINVAL, "the replacement model must have the same tree, base and collision shapes");
    const std::string nm = (name && *name) ? name : cm.name;
    for (size_t k = 0; k < s->models.size(); ++k)
        if (static_cast<int>(k) != model && s->models[k].name == nm)
            return fail(MW_EINVAL, "a model named '" + nm + "' is already in the scene");
    SceneModel sm = old;
    sm.m = cm;
    sm.name = nm;
    for (int k = 0; k < 7; ++k) sm.pose[k] = (pose ? pose : ident)[k];
    sm.controller = false;
    sm.period_ns = std::numeric_limits<int64_t>::max();
    sm.prev_ns = 0;
    sm.stepped = false;
    // commit only when the parameter block builds: on failure the slot keeps
    // its previous model (name, tree and device parameters stay consistent)
    SceneModel prev = old;
    old = sm;
    try {
        build_params(s);
    } catch (const std::exception& e) {
        s->models[model] = prev;
        try { build_params(s); } catch (const std::exception&) {}
        return fail(MW_EPARSE, e.what());
    }
    for (int i = 0; i < cm.dofs(); ++i) s->pid[s->models[model].body0 + i] = kDefaultPid;
    s->params_dirty = s->pid_dirty = true;
    return MW_OK;
}

int mw_scene_present(const mw_scene* s, int32_t model, int32_t w, int32_t* present) {
    if (int rc = check_model(s, model)) return rc;
    if (!present || w < 0 || w >= s->W) return fail(MW_EINVAL, "bad argument");
    *present = (s->h_present[w] >> model) & 1u;
    return MW_OK;
}

int mw_scene_n_worlds(const mw_scene* s, int32_t* n) {
    if (int rc = check(s)) return rc;
    if (!n) return fail(MW_EINVAL, "null argument");
    *n = s->W;
    return MW_OK;
}

int mw_scene_n_models(const mw_scene* s, int32_t* n) {
    if (int rc = check(s)) return rc;
    if (!n) return fail(MW_EINVAL, "null argument");
    *n = static_cast<int32_t>(s->models.size());
    return MW_OK;
}

int mw_scene_model_info(const mw_scene* s, int32_t model, int32_t* first, int32_t* n, int32_t* floating) {
    if (int rc = check_model(s, model)) return rc;
    const SceneModel& sm = s->models[model];
    if (first) *first = sm.body0;
    if (n) *n = sm.m.dofs();
    if (floating) *floating = sm.m.floating ? 1 : 0;
    return MW_OK;
}

int mw_scene_model_name(const mw_scene* s, int32_t model, char* buf, int32_t len) {
    if (int rc = check_model(s, model)) return rc;
    return copy_str(s->models[model].name, buf, len);
}

int mw_scene_base_frame(const mw_scene* s, int32_t model, char* buf, int32_t len) {
    if (int rc = check_model(s, model)) return rc;
    return copy_str(s->models[model].m.base_link, buf, len);
}

int mw_scene_joint_name(const mw_scene* s, int32_t dof, char* buf, int32_t len) {
    if (int rc = check(s)) return rc;
    const int m = s->model_of_dof(dof);
    if (m < 0) return fail(MW_EINVAL, "dof out of range");
    return copy_str(s->models[m].m.bodies[dof - s->models[m].body0].joint_name, buf, len);
}

int mw_scene_link_name(const mw_scene* s, int32_t dof, char* buf, int32_t len) {
    if (int rc = check(s)) return rc;
    const int m = s->model_of_dof(dof);
    if (m < 0) return fail(MW_EINVAL, "dof out of range");
    return copy_str(s->models[m].m.bodies[dof - s->models[m].body0].link_name, buf, len);
}

int mw_scene_joint_type(const mw_scene* s, int32_t dof, int32_t* type) {
    if (int rc = check(s)) return rc;
    const int m = s->model_of_dof(dof);
    if (m < 0 || !type) return fail(MW_EINVAL, "bad argument");
    const mw::ChainBody& b = s->models[m].m.bodies[dof - s->models[m].body0];
    *type = b.ball ? MW_JOINT_BALL : ((b.type == mw::JType::Prismatic) ? MW_JOINT_PRISMATIC : MW_JOINT_REVOLUTE);
    return MW_OK;
}

int mw_scene_model_export(const mw_scene* s, int32_t model, double* out, int32_t len) {
    if (int rc = check_model(s, model)) return rc;
    const mw::ChainModel& cm = s->models[model].m;
    const int n = cm.dofs();
    if (!out || len < 34 * n + 3) return fail(MW_EINVAL, "export buffer too small");
    double* o = out;
    for (const mw::ChainBody& b : cm.bodies) {
        *o++ = (b.type == mw::JType::Prismatic) ? 1.0 : 0.0;
        *o++ = b.limited ? 1.0 : 0.0;
        for (double v : b.E) *o++ = v;
        for (double v : b.r) *o++ = v;
        for (double v : b.axis) *o++ = v;
        *o++ = b.mass;
        for (double v : b.com) *o++ = v;
        for (double v : b.Ic) *o++ = v;
        *o++ = b.damping;
        *o++ = b.friction;
        *o++ = b.lower;
        *o++ = b.upper;
        *o++ = b.effort;
        *o++ = b.vel_limit;
        *o++ = b.parent;
    }
    const auto& R = cm.base_R;
    for (int k = 0; k < 3; ++k) *o++ = R[k] * s->gravity[0] + R[3 + k] * s->gravity[1] + R[6 + k] * s->gravity[2];
    if (len >= 34 * n + 7) {  // the base link's mass and COM (base frame)
        *o++ = cm.base_mass;
        for (int k = 0; k < 3; ++k) *o++ = cm.base_com[k];
    }
    return MW_OK;
}

static int scene_run(mw_scene* s, int32_t paused, bool defer, bool direct = false) {
    if (int rc = check(s)) return rc;
    if (s->models.empty()) {
        if (!paused) s->iterations += s->cfg.steps_per_run;
        return MW_OK;
    }
    if (int rc = flush(s, defer, direct)) return rc;
    mw::SceneDev D = s->dev;
    if (direct) {
        // the command block and the readback planes in the pinned mirror
        float* hj = s->h_joint_dev;
        const size_t r = s->jrows;
        D.cmd = hj + 3 * r; D.vtgt = hj + 4 * r; D.rq = hj + 5 * r; D.rqd = hj + 6 * r; D.ptgt = hj + 7 * r;
        D.act = reinterpret_cast<uint8_t*>(hj + 8 * r);
        D.rflag = D.act + r;
        D.rb = hj;
        D.rb_plane = static_cast<int32_t>(r);
    }
    mw::SceneArgs a{};
    a.dt = static_cast<float>(s->cfg.step_size);
    a.inv_dt = static_cast<float>(1.0 / s->cfg.step_size);
    a.paused = paused ? 1 : 0;
    a.pgs_iters = s->cfg.pgs_iters;
    a.lcp_solves = s->lcp_solves;
    a.first = 1;
    a.want_contacts = 1;
    const int spr = s->cfg.steps_per_run;
    int done = 0;
    do {
        const int chunk = paused ? 0 : std::min(64, spr - done);
        a.substeps = chunk;
        a.iter0 = static_cast<int32_t>(s->iterations + done);
        mw::SceneGates G{};
        // JointController::PreUpdate period gating per model (JointController.cpp:130-169)
        for (size_t m = 0; m < s->models.size(); ++m) {
            SceneModel& sm = s->models[m];
            for (int k = 0; k < chunk && sm.controller; ++k) {
                const int64_t sim_ns = (s->iterations + done + k + 1) * s->dt_ns;
                const int64_t elapsed = (sm.prev_ns == 0) ? sm.period_ns : sim_ns - sm.prev_ns;
                if (elapsed >= sm.period_ns) {
                    sm.prev_ns = sim_ns;
                    G.gate[m] |= uint64_t{1} << k;
                }
            }
        }
        SC_HIP(mw::launch_scene_run(s->dp, s->nv, D, s->d_pid, G, s->W, a, s->stream));
        s->idle = false;
        a.first = 0;
        done += chunk;
    } while (!paused && done < spr);
    if (!paused) {
        s->iterations += spr;
        for (auto& sm : s->models) sm.stepped = true;
        s->contacts_stale = true;
    }
    s->joints_stale = s->base_stale = true;
    return MW_OK;
}

// joint planes (q, qd, qdd) up to this size run direct (mw_scene_run)
constexpr size_t kDirectBytes = size_t{64} << 10;

int mw_scene_run(mw_scene* s, int32_t paused) {
    // one synchronisation per run: uploads, the launch and the readback of
    // the joint and base state are queued back to back
    // small scenes (the per-env path, BASELINE config 1) run direct: no
    // command upload, no joint readback copy -- one launch, one synchronisation
    const bool direct = s->h_joint_dev && 3 * s->jrows * sizeof(float) <= kDirectBytes;
    if (int rc = scene_run(s, paused, true, direct)) return rc;
    if (s->models.empty()) return MW_OK;
    // per-env runs: skip the copies that cannot carry news
    if (direct) {
        const size_t brows = static_cast<size_t>(13 * s->models.size()) * s->W * sizeof(float);
        if (brows && needs_base_readback(s))
            SC_HIP(hipMemcpyAsync(s->h_base, s->d_base, brows, hipMemcpyDeviceToHost, s->stream));
    } else if (int rc = queue_readback(s, needs_base_readback(s))) {
        return rc;
    }
    // the drop counter rides on the same synchronisation, and so does the
    // divergence count of the larger scenes (a direct run's state is in the
    // pinned mirror already: it is checked there, below)
    if (can_overflow(s))
        SC_HIP(hipMemcpyAsync(s->h_overflow, s->dev.overflow, sizeof(int32_t), hipMemcpyDeviceToHost, s->stream));
    if (!direct)
        SC_HIP(hipMemcpyAsync(s->h_ndiv, s->dev.overflow + 4, sizeof(uint64_t), hipMemcpyDeviceToHost, s->stream));
    if (int rc = sync(s)) return rc;
    clear_consumed(s);
    s->joints_stale = s->base_stale = false;
    if (direct) {
        // the kernel flags a world whose stored state is not finite; a direct
        // run reads the count only when its mirror holds such a value
        bool bad = false;
        const uint32_t* jb = reinterpret_cast<const uint32_t*>(s->h_joint);
        for (size_t k = 0; k < 2 * s->jrows && !bad; ++k) bad = (jb[k] & 0x7f800000u) == 0x7f800000u;
        if (!bad && needs_base_readback(s)) {
            const uint32_t* bb = reinterpret_cast<const uint32_t*>(s->h_base);
            const size_t nb = static_cast<size_t>(13 * s->models.size()) * s->W;
            for (size_t k = 0; k < nb && !bad; ++k) bad = (bb[k] & 0x7f800000u) == 0x7f800000u;
        }
        if (bad) {
            SC_HIP(hipMemcpyAsync(s->h_ndiv, s->dev.overflow + 4, sizeof(uint64_t), hipMemcpyDeviceToHost, s->stream));
            if (int rc = sync(s)) return rc;
        }
    }
    const int64_t dropped = *s->h_overflow;
    if (dropped > s->overflow_seen) {
        const int64_t d = dropped - s->overflow_seen;
        s->overflow_seen = dropped;
        char msg[256];
        std::snprintf(msg, sizeof msg,
                      "this run dropped %lld contact points / constraint rows: a world exceeded the per-step "
                      "capacity (%d contact points, %d constraint rows)",
                      static_cast<long long>(d), s->dev.big ? s->dev.big_cmax : CMAX,
                      s->dev.big ? s->dev.big_rows : mw::kScMaxRows);
        return fail(MW_ECAPACITY, msg);
    }
    const int64_t nd = static_cast<int64_t>(*s->h_ndiv);
    if (nd > s->div_seen) {
        const int64_t d = nd - s->div_seen;
        s->div_seen = nd;
        return fail(MW_EDIVERGED, std::to_string(d) + " world(s) diverged in this run: their joint or base state "
                                                      "is not finite (mw_scene_diverged lists them)");
    }
    return MW_OK;
}

int mw_scene_diverged(mw_scene* s, int32_t w0, int32_t nw, uint8_t* flags, int64_t* count) {
    if (int rc = check(s)) return rc;
    if (int rc = check_worlds(s, w0, nw)) return rc;
    if (flags && nw) SC_HIP(hipMemcpyAsync(flags, s->dev.diverged + w0, nw, hipMemcpyDeviceToHost, s->stream));
    uint64_t n = 0;
    SC_HIP(hipMemcpyAsync(&n, s->dev.overflow + 4, sizeof(n), hipMemcpyDeviceToHost, s->stream));
    SC_HIP(hipStreamSynchronize(s->stream));
    if (count) *count = static_cast<int64_t>(n);
    return MW_OK;
}

int mw_scene_clear_diverged(mw_scene* s, int32_t w0, int32_t nw) {
    if (int rc = check(s)) return rc;
    if (int rc = check_worlds(s, w0, nw)) return rc;
    if (nw) SC_HIP(hipMemsetAsync(s->dev.diverged + w0, 0, nw, s->stream));
    return MW_OK;
}

int mw_scene_run_device(mw_scene* s, int32_t runs) {
    if (runs < 0) return fail(MW_EINVAL, "runs must be >= 0");
    for (int32_t k = 0; k < runs; ++k)
        if (int rc = scene_run(s, 0, false)) return rc;
    return MW_OK;
}

int mw_scene_time(const mw_scene* s, double* t) {
    if (int rc = check(s)) return rc;
    if (!t) return fail(MW_EINVAL, "null argument");
    *t = static_cast<double>(s->iterations * s->dt_ns) / 1e9;
    return MW_OK;
}

int mw_scene_set_gravity(mw_scene* s, const double g[3]) {
    if (int rc = check(s)) return rc;
    if (!g) return fail(MW_EINVAL, "null argument");
    for (int k = 0; k < 3; ++k) s->gravity[k] = g[k];
    try { build_params(s); } catch (const std::exception& e) { return fail(MW_EPARSE, e.what()); }
    s->params_dirty = true;
    return mw_scene_set_world_gravity(s, 0, s->W, g);
}

// World::setGravity of the worlds [w0, w0 + nw) (World.cpp:301-319: every
// world has its own Gravity component)
int mw_scene_set_world_gravity(mw_scene* s, int32_t w0, int32_t nw, const double g[3]) {
    if (int rc = check(s)) return rc;
    if (!g) return fail(MW_EINVAL, "null argument");
    if (w0 < 0 || nw < 0 || w0 + nw > s->W) return fail(MW_EINVAL, "world range out of bounds");
    const size_t W = static_cast<size_t>(s->W);
    for (int w = w0; w < w0 + nw; ++w)
        for (int k = 0; k < 3; ++k) s->h_wphys[k * W + w] = static_cast<float>(g[k]);
    s->present_dirty = true;
    return MW_OK;
}

int mw_scene_world_gravity(const mw_scene* s, int32_t w, double g[3]) {
    if (int rc = check(s)) return rc;
    if (!g) return fail(MW_EINVAL, "null argument");
    if (w < 0 || w >= s->W) return fail(MW_EINVAL, "world out of range");
    for (int k = 0; k < 3; ++k) g[k] = s->h_wphys[static_cast<size_t>(k) * s->W + w];
    return MW_OK;
}

// friction coefficient of the ground plane of the worlds [w0, w0 + nw)
// (every contact of those worlds uses it)
int mw_scene_set_world_friction(mw_scene* s, int32_t w0, int32_t nw, double mu) {
    if (int rc = check(s)) return rc;
    if (!(mu >= 0.0)) return fail(MW_EINVAL, "the friction coefficient must be >= 0");
    if (w0 < 0 || nw < 0 || w0 + nw > s->W) return fail(MW_EINVAL, "world range out of bounds");
    for (int w = w0; w < w0 + nw; ++w) s->h_wphys[3 * static_cast<size_t>(s->W) + w] = static_cast<float>(mu);
    s->present_dirty = true;
    return MW_OK;
}

int mw_scene_gravity(const mw_scene* s, double g[3]) {
    if (int rc = check(s)) return rc;
    if (!g) return fail(MW_EINVAL, "null argument");
    for (int k = 0; k < 3; ++k) g[k] = s->gravity[k];
    return MW_OK;
}

int mw_scene_set_ground_plane(mw_scene* s, int32_t enabled, double mu) {
    if (int rc = check(s)) return rc;
    if (!(mu >= 0.0)) return fail(MW_EINVAL, "the friction coefficient must be >= 0");
    // the plane's friction is scene-wide; its presence is a per-world bit
    // (mw_scene_set_world_ground), set here for every world
    s->ground = true;
    s->mu = mu;
    try { build_params(s); } catch (const std::exception& e) { return fail(MW_EPARSE, e.what()); }
    s->params_dirty = true;
    if (int rc = mw_scene_set_world_friction(s, 0, s->W, mu)) return rc;
    return mw_scene_set_world_ground(s, 0, s->W, enabled);
}

int mw_scene_get_joints(const mw_scene* cs, int32_t field, int32_t w0, int32_t nw, const int32_t* dofs, int32_t nd,
                        double* out) {
    mw_scene* s = const_cast<mw_scene*>(cs);
    if (int rc = check(s)) return rc;
    if (!out && nw > 0) return fail(MW_EINVAL, "null argument");
    std::vector<int32_t> sel;
    if (int rc = selection(s, w0, nw, dofs, nd, sel)) return rc;
    if (field <= MW_SC_ACCELERATION || field == MW_SC_FORCE)
        if (int rc = pull_joints(s)) return rc;
    const size_t m = sel.size();
    for (int32_t w = 0; w < nw; ++w)
        for (size_t k = 0; k < m; ++k) {
            const size_t i = s->jidx(sel[k], w0 + w);
            double v = 0.0;
            switch (field) {
            case MW_SC_POSITION: v = s->hq()[i]; break;
            case MW_SC_VELOCITY: v = s->hqd()[i]; break;
            case MW_SC_ACCELERATION: v = s->hqdd()[i]; break;
            case MW_SC_FORCE_TARGET: v = s->cmd64[i]; break;
            case MW_SC_VELOCITY_TARGET: v = s->hvt()[i]; break;
            case MW_SC_POSITION_TARGET: v = s->ptgt64[i]; break;
            // DART clears the joint forces at the end of World::step, so the
            // JointForce readback (Physics.cpp:2330-2345) is 0
            case MW_SC_FORCE: v = 0.0; break;
            default: return fail(MW_EINVAL, "unknown joint field");
            }
            out[w * m + k] = v;
        }
    return MW_OK;
}

int mw_scene_set_joints(mw_scene* s, int32_t field, int32_t w0, int32_t nw, const int32_t* dofs, int32_t nd,
                        const double* v) {
    if (int rc = check(s)) return rc;
    if (!v && nw > 0) return fail(MW_EINVAL, "null argument");
    std::vector<int32_t> sel;
    if (int rc = selection(s, w0, nw, dofs, nd, sel)) return rc;
    const size_t m = sel.size();
    // validate first (Joint.cpp:694-815 mode checks): a failing call changes nothing
    for (int32_t w = 0; w < nw; ++w)
        for (size_t k = 0; k < m; ++k) {
            const int md = s->mode[s->jidx(sel[k], w0 + w)];
            switch (field) {
            case MW_SC_FORCE_TARGET:
                if (md != MW_MODE_FORCE && md != MW_MODE_POSITION && md != MW_MODE_POSITION_INTERPOLATED &&
                    md != MW_MODE_VELOCITY)
                    return fail(MW_ESTATE, "The active joint control mode does not accept a force target");
                break;
            case MW_SC_VELOCITY_TARGET:
                if (md != MW_MODE_VELOCITY && md != MW_MODE_VELOCITY_FOLLOWER_DART && md != MW_MODE_FORCE)
                    return fail(MW_ESTATE, "The active joint control mode does not accept a velocity target");
                break;
            case MW_SC_POSITION_TARGET:
                if (md != MW_MODE_POSITION && md != MW_MODE_POSITION_INTERPOLATED && md != MW_MODE_IDLE &&
                    md != MW_MODE_FORCE)
                    return fail(MW_ESTATE, "The active joint control mode does not accept a position target");
                break;
            case MW_SC_RESET_POSITION:
            case MW_SC_RESET_VELOCITY:
                break;
            default:
                return fail(MW_EINVAL, "field is not settable");
            }
        }
    for (int32_t w = 0; w < nw; ++w)
        for (size_t k = 0; k < m; ++k) {
            const size_t i = s->jidx(sel[k], w0 + w);
            const double x = v[w * m + k];
            switch (field) {
            case MW_SC_FORCE_TARGET: s->cmd64[i] = x; s->hcmd()[i] = static_cast<float>(x); break;
            case MW_SC_VELOCITY_TARGET: s->hvt()[i] = static_cast<float>(x); break;
            case MW_SC_POSITION_TARGET: s->ptgt64[i] = x; s->hptgt()[i] = static_cast<float>(x); break;
            // Joint::resetPosition / resetVelocity also reset the PID (Joint.cpp:132-180)
            case MW_SC_RESET_POSITION: s->hrq()[i] = static_cast<float>(x); s->hrflag()[i] |= 1u | 4u; break;
            case MW_SC_RESET_VELOCITY: s->hrqd()[i] = static_cast<float>(x); s->hrflag()[i] |= 2u | 4u; break;
            default: break;
            }
        }
    s->cmd_dirty = true;
    if (field == MW_SC_RESET_POSITION || field == MW_SC_RESET_VELOCITY) return rearm_diverged(s, w0, nw);
    return MW_OK;
}

int mw_scene_set_control_mode(mw_scene* s, int32_t w0, int32_t nw, const int32_t* dofs, int32_t nd, int32_t mode) {
    if (int rc = check(s)) return rc;
    // Joint::setControlMode, Joint.cpp:369-460
    if (mode == MW_MODE_POSITION_INTERPOLATED) return fail(MW_EINVAL, "PositionInterpolated not yet supported");
    if (mode != MW_MODE_IDLE && mode != MW_MODE_FORCE && mode != MW_MODE_VELOCITY_FOLLOWER_DART &&
        mode != MW_MODE_POSITION && mode != MW_MODE_VELOCITY)
        return fail(MW_EINVAL, "You cannot set the Invalid control mode");
    std::vector<int32_t> sel;
    if (int rc = selection(s, w0, nw, dofs, nd, sel)) return rc;
    if (int rc = pull_joints(s)) return rc;
    for (int32_t w = w0; w < w0 + nw; ++w)
        for (int32_t dof : sel) {
            const size_t i = s->jidx(dof, w);
            s->mode[i] = mode;
            // targets deleted and re-initialised from the current state (:418-446)
            s->hcmd()[i] = 0.f;
            s->cmd64[i] = 0.0;
            const bool vel = (mode == MW_MODE_VELOCITY_FOLLOWER_DART || mode == MW_MODE_VELOCITY);
            s->hvt()[i] = vel ? s->hqd()[i] : 0.f;
            s->ptgt64[i] = s->hq()[i];
            s->hptgt()[i] = s->hq()[i];
            uint8_t act = mw::kActForce;
            if (mode == MW_MODE_VELOCITY_FOLLOWER_DART) act = mw::kActServo;
            else if (mode == MW_MODE_POSITION) act = mw::kActPidPos;
            else if (mode == MW_MODE_VELOCITY) act = mw::kActPidVel;
            s->hact()[i] = act;
            s->hrflag()[i] |= 4u;  // pid.Reset() (:453-457)
        }
    if (mode == MW_MODE_POSITION || mode == MW_MODE_VELOCITY || mode == MW_MODE_VELOCITY_FOLLOWER_DART)
        for (int32_t dof : sel) s->models[s->model_of_dof(dof)].controller = true;
    s->cmd_dirty = true;
    return MW_OK;
}

int mw_scene_control_mode(const mw_scene* s, int32_t w, int32_t dof, int32_t* mode) {
    if (int rc = check(s)) return rc;
    if (!mode || w < 0 || w >= s->W || dof < 0 || dof >= s->NB) return fail(MW_EINVAL, "index out of range");
    *mode = s->mode[s->jidx(dof, w)];
    return MW_OK;
}

int mw_scene_set_joint_pid(mw_scene* s, int32_t dof, const double gains[8]) {
    if (int rc = check(s)) return rc;
    if (!gains || dof < 0 || dof >= s->NB) return fail(MW_EINVAL, "bad argument");
    // Joint::setPID, Joint.cpp:479-525
    std::array<double, 8> g;
    std::memcpy(g.data(), gains, sizeof(double) * 8);
    const int m = s->model_of_dof(dof);
    const double maxf = s->models[m].m.bodies[dof - s->models[m].body0].effort;
    if (g[3] < -maxf || g[4] > maxf) {
        g[3] = -maxf;
        g[4] = maxf;
    }
    s->pid[dof] = g;
    s->pid_dirty = true;
    for (int32_t w = 0; w < s->W; ++w) s->hrflag()[s->jidx(dof, w)] |= 4u;
    s->cmd_dirty = true;
    return MW_OK;
}

int mw_scene_joint_pid(const mw_scene* s, int32_t dof, double gains[8]) {
    if (int rc = check(s)) return rc;
    if (!gains || dof < 0 || dof >= s->NB) return fail(MW_EINVAL, "bad argument");
    std::memcpy(gains, s->pid[dof].data(), sizeof(double) * 8);
    return MW_OK;
}

int mw_scene_set_joint_param(mw_scene* s, int32_t dof, int32_t which, double value) {
    if (int rc = check(s)) return rc;
    const int m = s->model_of_dof(dof);
    if (m < 0) return fail(MW_EINVAL, "dof out of range");
    SceneModel& sm = s->models[m];
    // Joint.cpp:262-266: parameters can change only while the model was just created
    if (sm.stepped) return fail(MW_ESTATE, "The model has been already processed and its parameters cannot be modified");
    mw::ChainBody& b = sm.m.bodies[dof - sm.body0];
    switch (which) {
    case MW_PARAM_COULOMB_FRICTION: b.friction = value; break;
    case MW_PARAM_VISCOUS_FRICTION: b.damping = value; break;
    case MW_PARAM_MAX_GENERALIZED_FORCE: b.effort = value; break;
    case MW_PARAM_POSITION_LIMIT_MIN: b.lower = value; break;
    case MW_PARAM_POSITION_LIMIT_MAX: b.upper = value; break;
    default: return fail(MW_EINVAL, "unknown joint parameter");
    }
    try { build_params(s); } catch (const std::exception& e) { return fail(MW_EPARSE, e.what()); }
    s->params_dirty = true;
    return MW_OK;
}

int mw_scene_joint_param(const mw_scene* s, int32_t dof, int32_t which, double* value) {
    if (int rc = check(s)) return rc;
    const int m = s->model_of_dof(dof);
    if (m < 0 || !value) return fail(MW_EINVAL, "bad argument");
    const mw::ChainBody& b = s->models[m].m.bodies[dof - s->models[m].body0];
    switch (which) {
    case MW_PARAM_COULOMB_FRICTION: *value = b.friction; break;
    case MW_PARAM_VISCOUS_FRICTION: *value = b.damping; break;
    case MW_PARAM_MAX_GENERALIZED_FORCE: *value = b.effort; break;
    case MW_PARAM_POSITION_LIMIT_MIN: *value = b.lower; break;
    case MW_PARAM_POSITION_LIMIT_MAX: *value = b.upper; break;
    default: return fail(MW_EINVAL, "unknown joint parameter");
    }
    return MW_OK;
}

int mw_scene_set_controller_period(mw_scene* s, int32_t model, double period) {
    if (int rc = check_model(s, model)) return rc;
    // Model::setControllerPeriod, Model.cpp:589-602
    if (!(period > 0.0)) return fail(MW_EINVAL, "The controller period must be greater than zero");
    const double ns = period * 1e9;
    s->models[model].period_ns = ns >= 9.2e18 ? std::numeric_limits<int64_t>::max() : static_cast<int64_t>(ns);
    return MW_OK;
}

int mw_scene_controller_period(const mw_scene* s, int32_t model, double* period) {
    if (int rc = check_model(s, model)) return rc;
    if (!period) return fail(MW_EINVAL, "null argument");
    *period = static_cast<double>(s->models[model].period_ns) / 1e9;
    return MW_OK;
}

int mw_scene_get_base_pose(const mw_scene* cs, int32_t model, int32_t w0, int32_t nw, double* out) {
    mw_scene* s = const_cast<mw_scene*>(cs);
    if (int rc = check_model(s, model)) return rc;
    if (int rc = check_worlds(s, w0, nw)) return rc;
    if (int rc = pull_base(s)) return rc;
    const SceneModel& sm = s->models[model];
    for (int w = 0; w < nw; ++w) {
        if (!sm.m.floating) {
            double q[4];
            quat_of(sm.m.base_R, q);
            const double v[7] = {sm.m.base_p[0], sm.m.base_p[1], sm.m.base_p[2], q[0], q[1], q[2], q[3]};
            for (int f = 0; f < 7; ++f) out[w * 7 + f] = v[f];
        } else {
            for (int f = 0; f < 7; ++f) out[w * 7 + f] = *s->hbase(model, f, w0 + w);
        }
    }
    return MW_OK;
}

int mw_scene_get_base_velocity(const mw_scene* cs, int32_t model, int32_t w0, int32_t nw, double* out) {
    mw_scene* s = const_cast<mw_scene*>(cs);
    if (int rc = check_model(s, model)) return rc;
    if (int rc = check_worlds(s, w0, nw)) return rc;
    if (int rc = pull_base(s)) return rc;
    for (int w = 0; w < nw; ++w) {
        // body-frame twist [w; v] -> world linear (origin), world angular
        auto at = [&](int f) { return static_cast<double>(*s->hbase(model, f, w0 + w)); };
        const double qw = at(3), qx = at(4), qy = at(5), qz = at(6);
        const double R[9] = {1 - 2 * (qy * qy + qz * qz), 2 * (qx * qy - qw * qz), 2 * (qx * qz + qw * qy),
                             2 * (qx * qy + qw * qz), 1 - 2 * (qx * qx + qz * qz), 2 * (qy * qz - qw * qx),
                             2 * (qx * qz - qw * qy), 2 * (qy * qz + qw * qx), 1 - 2 * (qx * qx + qy * qy)};
        const double wb[3] = {at(7), at(8), at(9)}, vb[3] = {at(10), at(11), at(12)};
        for (int r = 0; r < 3; ++r) {
            out[w * 6 + r] = R[r * 3] * vb[0] + R[r * 3 + 1] * vb[1] + R[r * 3 + 2] * vb[2];
            out[w * 6 + 3 + r] = R[r * 3] * wb[0] + R[r * 3 + 1] * wb[1] + R[r * 3 + 2] * wb[2];
        }
        if (!s->models[model].m.floating)
            for (int f = 0; f < 6; ++f) out[w * 6 + f] = 0.0;
    }
    return MW_OK;
}

int mw_scene_reset_base_pose(mw_scene* s, int32_t model, int32_t w0, int32_t nw, const double* pose) {
    if (int rc = check_model(s, model)) return rc;
    if (int rc = check_worlds(s, w0, nw)) return rc;
    if (!pose) return fail(MW_EINVAL, "null argument");
    if (!s->models[model].m.floating) return fail(MW_ESTATE, "the model has a fixed base");
    for (int w = 0; w < nw; ++w) {
        for (int f = 0; f < 7; ++f) *s->hrpose(model, f, w0 + w) = static_cast<float>(pose[w * 7 + f]);
        s->hbflag()[static_cast<size_t>(model) * s->W + w0 + w] |= 1u;
    }
    s->base_dirty = true;
    return rearm_diverged(s, w0, nw);
}

int mw_scene_reset_base_velocity(mw_scene* s, int32_t model, int32_t w0, int32_t nw, const double* v) {
    if (int rc = check_model(s, model)) return rc;
    if (int rc = check_worlds(s, w0, nw)) return rc;
    if (!v) return fail(MW_EINVAL, "null argument");
    if (!s->models[model].m.floating) return fail(MW_ESTATE, "the model has a fixed base");
    for (int w = 0; w < nw; ++w) {
        for (int f = 0; f < 6; ++f) *s->hrvel(model, f, w0 + w) = static_cast<float>(v[w * 6 + f]);
        s->hbflag()[static_cast<size_t>(model) * s->W + w0 + w] |= 2u;
    }
    s->base_dirty = true;
    return rearm_diverged(s, w0, nw);
}

int mw_scene_get_contacts(const mw_scene* cs, int32_t w, double* out, int32_t cap, int32_t* n) {
    mw_scene* s = const_cast<mw_scene*>(cs);
    if (int rc = check(s)) return rc;
    if (!n || w < 0 || w >= s->W) return fail(MW_EINVAL, "bad argument");
    if (int rc = pull_contacts(s)) return rc;
    const int nc = std::min(s->h_ncontact[w], s->contact_cap);
    *n = nc;
    const mw::SceneF& P = s->hp;
    for (int c = 0; c < nc && c < cap; ++c) {
        auto at = [&](int f) { return s->h_contact[(static_cast<size_t>(c) * 12 + f) * s->W + w]; };
        for (int f = 0; f < 10; ++f) out[c * 14 + f] = at(f);
        int32_t na, nb;
        const float fa = at(10), fb = at(11);
        std::memcpy(&na, &fa, 4);
        std::memcpy(&nb, &fb, 4);
        for (int side = 0; side < 2; ++side) {
            const int nd = side ? nb : na;
            double mo = -1.0, li = -1.0;
            if (nd >= 0) {
                mo = P.node_model[nd];
                const int bd = P.node_body[nd];
                li = bd < 0 ? -1.0 : static_cast<double>(bd - s->models[P.node_model[nd]].body0);
            }
            out[c * 14 + 10 + 2 * side] = mo;
            out[c * 14 + 11 + 2 * side] = li;
        }
    }
    return MW_OK;
}

int mw_scene_apply_world_wrench(mw_scene* s, int32_t model, int32_t link, int32_t w0, int32_t nw,
                                const double* wrench, double duration) {
    if (int rc = check_model(s, model)) return rc;
    if (int rc = check_worlds(s, w0, nw)) return rc;
    if (!wrench) return fail(MW_EINVAL, "null argument");
    const SceneModel& sm = s->models[model];
    if (link < -1 || link >= sm.m.dofs()) return fail(MW_EINVAL, "link index out of range");
    if (!(duration >= 0.0)) return fail(MW_EINVAL, "the wrench duration must be >= 0");
    const int node = sm.node0 + 1 + link;
    // applied from the next physics step for max(1, ceil(duration / dt)) steps
    // (expiry = now + duration, removed after the step whose time reaches it)
    const int64_t d_ns = static_cast<int64_t>(duration * 1e9);
    const int64_t k = std::max<int64_t>(1, (d_ns + s->dt_ns - 1) / s->dt_ns);
    const int64_t last = s->iterations + k;
    if (last > std::numeric_limits<int32_t>::max()) return fail(MW_EINVAL, "wrench expiry beyond the counter range");
    for (int w = w0; w < w0 + nw; ++w) {
        int slot = -1;
        for (int sl = 0; sl < SLOTS && slot < 0; ++sl)
            if (s->h_wlast[(static_cast<size_t>(sl) * NNMAX + node) * s->W + w] == last) slot = sl;
        for (int sl = 0; sl < SLOTS && slot < 0; ++sl)
            if (s->h_wlast[(static_cast<size_t>(sl) * NNMAX + node) * s->W + w] <= s->iterations) {
                slot = sl;
                for (int e = 0; e < 6; ++e)
                    s->h_wrench[((static_cast<size_t>(sl) * 6 + e) * NNMAX + node) * s->W + w] = 0.f;
            }
        if (slot < 0) return fail(MW_ESTATE, "too many concurrent wrenches with different durations on one link");
        s->h_wlast[(static_cast<size_t>(slot) * NNMAX + node) * s->W + w] = static_cast<int32_t>(last);
        for (int e = 0; e < 6; ++e)
            s->h_wrench[((static_cast<size_t>(slot) * 6 + e) * NNMAX + node) * s->W + w] +=
                static_cast<float>(wrench[(w - w0) * 6 + e]);
    }
    s->wrench_dirty = true;
    return MW_OK;
}

int mw_scene_set_lcp_solver(mw_scene* s, int32_t mode, int32_t max_solves) {
    if (int rc = check(s)) return rc;
    if (mode != MW_LCP_PGS && mode != MW_LCP_EXACT) return fail(MW_EINVAL, "unknown LCP solver mode");
    if (mode == MW_LCP_EXACT && (max_solves < 1 || max_solves > 256))
        return fail(MW_EINVAL, "the exact solve's budget must be 1..256 linear solves per step");
    s->lcp_mode = mode;
    s->lcp_solves = (mode == MW_LCP_EXACT) ? max_solves : 0;
    return MW_OK;
}

int mw_scene_lcp_solver(const mw_scene* s, int32_t* mode, int32_t* max_solves) {
    if (int rc = check(s)) return rc;
    if (!mode || !max_solves) return fail(MW_EINVAL, "null argument");
    *mode = s->lcp_mode;
    *max_solves = s->lcp_solves;
    return MW_OK;
}

int mw_scene_lcp_unconverged(const mw_scene* s, int64_t* world_steps) {
    if (int rc = check(s)) return rc;
    if (!world_steps) return fail(MW_EINVAL, "null argument");
    uint64_t v = 0;
    SC_HIP(hipMemcpyAsync(&v, s->dev.overflow + 2, sizeof(v), hipMemcpyDeviceToHost, s->stream));
    SC_HIP(hipStreamSynchronize(s->stream));
    *world_steps = static_cast<int64_t>(v);
    return MW_OK;
}

int mw_scene_overflow(const mw_scene* s, int64_t* dropped) {
    if (int rc = check(s)) return rc;
    if (!dropped) return fail(MW_EINVAL, "null argument");
    int v = 0;
    SC_HIP(hipMemcpyAsync(&v, s->dev.overflow, sizeof(int), hipMemcpyDeviceToHost, s->stream));
    SC_HIP(hipStreamSynchronize(s->stream));
    *dropped = v;
    return MW_OK;
}

}  // extern "C"

// ---- test hook (include/mwstep_testhooks.h): the hull the scene kernel's mesh
// narrow phase uses for a point set (hull.hpp build_hull; host only) ----------
extern "C" int mw_debug_hull(const double* pts, int32_t n, double* planes, int32_t* faces, int32_t* edges,
                             int32_t* counts) {
    if (!pts || !planes || !faces || !edges || !counts || n < 1 || n > mw::kHullMaxV) return MW_EINVAL;
    std::vector<std::array<double, 3>> v(static_cast<size_t>(n));
    for (int i = 0; i < n; ++i) v[i] = {pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]};
    mw::HostHull h;
    if (!mw::build_hull(v, h)) {
        counts[0] = counts[1] = 0;
        return MW_OK;
    }
    counts[0] = h.nf;
    counts[1] = h.ne;
    for (int f = 0; f < h.nf; ++f) {
        for (int k = 0; k < 3; ++k) planes[4 * f + k] = h.n[f][k];
        planes[4 * f + 3] = h.d[f];
        faces[17 * f] = h.fnv[f];
        for (int t = 0; t < h.fnv[f]; ++t) faces[17 * f + 1 + t] = h.fv[f][t];
    }
    for (int e = 0; e < h.ne; ++e) {
        edges[4 * e] = h.e[e][0];
        edges[4 * e + 1] = h.e[e][1];
        edges[4 * e + 2] = h.ef[e][0];
        edges[4 * e + 3] = h.ef[e][1];
    }
    return MW_OK;
}

// test hook (include/mwstep_testhooks.h): world w's large-contact workspace
extern "C" int mw_debug_scene_big_ws(mw_scene* s, int32_t w, float* out, int64_t cap, int32_t* cmax, int32_t* rows) {
    if (int rc = check(s)) return rc;
    if (!out || !cmax || !rows || w < 0 || w >= s->W) return fail(MW_EINVAL, "bad argument");
    const mw::SceneDev& D = s->dev;
    *cmax = D.big ? D.big_cmax : 0;
    *rows = D.big ? D.big_rows : 0;
    if (!D.big) return MW_OK;
    const int64_t n = std::min<int64_t>(cap, static_cast<int64_t>(mw::kScBigContactWords) * D.big_cmax +
                                                  11LL * D.big_rows);
    SC_HIP(hipStreamSynchronize(s->stream));
    SC_HIP(hipMemcpy(out, D.big + static_cast<size_t>(w) * static_cast<size_t>(D.big_stride), n * sizeof(float),
                     hipMemcpyDeviceToHost));
    return MW_OK;
}
