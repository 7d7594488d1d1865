// sim.cpp -- C ABI (include/mwstep.h) of the many-worlds stepper.
//
// Host-side counterpart of the reference's GazeboSimulator + ECM components
// (cpp/scenario/gazebo/src/GazeboSimulator.cpp, Joint.cpp, Model.cpp):
// component reads/writes become reads/writes of a host mirror of the device
// SoA arrays; one run() = [one H2D copy of the command slab if dirty] +
// one kernel + one D2H copy of the readback slab.
#include "mwstep.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "baked_models.hpp"
#include "chain_params.hpp"
#include "float_tree.hpp"
#include "free_body.hpp"
#include "kernels.hpp"
#include "model.hpp"
#include "errors.hpp"

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

}  // namespace

// the calling thread's last error (mw_last_error), shared with scene.cpp
void mw::set_last_error(const std::string& msg) { g_last_error = msg; }

namespace {

#define MW_HIP(call)                                                                      \
    do {                                                                                  \
        hipError_t e_ = (call);                                                           \
        if (e_ != hipSuccess)                                                             \
            return fail(MW_EHIP, std::string(#call " failed: ") + hipGetErrorString(e_)); \
    } while (0)

}  // namespace

struct mw_sim {
    mw_config cfg{};
    bool own_stream = false;
    bool stream_set = false;  // mw_set_stream called (NULL = the legacy default stream)
    hipStream_t stream = nullptr;
    bool loaded = false;
    bool initialized = false;
    bool stepped = false;     // model parameters become read-only after the first run
    bool servo_used = false;  // a joint was put in VelocityFollowerDart
    bool host_stale = false;  // device state changed by the VecEnv path
    bool cmd_dirty = true;
    bool ptgt_dirty = false;  // host position targets newer than the device copy
    bool ptgt_stale = false;  // device position targets newer than the host mirror
    bool ptgt_view = false;   // a device view of the targets was handed out (always re-read)
    int topo = 0;             // kernel topology id (kernels.hpp: kernel_topology)
    mw::ChainModel model;
    std::string model_name;
    double gravity[3] = {0.0, 0.0, -9.8};  // sdformat default world gravity
    int64_t iterations = 0;
    int64_t dt_ns = 0;
    // JointController (one per model): Model.cpp:181-185 initialises the period
    // to the maximum duration; the plugin is inserted by the first Position /
    // Velocity / VelocityFollowerDart joint (Joint.cpp:376-404)
    bool controller = false;
    int64_t period_ns = std::numeric_limits<int64_t>::max();
    int64_t prev_ns = 0;      // JointController prevUpdateTime (0 = first iteration)
    // JointPID per dof in scenario::core::PID order {p, i, d, cmdMin, cmdMax,
    // cmdOffset, iMin, iMax}; default = Joint.cpp:63 DefaultPID
    std::vector<std::array<double, 8>> pid;

    int n = 0, W = 0;
    size_t nw = 0;  // n * W
    // device block layout: [q qd qdd | cmd vtgt rq rqd | act rflag]; the host
    // mirror has the same layout so the command slab moves in one copy
    void* d_block = nullptr;
    uint8_t* h_block = nullptr;
    size_t block_bytes = 0, cmd_off = 0, cmd_bytes = 0, state_bytes = 0;
    mw::ChainF* d_params = nullptr;
    mw::ChainF h_params{};
    // [ptgt | pid_e | pid_i | pid_u | qlo] on the device; h_ptgt mirrors ptgt
    float* d_aux = nullptr;
    float* h_ptgt = nullptr;
    // pinned staging copy of [command slab | position targets]: the H2D copies
    // of a run read it, so the host mirror can be cleared / rewritten right
    // after the launch; stage_ev marks when the last copy out of it finished
    uint8_t* h_stage = nullptr;
    hipEvent_t stage_ev = nullptr;
    bool stage_pending = false;
    // floating single-body models (free_body.hpp)
    bool floating = false;
    bool ground = false;          // a ground plane z = 0 is in the world
    double ground_mu = 1.0;       // SDF <surface><friction><ode><mu> default
    bool contacts = false;        // Model::enableContacts
    mw::FreeF h_free{};
    mw::FreeF* d_free = nullptr;
    mw::FreeDev fdev{};
    void* d_fblock = nullptr;     // [base 13 | rpose 7 | rvel 6 | contacts 7*slots][W] f32 + rflag u8 + cmask u32
    float* h_base = nullptr;      // [13][W] host mirror (pinned)
    float* h_cdata = nullptr;     // [slots][7][W]
    uint32_t* h_cmask = nullptr;  // [W]
    std::vector<float> h_rpose, h_rvel;
    std::vector<uint8_t> h_rflag;
    bool free_dirty = false;
    bool contacts_stale = false;  // contacts written on the device by mw_run_device
    // articulated models on a floating base (float_tree.hpp): the joint state
    // of a fixed-base model plus the base block above
    bool float_tree = false;
    // a fixed-base tree outside the compiled chain topologies (more than 9
    // dofs, or branched other than the Panda): the world-per-wavefront kernel
    // with a welded base (FloatF::fixed); its joint and base state live where a
    // floating tree's do
    bool fixed_tree = false;
    bool fbase() const { return floating || fixed_tree; }
    mw::FloatF h_float{};
    mw::FloatF* d_float = nullptr;
    float* d_ws = nullptr;        // constraint-row workspace [words][W]
    int n_slots = mw::kMaxFreeSlots;
    std::vector<int32_t> slot_body;  // body of every contact slot (-1 = base)
    // large trees (or MWSTEP_WAVE_TREE=1): one world per wavefront (wave_tree.hpp)
    bool wave = false;
    bool wave_depth_ok = false;   // the tree fits the wave kernel's depth stack
    int wave_depth = 0;           // the tree's depth in joints (picks the wave kernel's instance)
    mw::PidF* d_pid = nullptr;    // PID gains of every dof (device)
    mw::PidF* h_pid = nullptr;    // pinned staging copy
    bool pid_dirty = true;        // gains changed since the last upload
    int* d_overflow = nullptr;    // constraint rows dropped by the wave kernel
    float* d_warm = nullptr;      // wave kernel: previous step's PGS impulses [kWaveWarmWordsHost][W]
    double pgs_tol = 0.0;         // mw_set_pgs_options
    bool pgs_warm = false;
    // world wrenches (mw_apply_link_wrench, wave kernel): host records
    // [slot][6][node][W] / [slot][node][W], device copies, the last iteration
    // any record covers
    std::vector<float> h_wr;
    std::vector<int32_t> h_wl;
    float* d_ext = nullptr;        // [6][node][W]: the summed wrenches of one launch
    float* h_ext = nullptr;        // pinned staging of d_ext
    int64_t wr_until = 0;
    int* h_overflow = nullptr;    // pinned copy read back with each synchronous run
    int64_t overflow_seen = 0;    // drops already reported
    // divergence detection: [W] sticky per-world flags + the uint64 count of
    // worlds flagged (device), its pinned copy (read back with every
    // synchronous run) and the flags already reported
    uint8_t* d_health = nullptr;
    uint64_t* h_ndiv = nullptr;
    int64_t div_seen = 0;
    int32_t lcp_mode = MW_LCP_EXACT;  // mw_set_lcp_solver (wave kernel)
    int32_t lcp_solves = 48;          // linear-solve budget of the exact solve per step (r06: a random humanoid impact needed 25-32)
    mw::SimDev dev;
    // host-only component data
    std::vector<int32_t> mode;      // JointControlMode per [d][w]
    std::vector<double> ptgt;       // JointPositionTarget
    std::vector<double> cmd64;      // JointForceCmd exactly as set (double)

    float* hq() { return reinterpret_cast<float*>(h_block); }
    float* hqd() { return hq() + nw; }
    float* hqdd() { return hq() + 2 * nw; }
    float* hcmd() { return hq() + 3 * nw; }
    float* hvt() { return hq() + 4 * nw; }
    float* hrq() { return hq() + 5 * nw; }
    float* hrqd() { return hq() + 6 * nw; }
    uint8_t* hact() { return h_block + 7 * nw * sizeof(float); }
    uint8_t* hrflag() { return hact() + nw; }
    size_t idx(int d, int w) const { return static_cast<size_t>(d) * W + w; }
};

struct mw_vecenv {
    mw_sim* sim = nullptr;
    mw_task_config cfg{};
    mw::TaskF task{};
    mw::VecDev dev{};
    void* d_counters = nullptr;
    void* d_physics = nullptr;  // per-world randomised masses + gravity
    // lane-group Panda kernel: per-dof PID gains + reset pose (device), and
    // the host copy last uploaded
    mw::GLaneTask* d_lane = nullptr;
    mw::GLaneTask h_lane[mw::kMaxKernelDofs] = {};
    bool lane_uploaded = false;
};

namespace {

int check_sim(const mw_sim* s, bool need_init = true) {
    if (!s) return fail(MW_EINVAL, "null simulator handle");
    if (need_init && !s->initialized) return fail(MW_ESTATE, "the simulator was not initialized");
    return MW_OK;
}

void build_params(mw_sim* s) {
    mw::ChainF& P = s->h_params;
    std::memset(&P, 0, sizeof(P));
    P.n = s->n;
    // gravity in the base frame: R_base^T g
    const auto& R = s->model.base_R;
    for (int k = 0; k < 3; ++k)
        P.g[k] = static_cast<float>(R[k] * s->gravity[0] + R[3 + k] * s->gravity[1] + R[6 + k] * s->gravity[2]);
    int flags = 0;
    for (int i = 0; i < s->n; ++i) {
        const mw::ChainBody& b = s->model.bodies[i];
        mw::BodyF& f = P.b[i];
        // rotation entries below 1e-12 are the residue of cos(pi/2) etc. in the
        // rpy conversion: exact zeros let the constant-folded kernels drop them
        // (a 6e-17 change, far below float32 resolution of the unit entries)
        auto snap = [](double v) { return std::fabs(v) < 1e-12 ? 0.0 : v; };
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
        // inertia about the body origin: Ic + m (|c|^2 1 - c c^T)
        const double c2 = b.com[0] * b.com[0] + b.com[1] * b.com[1] + b.com[2] * b.com[2];
        f.Io[0] = static_cast<float>(b.Ic[0] + b.mass * (c2 - b.com[0] * b.com[0]));
        f.Io[1] = static_cast<float>(b.Ic[1] + b.mass * (c2 - b.com[1] * b.com[1]));
        f.Io[2] = static_cast<float>(b.Ic[2] + b.mass * (c2 - b.com[2] * b.com[2]));
        f.Io[3] = static_cast<float>(b.Ic[3] - b.mass * b.com[0] * b.com[1]);
        f.Io[4] = static_cast<float>(b.Ic[4] - b.mass * b.com[0] * b.com[2]);
        f.Io[5] = static_cast<float>(b.Ic[5] - b.mass * b.com[1] * b.com[2]);
        f.damping = static_cast<float>(b.damping);
        f.friction = static_cast<float>(b.friction);
        auto clampf = [](double v) {
            const double big = static_cast<double>(std::numeric_limits<float>::max());
            // "unlimited" is FLT_MAX on the device (finite-math-only kernels)
            return static_cast<float>(v > big ? big : (v < -big ? -big : v));
        };
        f.lower = clampf(b.lower);
        f.upper = clampf(b.upper);
        f.effort = clampf(b.effort);
        f.vel_limit = clampf(b.vel_limit);
        f.limited = b.limited ? 1 : 0;
        f.parent = b.parent;
        if (b.damping != 0.0) flags |= mw::kHasDamping;
        if (b.limited) flags |= mw::kHasLimits;
        if (b.friction != 0.0) flags |= mw::kHasFriction;
    }
    P.flags = flags;
    mw::group_topology_words(P);
}

// FreeF of a floating single-body model: inertia about the body origin, its
// 6x6 spatial inverse (fp64 Gauss-Jordan, stored float32), shapes, gravity
void build_free(mw_sim* s) {
    mw::FreeF& F = s->h_free;
    std::memset(&F, 0, sizeof(F));
    const auto& M = s->model;
    const double m = M.base_mass, *c = M.base_com.data(), *ic = M.base_Ic.data();
    F.mass = static_cast<float>(m);
    for (int k = 0; k < 3; ++k) F.com[k] = static_cast<float>(c[k]);
    const double c2 = c[0] * c[0] + c[1] * c[1] + c[2] * c[2];
    const double Io[6] = {ic[0] + m * (c2 - c[0] * c[0]), ic[1] + m * (c2 - c[1] * c[1]), ic[2] + m * (c2 - c[2] * c[2]),
                          ic[3] - m * c[0] * c[1], ic[4] - m * c[0] * c[2], ic[5] - m * c[1] * c[2]};
    for (int k = 0; k < 6; ++k) F.Io[k] = static_cast<float>(Io[k]);
    // spatial inertia [[Io, m[c]x], [m[c]x^T, m 1]] and its inverse
    double A[6][12] = {};
    const double Sy[9] = {Io[0], Io[3], Io[4], Io[3], Io[1], Io[5], Io[4], Io[5], Io[2]};
    const double C[9] = {0, -c[2], c[1], c[2], 0, -c[0], -c[1], c[0], 0};
    for (int r = 0; r < 3; ++r)
        for (int q = 0; q < 3; ++q) {
            A[r][q] = Sy[r * 3 + q];
            A[r][q + 3] = m * C[r * 3 + q];
            A[r + 3][q] = m * C[q * 3 + r];
            A[r + 3][q + 3] = (r == q) ? m : 0.0;
        }
    for (int r = 0; r < 6; ++r) A[r][6 + r] = 1.0;
    for (int col = 0; col < 6; ++col) {
        int piv = col;
        for (int r = col + 1; r < 6; ++r)
            if (std::fabs(A[r][col]) > std::fabs(A[piv][col])) piv = r;
        for (int k = 0; k < 12; ++k) std::swap(A[col][k], A[piv][k]);
        const double d = A[col][col];
        for (int k = 0; k < 12; ++k) A[col][k] /= d;
        for (int r = 0; r < 6; ++r)
            if (r != col) {
                const double f = A[r][col];
                for (int k = 0; k < 12; ++k) A[r][k] -= f * A[col][k];
            }
    }
    for (int r = 0; r < 6; ++r)
        for (int q = 0; q < 6; ++q) F.Minv[r * 6 + q] = static_cast<float>(A[r][6 + q]);
    for (int k = 0; k < 3; ++k) F.g[k] = static_cast<float>(s->gravity[k]);
    F.mu = static_cast<float>(s->ground_mu);
    F.ground = s->ground ? 1 : 0;
    F.n_shapes = static_cast<int32_t>(M.base_shapes.size());
    for (size_t i = 0; i < M.base_shapes.size(); ++i) {
        const mw::Shape& sh = M.base_shapes[i];
        F.shape_type[i] = sh.type;
        for (int k = 0; k < 3; ++k) {
            F.shape_size[i][k] = static_cast<float>(sh.size[k]);
            F.shape_p[i][k] = static_cast<float>(sh.p[k]);
        }
        for (int k = 0; k < 9; ++k) F.shape_R[i][k] = static_cast<float>(sh.R[k]);
        F.mesh_npts[i] = static_cast<int32_t>(sh.points.size());
        for (size_t c = 0; c < sh.points.size() && c < 8; ++c)
            for (int k = 0; k < 3; ++k) F.mesh_pt[i][c][k] = static_cast<float>(sh.points[c][k]);
    }
}

// FloatF of an articulated floating model: base inertia about its origin,
// shapes in the oracle's order (base first, then by body), their contact
// slots and the bodies on each shape's path to the base.
void build_float(mw_sim* s) {
    mw::FloatF& F = s->h_float;
    std::memset(&F, 0, sizeof(F));
    const auto& M = s->model;
    const double m = M.base_mass, *c = M.base_com.data(), *ic = M.base_Ic.data();
    F.mass = static_cast<float>(m);
    for (int k = 0; k < 3; ++k) F.com[k] = static_cast<float>(c[k]);
    const double c2 = c[0] * c[0] + c[1] * c[1] + c[2] * c[2];
    const double Io[6] = {ic[0] + m * (c2 - c[0] * c[0]), ic[1] + m * (c2 - c[1] * c[1]), ic[2] + m * (c2 - c[2] * c[2]),
                          ic[3] - m * c[0] * c[1], ic[4] - m * c[0] * c[2], ic[5] - m * c[1] * c[2]};
    for (int k = 0; k < 6; ++k) F.Io[k] = static_cast<float>(Io[k]);
    for (int k = 0; k < 3; ++k) F.g[k] = static_cast<float>(s->gravity[k]);
    F.mu = static_cast<float>(s->ground_mu);
    F.ground = s->ground ? 1 : 0;
    std::vector<std::pair<int, const mw::Shape*>> shapes;
    if (!s->fixed_tree)  // a welded base never touches the ground
        for (const auto& sh : M.base_shapes) shapes.push_back({-1, &sh});
    for (int b = 0; b < M.dofs(); ++b)
        for (const auto& sh : M.bodies[b].shapes) shapes.push_back({b, &sh});
    int slot = 0;
    s->slot_body.clear();
    for (size_t i = 0; i < shapes.size() && i < static_cast<size_t>(mw::kMaxFloatShapes); ++i) {
        const int b = shapes[i].first;
        const mw::Shape& sh = *shapes[i].second;
        F.shape_body[i] = b;
        F.shape_type[i] = sh.type;
        F.shape_slot0[i] = slot;
        uint64_t path = 0;
        for (int k = b; k >= 0; k = M.bodies[k].parent) path |= uint64_t{1} << k;
        F.shape_path[i] = path;
        for (int k = 0; k < 3; ++k) {
            F.shape_size[i][k] = static_cast<float>(sh.size[k]);
            F.shape_p[i][k] = static_cast<float>(sh.p[k]);
        }
        for (int k = 0; k < 9; ++k) F.shape_R[i][k] = static_cast<float>(sh.R[k]);
        const int ns = (sh.type == mw::Shape::Sphere) ? 1 : 8;
        for (int k = 0; k < ns; ++k) s->slot_body.push_back(b);
        slot += ns;
    }
    F.n_shapes = static_cast<int32_t>(std::min(shapes.size(), static_cast<size_t>(mw::kMaxFloatShapes)));
    F.n_slots = slot;
    const int n = std::min(M.dofs(), mw::kMaxBodies);
    std::vector<int> children(n + 1, 0);  // [n] = the base
    F.levels = 0;
    for (int i = n - 1; i >= 0; --i) {
        const int pa = M.bodies[i].parent;
        F.body_srank[i] = static_cast<int8_t>(children[pa >= 0 ? pa : n]++);
    }
    for (int i = 0; i < n; ++i) {
        const int pa = M.bodies[i].parent;
        F.body_depth[i] = static_cast<int8_t>(pa >= 0 ? F.body_depth[pa] + 1 : 0);
        F.levels = std::max<int32_t>(F.levels, F.body_depth[i] + 1);
        F.body_path[i] = (uint64_t{1} << i) | (pa >= 0 ? F.body_path[pa] : uint64_t{0});
    }
    F.fanout = *std::max_element(children.begin(), children.end());
    F.dual = 0;
    for (int i = 0; i < n; ++i)
        if (M.bodies[i].damping != 0.0) F.dual = 1;
    F.fixed = s->fixed_tree ? 1 : 0;
}

int upload_params(mw_sim* s) {
    if (s->float_tree) {
        build_params(s);
        build_float(s);
        MW_HIP(hipMemcpyAsync(s->d_params, &s->h_params, sizeof(mw::ChainF), hipMemcpyHostToDevice, s->stream));
        MW_HIP(hipMemcpyAsync(s->d_float, &s->h_float, sizeof(mw::FloatF), hipMemcpyHostToDevice, s->stream));
        return MW_OK;
    }
    if (s->floating) {
        build_free(s);
        MW_HIP(hipMemcpyAsync(s->d_free, &s->h_free, sizeof(mw::FreeF), hipMemcpyHostToDevice, s->stream));
        return MW_OK;
    }
    build_params(s);
    MW_HIP(hipMemcpyAsync(s->d_params, &s->h_params, sizeof(mw::ChainF), hipMemcpyHostToDevice, s->stream));
    return MW_OK;
}

bool needs_cons(const mw_sim* s) {
    return (s->h_params.flags & (mw::kHasLimits | mw::kHasFriction)) != 0 || s->servo_used;
}
bool needs_dual(const mw_sim* s) { return (s->h_params.flags & mw::kHasDamping) != 0; }

// id of the shipped model whose float32 parameter block is bit-identical to the
// loaded one (constant-folded kernels, baked_models.hpp), else 0.
// MWSTEP_DISABLE_BAKED=1 forces the generic kernels.
int baked_id(const mw_sim* s) {
    const char* off = std::getenv("MWSTEP_DISABLE_BAKED");
    if (off && *off && *off != '0') return 0;
    const size_t words = 8 + 40 * static_cast<size_t>(s->n);
    if (words * 4 == sizeof(mw::baked::kCartpoleHost) &&
        std::memcmp(&s->h_params, &mw::baked::kCartpoleHost, words * 4) == 0)
        return mw::baked::kCartpoleId;
    if (words * 4 == sizeof(mw::baked::kPendulumHost) &&
        std::memcmp(&s->h_params, &mw::baked::kPendulumHost, words * 4) == 0)
        return mw::baked::kPendulumId;
    if (words * 4 == sizeof(mw::baked::kPandaHost) &&
        std::memcmp(&s->h_params, &mw::baked::kPandaHost, words * 4) == 0)
        return mw::baked::kPandaId;
    return 0;
}

int pull_state(mw_sim* s) {
    if (!s->host_stale) return MW_OK;
    if (s->fbase()) {
        MW_HIP(hipMemcpyAsync(s->h_base, s->fdev.base, 13 * static_cast<size_t>(s->W) * sizeof(float),
                              hipMemcpyDeviceToHost, s->stream));
        if (!s->float_tree) {
            MW_HIP(hipStreamSynchronize(s->stream));
            s->host_stale = false;
            return MW_OK;
        }
    }
    MW_HIP(hipMemcpyAsync(s->h_block, s->d_block, s->state_bytes, hipMemcpyDeviceToHost, s->stream));
    MW_HIP(hipStreamSynchronize(s->stream));
    s->host_stale = false;
    return MW_OK;
}

// position targets written on the device (mw_device_ptr) -> host mirror
int pull_ptgt(mw_sim* s) {
    if (!s->ptgt_stale) return MW_OK;
    MW_HIP(hipMemcpyAsync(s->h_ptgt, s->d_aux, s->nw * sizeof(float), hipMemcpyDeviceToHost, s->stream));
    MW_HIP(hipStreamSynchronize(s->stream));
    for (size_t k = 0; k < s->nw; ++k) s->ptgt[k] = s->h_ptgt[k];
    s->ptgt_stale = s->ptgt_view;
    return MW_OK;
}

float to_f32(double v) {
    const double big = static_cast<double>(std::numeric_limits<float>::max());
    return static_cast<float>(v > big ? big : (v < -big ? -big : v));
}

mw::PidSet pid_set(const mw_sim* s) {
    mw::PidSet P{};
    for (int d = 0; d < s->n && d < mw::kMaxKernelDofs; ++d) {
        const auto& g = s->pid[d];
        P.g[d] = {to_f32(g[0]), to_f32(g[1]), to_f32(g[2]), to_f32(g[7]), to_f32(g[6]),
                  to_f32(g[4]), to_f32(g[3]), to_f32(g[5])};
    }
    return P;
}

// ignition::math::PID(1, 0.1, 0.01, -1, 0, -1, 0, 0) (Joint.cpp:63) as
// {p, i, d, cmdMin, cmdMax, cmdOffset, iMin, iMax}
constexpr std::array<double, 8> kDefaultPid = {1.0, 0.1, 0.01, 0.0, -1.0, 0.0, 0.0, -1.0};

// resolve a (dofs, ndofs) selection; dofs == NULL -> all dofs
int selection(const mw_sim* s, int32_t w0, int32_t nw, const int32_t* dofs, int32_t ndofs,
              std::vector<int32_t>& out) {
    if (w0 < 0 || nw < 0 || w0 + nw > s->W)
        return fail(MW_EINVAL, "world range [" + std::to_string(w0) + ", " + std::to_string(w0 + nw) +
                                   ") out of [0, " + std::to_string(s->W) + ")");
    out.clear();
    if (!dofs) {
        for (int d = 0; d < s->n; ++d) out.push_back(d);
        return MW_OK;
    }
    for (int k = 0; k < ndofs; ++k) {
        if (dofs[k] < 0 || dofs[k] >= s->n)
            return fail(MW_EINVAL, "dof index " + std::to_string(dofs[k]) + " out of range");
        out.push_back(dofs[k]);
    }
    return MW_OK;
}

template <typename Get>
int getter(mw_sim* s, int32_t w0, int32_t nw, const int32_t* dofs, int32_t ndofs, double* out, Get get) {
    int rc = check_sim(s);
    if (rc) return rc;
    std::vector<int32_t> sel;
    if ((rc = selection(s, w0, nw, dofs, ndofs, sel))) return rc;
    if ((rc = pull_state(s))) return rc;
    const size_t m = sel.size();
    for (int32_t w = 0; w < nw; ++w)
        for (size_t k = 0; k < m; ++k) out[w * m + k] = get(sel[k], w0 + w);
    return MW_OK;
}

template <typename Set>
int setter(mw_sim* s, int32_t w0, int32_t nw, const int32_t* dofs, int32_t ndofs, const double* v, Set set) {
    int rc = check_sim(s);
    if (rc) return rc;
    std::vector<int32_t> sel;
    if ((rc = selection(s, w0, nw, dofs, ndofs, sel))) return rc;
    const size_t m = sel.size();
    // validate everything first: a failing call changes nothing
    for (int32_t w = 0; w < nw; ++w)
        for (size_t k = 0; k < m; ++k)
            if ((rc = set(sel[k], w0 + w, v[w * m + k], /*dry_run=*/true))) return rc;
    for (int32_t w = 0; w < nw; ++w)
        for (size_t k = 0; k < m; ++k) set(sel[k], w0 + w, v[w * m + k], false);
    s->cmd_dirty = true;
    return MW_OK;
}

// A reset of a world's state re-arms its divergence flag (the flags mark
// worlds whose state is not finite; a reset replaces that state): worlds that
// diverged, were reset and diverge again are reported again (mwstep.h).
int rearm_diverged(mw_sim* s, int32_t w0, int32_t nw) {
    if (s->dev.div && nw > 0) MW_HIP(hipMemsetAsync(s->dev.div + w0, 0, nw, s->stream));
    return MW_OK;
}

int copy_str(const std::string& v, char* buf, int32_t len) {
    if (!buf || len <= 0) return fail(MW_EINVAL, "invalid output buffer");
    if (static_cast<int32_t>(v.size()) + 1 > len) return fail(MW_EINVAL, "output buffer too small");
    std::memcpy(buf, v.c_str(), v.size() + 1);
    return MW_OK;
}

}  // namespace

namespace {

// the device rows of the per-world record (mw_get_state): {first row, rows},
// every row W floats
std::vector<std::pair<float*, int>> state_rows(const mw_sim* s) {
    std::vector<std::pair<float*, int>> v;
    if (s->nw) {
        v.push_back({s->dev.q, 3 * s->n});       // q, qd, qdd
        v.push_back({s->dev.pid_e, 4 * s->n});   // pid_e, pid_i, pid_u, qlo
    }
    if (s->fbase()) v.push_back({s->fdev.base, 13});
    if (s->d_warm) v.push_back({s->d_warm, mw::kWaveWarmWordsHost});
    return v;
}

int state_words(const mw_sim* s) {
    int k = 0;
    for (const auto& r : state_rows(s)) k += r.second;
    return k;
}

}  // namespace

extern "C" {

const char* mw_last_error(void) { return g_last_error.c_str(); }
const char* mw_version(void) { return "mwstep 0.1.0 (gfx950)"; }

int mw_create(const mw_config* cfg, mw_sim** out) {
    if (!cfg || !out) return fail(MW_EINVAL, "null argument");
    *out = nullptr;
    if (!(cfg->step_size > 0.0)) return fail(MW_EINVAL, "the step size must be positive");
    if (!(cfg->rtf > 0.0)) return fail(MW_EINVAL, "the real-time factor must be positive");
    if (cfg->steps_per_run <= 0) return fail(MW_EINVAL, "steps_per_run must be positive");
    if (cfg->n_worlds <= 0) return fail(MW_EINVAL, "n_worlds must be positive");
    auto s = std::make_unique<mw_sim>();
    s->cfg = *cfg;
    if (s->cfg.pgs_iters <= 0) s->cfg.pgs_iters = 20;
    s->W = cfg->n_worlds;
    s->dt_ns = static_cast<int64_t>(std::llround(cfg->step_size * 1e9));
    *out = s.release();
    return MW_OK;
}

void mw_destroy(mw_sim* s) {
    if (!s) return;
    if (s->initialized) {
        (void)hipSetDevice(s->cfg.device);
        if (s->stream) (void)hipStreamSynchronize(s->stream);
        (void)hipFree(s->d_block);
        (void)hipFree(s->d_params);
        (void)hipFree(s->d_aux);
        (void)hipHostFree(s->h_block);
        (void)hipHostFree(s->h_ptgt);
        (void)hipHostFree(s->h_stage);
        if (s->stage_ev) (void)hipEventDestroy(s->stage_ev);
        (void)hipFree(s->d_fblock);
        (void)hipFree(s->d_free);
        (void)hipFree(s->d_float);
        (void)hipFree(s->d_ws);
        (void)hipFree(s->d_pid);
        (void)hipHostFree(s->h_pid);
        (void)hipFree(s->d_overflow);
        (void)hipFree(s->d_warm);
        (void)hipFree(s->d_ext);
        (void)hipHostFree(s->h_ext);
        (void)hipHostFree(s->h_overflow);
        (void)hipHostFree(s->h_base);
        (void)hipHostFree(s->h_cdata);
        (void)hipHostFree(s->h_cmask);
        (void)hipFree(s->d_health);
        (void)hipHostFree(s->h_ndiv);
        if (s->own_stream) (void)hipStreamDestroy(s->stream);
    }
    delete s;
}

int mw_load_model(mw_sim* s, const char* urdf, const double pose[7], const char* name) {
    if (!s || !urdf) return fail(MW_EINVAL, "null argument");
    if (s->initialized) return fail(MW_ESTATE, "models must be loaded before mw_initialize");
    const double ident[7] = {0, 0, 0, 1, 0, 0, 0};
    try {
        s->model = mw::compile_urdf(urdf, pose ? pose : ident);
    } catch (const std::exception& e) {
        return fail(MW_EPARSE, e.what());
    }
    // DART solves every contact LCP exactly (wave_lcp.hpp, the default
    // MW_LCP_EXACT): every floating model then steps on the world-per-wavefront
    // kernel, whatever its size or world count, so the contact answer never
    // depends on the kernel; a joint-less body is its tree with no joints.  The
    // PGS-only lane kernels (free_body.hpp, float_tree.hpp) serve MW_LCP_PGS
    // chosen before mw_load_model (MWSTEP_FREE_KERNEL=1 forces the free-body one)
    const bool exact = s->lcp_mode == MW_LCP_EXACT;
    const char* free_kernel = std::getenv("MWSTEP_FREE_KERNEL");
    const bool free_wave = s->model.floating && s->model.dofs() == 0 && exact &&
                           !(free_kernel && *free_kernel == '1');
    // Mesh collisions (scene.cpp models them as ground slots at their support
    // points).  Articulated floating models (and joint-less bodies on the wave
    // kernel): every support point becomes a zero-radius sphere at that point
    // (the same ground contact: normal +z, depth -z, in slot order).  A
    // joint-less floating body on the free-body kernel (2 shape entries of 8
    // slots): the mesh splits into entries of <= 8 points.  Fixed bases never
    // touch the ground here: their meshes are dropped (counted).
    {
        int meshes = 0;
        const bool expand = s->model.floating && (s->model.dofs() > 0 || free_wave);
        const bool free_body = s->model.floating && s->model.dofs() == 0 && !free_wave;
        auto convert = [&](std::vector<mw::Shape>& v) {
            std::vector<mw::Shape> out;
            for (const mw::Shape& sh : v) {
                if (sh.type != mw::Shape::Mesh) {
                    out.push_back(sh);
                    continue;
                }
                ++meshes;
                if (free_body) {  // the free-body kernel: <= 8 points (one slot block) per shape entry
                    for (size_t c0 = 0; c0 < sh.points.size(); c0 += 8) {
                        mw::Shape part = sh;
                        part.points.assign(sh.points.begin() + c0,
                                           sh.points.begin() + std::min(sh.points.size(), c0 + 8));
                        out.push_back(part);
                    }
                    continue;
                }
                if (!expand) continue;
                for (const auto& pt : sh.points) {
                    mw::Shape sp;
                    sp.type = mw::Shape::Sphere;
                    sp.R = {1, 0, 0, 0, 1, 0, 0, 0, 1};
                    for (int r = 0; r < 3; ++r)
                        sp.p[r] = sh.p[r] + sh.R[3 * r] * pt[0] + sh.R[3 * r + 1] * pt[1] + sh.R[3 * r + 2] * pt[2];
                    out.push_back(sp);
                }
            }
            v.swap(out);
        };
        convert(s->model.base_shapes);
        for (auto& b : s->model.bodies) convert(b.shapes);
        if (!s->model.floating) s->model.unsupported_shapes += meshes;
    }
    if (s->model.dofs() > mw::kMaxBodies)
        return fail(MW_EPARSE, "models with more than " + std::to_string(mw::kMaxBodies) +
                                   " moving joints are not supported by this build");
    if (!s->model.floating && s->model.dofs() == 0)
        return fail(MW_EPARSE, "a welded model without moving joints has no dynamics of its own: insert it into a "
                               "scene (World.insert_model) where it is a collider");
    s->floating = s->model.floating;
    s->fixed_tree = false;
    // ball joints (DART's BallJoint coordinates, chain_dyn.hpp ball_part):
    // the world-per-wavefront kernel only
    bool has_ball = false;
    for (const auto& b : s->model.bodies) has_ball = has_ball || b.ball != 0;
    if (!s->floating) {
        // fixed bases: the compiled chain topologies run on the lane kernels,
        // every other tree on the world-per-wavefront kernel with a welded base
        std::vector<int> parents;
        for (const auto& b : s->model.bodies) parents.push_back(b.parent);
        s->fixed_tree = s->model.dofs() > 9 || mw::kernel_topology(parents.data(), s->model.dofs()) < 0 || has_ball;
    }
    s->float_tree = (s->floating && (s->model.dofs() > 0 || free_wave)) || s->fixed_tree;
    if (s->float_tree) {
        std::vector<int> parents;
        for (const auto& b : s->model.bodies) parents.push_back(b.parent);
        s->topo = mw::kernel_topology(parents.data(), s->model.dofs());
        size_t n_shapes = s->fixed_tree ? 0 : s->model.base_shapes.size();
        bool damped = false;  // joint damping: the wave kernel (its dual recursion) only
        for (const auto& b : s->model.bodies) {
            n_shapes += b.shapes.size();
            damped = damped || b.damping != 0.0;
        }
        if (n_shapes > static_cast<size_t>(mw::kMaxFloatShapes))
            return fail(MW_EPARSE, "an articulated model may have at most " +
                                       std::to_string(mw::kMaxFloatShapes) + " box / sphere collision shapes");
        s->n = s->model.dofs();
        build_float(s);
        if (s->h_float.n_slots > mw::kMaxFloatSlots)
            return fail(MW_EPARSE, "an articulated model may have at most " + std::to_string(mw::kMaxFloatSlots) +
                                       " contact slots (8 per box, 1 per sphere)");
        // small compiled topologies: one world per lane (float_tree.hpp); any
        // other tree: one world per wavefront (wave_tree.hpp)
        const bool compiled = ((s->topo == 0 && s->n <= 3) || s->topo == 2) &&
                              mw::float_workspace_words(s->n, s->h_float.n_slots) >= 0;
        const char* force_wave = std::getenv("MWSTEP_WAVE_TREE");
        // with the PGS-only solver, small compiled topologies at large world
        // counts take the lane kernel; up to kWaveWorldsMax worlds the wave
        // kernel is faster (quadruped, profiles/r01f/quadruped_*_sweep.log:
        // 1024 worlds 62 us/step wave vs 365 lane, 16384 worlds 638 wave vs 394
        // lane).  The exact solve runs on the wave kernel only.
        // MWSTEP_WAVE_TREE=1 / =0 forces the wave / lane kernel.
        constexpr int kWaveWorldsMax = 4096;
        if (force_wave && *force_wave)
            s->wave = !compiled || *force_wave != '0' || damped || has_ball;
        else
            s->wave = !compiled || s->W <= kWaveWorldsMax || damped || exact || has_ball;
        if (s->fixed_tree) s->wave = true;  // the lane kernel has no welded-base mode
        {
            std::vector<int> depth(s->n, 0);
            int max_depth = 0;
            for (int i = 0; i < s->n; ++i) {
                const int pa = s->model.bodies[i].parent;
                depth[i] = (pa >= 0) ? depth[pa] + 1 : 0;
                max_depth = std::max(max_depth, depth[i] + 1);
            }
            s->wave_depth_ok = max_depth <= mw::kWaveMaxDepthHost;
            s->wave_depth = max_depth;
            if (s->wave && !s->wave_depth_ok)
                return fail(MW_EPARSE, "the kinematic tree of this model is deeper than " +
                                           std::to_string(mw::kWaveMaxDepthHost) + " joints");
        }
        s->n_slots = s->h_float.n_slots;
        s->pid.assign(s->model.dofs(), kDefaultPid);
        s->model_name = (name && *name) ? name : s->model.name;
        s->loaded = true;
        build_params(s);
        return MW_OK;
    }
    if (s->floating) {
        if (s->model.base_shapes.size() > static_cast<size_t>(mw::kMaxFreeShapes))
            return fail(MW_EPARSE, "a floating body may have at most " + std::to_string(mw::kMaxFreeShapes) +
                                       " collision shape entries in this build (a mesh takes one per 8 support points)");
        s->model_name = (name && *name) ? name : s->model.name;
        s->loaded = true;
        s->n = 0;
        s->pid.clear();
        build_free(s);
        return MW_OK;
    }
    {
        std::vector<int> parents;
        for (const auto& b : s->model.bodies) parents.push_back(b.parent);
        s->topo = mw::kernel_topology(parents.data(), s->model.dofs());
        if (s->topo < 0)
            return fail(MW_EPARSE, "the kinematic topology of this branched model is not compiled into this "
                                   "build (supported: serial chains of 1..9 dofs and the Panda tree)");
    }
    s->pid.assign(s->model.dofs(), kDefaultPid);
    s->model_name = (name && *name) ? name : s->model.name;
    s->loaded = true;
    s->n = s->model.dofs();
    build_params(s);
    return MW_OK;
}

int mw_baked_model(const mw_sim* s, int32_t* id) {
    if (!s || !id) return fail(MW_EINVAL, "null argument");
    if (!s->loaded) return fail(MW_ESTATE, "no model loaded");
    *id = baked_id(s);
    return MW_OK;
}

int mw_device_params(const mw_sim* s, void* out, int32_t bytes) {
    if (!s || !out) return fail(MW_EINVAL, "null argument");
    if (!s->loaded) return fail(MW_ESTATE, "no model loaded");
    if (bytes < static_cast<int32_t>(sizeof(mw::ChainF))) return fail(MW_EINVAL, "buffer too small");
    mw_sim* m = const_cast<mw_sim*>(s);
    build_params(m);
    std::memcpy(out, &m->h_params, sizeof(mw::ChainF));
    return MW_OK;
}

// PGS sweeps of exact mode end once a sweep moves no constraint velocity by
// more than this (m/s, rad/s): the exact solve takes over from there
constexpr float kExactPgsTol = 1e-6f;

// Device buffers of the world-per-wavefront kernel: PID gains, the overflow
// counters ([0] constraint rows dropped, [1] exact-LCP solves that ran out of
// budget) and the warm-start record of the PGS impulses.  Called at
// initialisation, or when a model switches to the kernel mid-life (joint
// damping set after mw_initialize).
static int alloc_wave_buffers(mw_sim* s) {
    const size_t W = static_cast<size_t>(s->W);
    MW_HIP(hipMalloc(reinterpret_cast<void**>(&s->d_pid), mw::kMaxBodies * sizeof(mw::PidF)));
    MW_HIP(hipHostMalloc(reinterpret_cast<void**>(&s->h_pid), mw::kMaxBodies * sizeof(mw::PidF),
                         hipHostMallocDefault));
    // [0] dropped rows (int32, drained into overflow_seen), [2..3] unconverged
    // exact-LCP world-steps (uint64)
    MW_HIP(hipMalloc(reinterpret_cast<void**>(&s->d_overflow), 4 * sizeof(int)));
    MW_HIP(hipMemsetAsync(s->d_overflow, 0, 4 * sizeof(int), s->stream));
    MW_HIP(hipHostMalloc(reinterpret_cast<void**>(&s->h_overflow), 2 * sizeof(int), hipHostMallocDefault));
    s->h_overflow[0] = s->h_overflow[1] = 0;
    const size_t wb = static_cast<size_t>(mw::kWaveWarmWordsHost) * W * sizeof(float);
    MW_HIP(hipMalloc(reinterpret_cast<void**>(&s->d_warm), wb));
    MW_HIP(hipMemsetAsync(s->d_warm, 0, wb, s->stream));
    return MW_OK;
}

int mw_constraint_overflow(const mw_sim* s, int64_t* rows) {
    int rc = check_sim(s);
    if (rc) return rc;
    if (!rows) return fail(MW_EINVAL, "null argument");
    *rows = 0;
    if (!s->d_overflow) return MW_OK;
    int v = 0;
    MW_HIP(hipMemcpyAsync(&v, s->d_overflow, sizeof(int), hipMemcpyDeviceToHost, s->stream));
    MW_HIP(hipStreamSynchronize(s->stream));
    *rows = v;
    return MW_OK;
}

int mw_lcp_unconverged(const mw_sim* s, int64_t* worlds) {
    int rc = check_sim(s);
    if (rc) return rc;
    if (!worlds) return fail(MW_EINVAL, "null argument");
    *worlds = 0;
    if (!s->d_overflow) return MW_OK;
    uint64_t v = 0;
    MW_HIP(hipMemcpyAsync(&v, s->d_overflow + 2, sizeof(v), hipMemcpyDeviceToHost, s->stream));
    MW_HIP(hipStreamSynchronize(s->stream));
    *worlds = static_cast<int64_t>(v);
    return MW_OK;
}

int mw_float_kernel(const mw_sim* s, int32_t* kind) {
    if (!s || !kind) return fail(MW_EINVAL, "null argument");
    if (!s->loaded) return fail(MW_ESTATE, "no model loaded");
    *kind = !s->float_tree ? 0 : (s->wave ? 2 : 1);
    return MW_OK;
}

int mw_device_float_params(const mw_sim* s, void* out, int32_t bytes) {
    if (!s || !out) return fail(MW_EINVAL, "null argument");
    if (!s->loaded) return fail(MW_ESTATE, "no model loaded");
    if (!s->float_tree) return fail(MW_ESTATE, "not an articulated floating-base model");
    if (bytes < static_cast<int32_t>(sizeof(mw::FloatF))) return fail(MW_EINVAL, "buffer too small");
    mw_sim* m = const_cast<mw_sim*>(s);
    build_float(m);
    std::memcpy(out, &m->h_float, sizeof(mw::FloatF));
    return MW_OK;
}

int mw_initialize(mw_sim* s) {
    if (!s) return fail(MW_EINVAL, "null simulator handle");
    if (s->initialized) return MW_OK;
    if (!s->loaded) return fail(MW_ESTATE, "no model loaded");
    MW_HIP(hipSetDevice(s->cfg.device));
    if (!s->stream_set) {
        MW_HIP(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
        s->own_stream = true;
        s->stream_set = true;
    }
    s->n = s->model.dofs();
    {
        // divergence flags [W] (rounded to 8 bytes) + the uint64 count
        const size_t rw = (static_cast<size_t>(s->W) + 7) & ~size_t{7};
        MW_HIP(hipMalloc(reinterpret_cast<void**>(&s->d_health), rw + 8));
        MW_HIP(hipMemsetAsync(s->d_health, 0, rw + 8, s->stream));
        MW_HIP(hipHostMalloc(reinterpret_cast<void**>(&s->h_ndiv), sizeof(uint64_t), hipHostMallocDefault));
        *s->h_ndiv = 0;
        s->dev.div = s->fdev.div = s->d_health;
        s->dev.ndiv = s->fdev.ndiv = reinterpret_cast<unsigned long long*>(s->d_health + rw);
    }
    if (s->fbase()) {
        const size_t W = static_cast<size_t>(s->W);
        const size_t ns = static_cast<size_t>(s->n_slots);
        const size_t nf = (13 + 7 + 6 + 7 * ns) * W;
        MW_HIP(hipMalloc(&s->d_fblock, nf * sizeof(float) + W * (1 + sizeof(uint32_t)) + 64));
        if (s->float_tree) {
            MW_HIP(hipMalloc(reinterpret_cast<void**>(&s->d_float), sizeof(mw::FloatF)));
            if (s->wave) {
                if (int rc = alloc_wave_buffers(s)) return rc;
            } else {
                const size_t words = static_cast<size_t>(mw::float_workspace_words(s->n, s->n_slots));
                MW_HIP(hipMalloc(reinterpret_cast<void**>(&s->d_ws), words * W * sizeof(float)));
            }
        } else {
            MW_HIP(hipMalloc(reinterpret_cast<void**>(&s->d_free), sizeof(mw::FreeF)));
        }
        float* f = static_cast<float*>(s->d_fblock);
        s->fdev.base = f;
        s->fdev.rpose = f + 13 * W;
        s->fdev.rvel = f + 20 * W;
        s->fdev.cdata = f + 26 * W;
        s->fdev.cmask = reinterpret_cast<uint32_t*>(f + nf);
        s->fdev.rflag = reinterpret_cast<uint8_t*>(s->fdev.cmask + W);
        s->fdev.warm = s->d_warm;
        MW_HIP(hipHostMalloc(reinterpret_cast<void**>(&s->h_base), 13 * W * sizeof(float), hipHostMallocDefault));
        MW_HIP(hipHostMalloc(reinterpret_cast<void**>(&s->h_cdata), 7 * ns * W * sizeof(float),
                             hipHostMallocDefault));
        MW_HIP(hipHostMalloc(reinterpret_cast<void**>(&s->h_cmask), W * sizeof(uint32_t), hipHostMallocDefault));
        std::memset(s->h_cmask, 0, W * sizeof(uint32_t));
        // the insertion pose; at rest
        const auto& R = s->model.base_R;
        double qw, qx, qy, qz;
        {
            const double tr = R[0] + R[4] + R[8];
            if (tr > 0) {
                const double k = 0.5 / std::sqrt(tr + 1.0);
                qw = 0.25 / k; qx = (R[7] - R[5]) * k; qy = (R[2] - R[6]) * k; qz = (R[3] - R[1]) * k;
            } else if (R[0] > R[4] && R[0] > R[8]) {
                const double k = 2.0 * std::sqrt(1.0 + R[0] - R[4] - R[8]);
                qw = (R[7] - R[5]) / k; qx = 0.25 * k; qy = (R[1] + R[3]) / k; qz = (R[2] + R[6]) / k;
            } else if (R[4] > R[8]) {
                const double k = 2.0 * std::sqrt(1.0 + R[4] - R[0] - R[8]);
                qw = (R[2] - R[6]) / k; qx = (R[1] + R[3]) / k; qy = 0.25 * k; qz = (R[5] + R[7]) / k;
            } else {
                const double k = 2.0 * std::sqrt(1.0 + R[8] - R[0] - R[4]);
                qw = (R[3] - R[1]) / k; qx = (R[2] + R[6]) / k; qy = (R[5] + R[7]) / k; qz = 0.25 * k;
            }
        }
        const double init[13] = {s->model.base_p[0], s->model.base_p[1], s->model.base_p[2], qw, qx, qy, qz,
                                 0, 0, 0, 0, 0, 0};
        for (int f2 = 0; f2 < 13; ++f2)
            for (size_t w = 0; w < W; ++w) s->h_base[f2 * W + w] = static_cast<float>(init[f2]);
        MW_HIP(hipMemcpyAsync(s->fdev.base, s->h_base, 13 * W * sizeof(float), hipMemcpyHostToDevice, s->stream));
        MW_HIP(hipMemsetAsync(s->fdev.cmask, 0, W * (1 + sizeof(uint32_t)), s->stream));
        s->h_rpose.assign(7 * W, 0.f);
        s->h_rvel.assign(6 * W, 0.f);
        s->h_rflag.assign(W, 0);
        if (!s->float_tree) {
            s->initialized = true;
            int rc = upload_params(s);
            if (rc) return rc;
            MW_HIP(hipStreamSynchronize(s->stream));
            return MW_OK;
        }
    }
    s->nw = static_cast<size_t>(s->n) * s->W;
    s->state_bytes = 3 * s->nw * sizeof(float);
    s->cmd_off = s->state_bytes;
    s->cmd_bytes = 4 * s->nw * sizeof(float) + 2 * s->nw;
    s->block_bytes = s->state_bytes + s->cmd_bytes;
    // (a joint-less floating body on the wave kernel has no joint arrays:
    // every allocation keeps a minimal size)
    auto sz = [](size_t b) { return std::max<size_t>(b, 64); };
    MW_HIP(hipMalloc(&s->d_block, sz(s->block_bytes)));
    MW_HIP(hipMalloc(&s->d_params, sizeof(mw::ChainF)));
    MW_HIP(hipMalloc(reinterpret_cast<void**>(&s->d_aux), sz(5 * s->nw * sizeof(float))));
    MW_HIP(hipMemsetAsync(s->d_aux, 0, 5 * s->nw * sizeof(float), s->stream));
    MW_HIP(hipHostMalloc(reinterpret_cast<void**>(&s->h_ptgt), sz(s->nw * sizeof(float)), hipHostMallocDefault));
    std::memset(s->h_ptgt, 0, s->nw * sizeof(float));
    MW_HIP(hipHostMalloc(reinterpret_cast<void**>(&s->h_block), sz(s->block_bytes), hipHostMallocDefault));
    std::memset(s->h_block, 0, s->block_bytes);
    MW_HIP(hipHostMalloc(reinterpret_cast<void**>(&s->h_stage), sz(s->cmd_bytes + s->nw * sizeof(float)),
                         hipHostMallocDefault));
    MW_HIP(hipEventCreateWithFlags(&s->stage_ev, hipEventDisableTiming));
    float* base = reinterpret_cast<float*>(s->d_block);
    s->dev.q = base;
    s->dev.qd = base + s->nw;
    s->dev.qdd = base + 2 * s->nw;
    s->dev.cmd = base + 3 * s->nw;
    s->dev.vtgt = base + 4 * s->nw;
    s->dev.rq = base + 5 * s->nw;
    s->dev.rqd = base + 6 * s->nw;
    s->dev.act = reinterpret_cast<uint8_t*>(base + 7 * s->nw);
    s->dev.rflag = s->dev.act + s->nw;
    s->dev.ptgt = s->d_aux;
    s->dev.pid_e = s->d_aux + s->nw;
    s->dev.pid_i = s->d_aux + 2 * s->nw;
    s->dev.pid_u = s->d_aux + 3 * s->nw;
    s->dev.qlo = s->d_aux + 4 * s->nw;
    s->mode.assign(s->nw, MW_MODE_IDLE);
    s->ptgt.assign(s->nw, 0.0);
    s->cmd64.assign(s->nw, 0.0);
    s->initialized = true;
    int rc = upload_params(s);
    if (rc) return rc;
    MW_HIP(hipMemcpyAsync(s->d_block, s->h_block, s->block_bytes, hipMemcpyHostToDevice, s->stream));
    MW_HIP(hipStreamSynchronize(s->stream));
    s->cmd_dirty = false;
    return MW_OK;
}

int mw_initialized(const mw_sim* s) { return (s && s->initialized) ? 1 : 0; }

int mw_set_stream(mw_sim* s, void* stream) {
    if (!s) return fail(MW_EINVAL, "null simulator handle");
    if (s->initialized) MW_HIP(hipStreamSynchronize(s->stream));
    if (s->own_stream && s->stream) (void)hipStreamDestroy(s->stream);
    s->stream = static_cast<hipStream_t>(stream);
    s->own_stream = false;
    s->stream_set = true;
    return MW_OK;
}

// worlds newly flagged diverged by the run just read back (h_ndiv): the run
// has advanced every world, the flagged ones hold non-finite state
static int report_divergence(mw_sim* s) {
    const int64_t n = static_cast<int64_t>(*s->h_ndiv);
    if (n <= s->div_seen) return MW_OK;
    const int64_t d = n - s->div_seen;
    s->div_seen = n;
    return fail(MW_EDIVERGED, std::to_string(d) + " world(s) diverged in this run: their joint or base state is "
                                                  "not finite (mw_diverged lists them)");
}

// pending base resets: one H2D copy of [rpose | rvel] and the flags
static int upload_base_resets(mw_sim* s) {
    const size_t W = static_cast<size_t>(s->W);
    if (s->free_dirty) {
        // pending base resets: one H2D copy of [rpose | rvel] and the flags
        MW_HIP(hipMemcpyAsync(s->fdev.rpose, s->h_rpose.data(), 7 * W * sizeof(float), hipMemcpyHostToDevice,
                              s->stream));
        MW_HIP(hipMemcpyAsync(s->fdev.rvel, s->h_rvel.data(), 6 * W * sizeof(float), hipMemcpyHostToDevice,
                              s->stream));
        MW_HIP(hipMemcpyAsync(s->fdev.rflag, s->h_rflag.data(), W, hipMemcpyHostToDevice, s->stream));
        MW_HIP(hipStreamSynchronize(s->stream));  // the host vectors are reused below
        std::fill(s->h_rflag.begin(), s->h_rflag.end(), 0);
        s->free_dirty = false;
    }
    return MW_OK;
}

// contacts + base of the last run -> host mirrors (queued on the stream)
static int read_base(mw_sim* s, int paused) {
    const size_t W = static_cast<size_t>(s->W);
    MW_HIP(hipMemcpyAsync(s->h_base, s->fdev.base, 13 * W * sizeof(float), hipMemcpyDeviceToHost, s->stream));
    if (s->contacts && !paused) {
        MW_HIP(hipMemcpyAsync(s->h_cmask, s->fdev.cmask, W * sizeof(uint32_t), hipMemcpyDeviceToHost, s->stream));
        MW_HIP(hipMemcpyAsync(s->h_cdata, s->fdev.cdata, 7 * static_cast<size_t>(s->n_slots) * W * sizeof(float),
                              hipMemcpyDeviceToHost, s->stream));
    }
    return MW_OK;
}

static int run_free(mw_sim* s, int paused, bool readback = true) {
    int rc = upload_base_resets(s);
    if (rc) return rc;
    mw::RunArgs a{};
    a.dt = static_cast<float>(s->cfg.step_size);
    a.inv_dt = static_cast<float>(1.0 / s->cfg.step_size);
    a.paused = paused ? 1 : 0;
    a.pgs_iters = s->cfg.pgs_iters;
    a.first = 1;
    a.substeps = paused ? 0 : s->cfg.steps_per_run;
    int mesh = 0;
    for (int k = 0; k < s->h_free.n_shapes; ++k) mesh |= s->h_free.shape_type[k] == mw::Shape::Mesh;
    MW_HIP(mw::launch_free_run(s->d_free, s->fdev, s->W, a, s->contacts ? 1 : 0, mesh, s->stream));
    if (!paused) {
        s->iterations += s->cfg.steps_per_run;
        s->stepped = true;
    }
    if (!readback) {
        s->host_stale = true;
        s->contacts_stale = s->contacts;
        return MW_OK;
    }
    if ((rc = read_base(s, paused))) return rc;
    MW_HIP(hipMemcpyAsync(s->h_ndiv, s->dev.ndiv, sizeof(uint64_t), hipMemcpyDeviceToHost, s->stream));
    MW_HIP(hipStreamSynchronize(s->stream));
    s->contacts_stale = false;
    return report_divergence(s);
}

// The world wrenches of the substeps (it0, it0 + chunk]: the launch ends
// before the first expiry inside it (chunk shrinks), the records active
// through it are summed per node into d_ext (Link.cpp:484-560 semantics, as
// mw_scene_apply_world_wrench).
static int stage_wrenches(mw_sim* s, int64_t it0, int& chunk) {
    const int nn = s->n + 1;
    const size_t W = static_cast<size_t>(s->W), st = static_cast<size_t>(nn) * W;
    for (size_t k = 0; k < s->h_wl.size(); ++k) {
        const int64_t last = s->h_wl[k];
        if (last > it0 && last < it0 + chunk) chunk = static_cast<int>(last - it0);
    }
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    MW_HIP(hipStreamIsCapturing(s->stream, &cap));
    if (cap != hipStreamCaptureStatusNone)
        return fail(MW_ESTATE, "world wrenches cannot be captured into a graph: run them outside the capture");
    MW_HIP(hipStreamSynchronize(s->stream));  // the staging buffer of the previous launch
    std::fill(s->h_ext, s->h_ext + 6 * st, 0.f);
    for (int sl = 0; sl < mw::kSimWrenchSlots; ++sl)
        for (size_t nw = 0; nw < st; ++nw) {
            if (s->h_wl[sl * st + nw] < it0 + chunk) continue;
            for (int e = 0; e < 6; ++e) s->h_ext[e * st + nw] += s->h_wr[(static_cast<size_t>(sl) * 6 + e) * st + nw];
        }
    MW_HIP(hipMemcpyAsync(s->d_ext, s->h_ext, 6 * st * sizeof(float), hipMemcpyHostToDevice, s->stream));
    return MW_OK;
}

static int run_impl(mw_sim* s, int paused, bool readback) {
    int rc = check_sim(s);
    if (rc) return rc;
    // a device-resident run never needs the host mirror (and must not
    // synchronise: it may be captured into a graph)
    if (readback && (rc = pull_state(s))) return rc;
    if (s->floating && !s->float_tree) return run_free(s, paused, readback);
    if (s->float_tree && (rc = upload_base_resets(s))) return rc;
    if (s->cmd_dirty || s->ptgt_dirty) {
        // pending commands / resets / targets go through the staging buffer:
        // the host mirror is cleared below while the copy may still be queued
        // (a device-resident run does not synchronise).  A graph would replay
        // a host-memory copy with whatever the buffer holds at replay time, so
        // pending commands cannot be captured.
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        MW_HIP(hipStreamIsCapturing(s->stream, &cap));
        if (cap != hipStreamCaptureStatusNone)
            return fail(MW_ESTATE, "pending joint commands, resets or targets cannot be captured into a graph: "
                                   "apply them with a run before capturing");
        if (s->stage_pending) {
            MW_HIP(hipEventSynchronize(s->stage_ev));  // the previous copy out of the stage is done
            s->stage_pending = false;
        }
        if (s->cmd_dirty) {
            std::memcpy(s->h_stage, s->h_block + s->cmd_off, s->cmd_bytes);
            MW_HIP(hipMemcpyAsync(static_cast<uint8_t*>(s->d_block) + s->cmd_off, s->h_stage, s->cmd_bytes,
                                  hipMemcpyHostToDevice, s->stream));
            s->cmd_dirty = false;
        }
        if (s->ptgt_dirty) {
            std::memcpy(s->h_stage + s->cmd_bytes, s->h_ptgt, s->nw * sizeof(float));
            MW_HIP(hipMemcpyAsync(s->d_aux, s->h_stage + s->cmd_bytes, s->nw * sizeof(float),
                                  hipMemcpyHostToDevice, s->stream));
            s->ptgt_dirty = false;
        }
        MW_HIP(hipEventRecord(s->stage_ev, s->stream));
        s->stage_pending = true;
    }
    const mw::PidSet pid = pid_set(s);
    if (s->wave && s->pid_dirty) {
        // the wave kernel reads every dof's gains from device memory; the pinned
        // staging buffer is only rewritten after the stream has drained it (gains
        // change between runs, never inside a captured device-resident run)
        MW_HIP(hipStreamSynchronize(s->stream));
        s->pid_dirty = false;
        for (int d = 0; d < s->n; ++d) {
            const auto& g = s->pid[d];
            s->h_pid[d] = {to_f32(g[0]), to_f32(g[1]), to_f32(g[2]), to_f32(g[7]), to_f32(g[6]),
                           to_f32(g[4]), to_f32(g[3]), to_f32(g[5])};
        }
        MW_HIP(hipMemcpyAsync(s->d_pid, s->h_pid, s->n * sizeof(mw::PidF), hipMemcpyHostToDevice, s->stream));
    }
    mw::RunArgs a{};
    a.dt = static_cast<float>(s->cfg.step_size);
    a.inv_dt = static_cast<float>(1.0 / s->cfg.step_size);
    a.paused = paused ? 1 : 0;
    a.pgs_iters = s->cfg.pgs_iters;
    a.pgs_tol = static_cast<float>(s->pgs_tol);
    a.lcp_solves = s->wave ? s->lcp_solves : 0;
    // exact mode always starts from the previous step's impulses (the solve's
    // result does not depend on its start) and ends the sweeps once they stop
    // moving the constraint velocities: a steady contact set is then a
    // few-sweep, zero-solve step
    a.warm = (s->wave && (s->pgs_warm || a.lcp_solves > 0) && s->d_warm) ? 1 : 0;
    if (a.lcp_solves > 0) a.pgs_tol = std::max(a.pgs_tol, kExactPgsTol);
    a.first = 1;
    const int spr = s->cfg.steps_per_run;
    int done = 0;
    do {
        int chunk = paused ? 0 : std::min(64, spr - done);
        a.wrenches = 0;
        if (chunk > 0 && s->d_ext && s->wr_until > s->iterations + done) {
            if (int rc2 = stage_wrenches(s, s->iterations + done, chunk)) return rc2;
            a.wrenches = 1;
        }
        a.substeps = chunk;
        a.pid_gate = 0;
        // JointController::PreUpdate period gating on the simulated time
        // (JointController.cpp:130-169): integer nanoseconds like the
        // reference's steady_clock durations; the first iteration always computes
        for (int k = 0; k < chunk && s->controller; ++k) {
            const int64_t sim_ns = (s->iterations + done + k + 1) * s->dt_ns;
            const int64_t elapsed = (s->prev_ns == 0) ? s->period_ns : sim_ns - s->prev_ns;
            if (elapsed >= s->period_ns) {
                s->prev_ns = sim_ns;
                a.pid_gate |= (uint64_t{1} << k);
            }
        }
        if (s->wave)
            MW_HIP(mw::launch_wave_run(s->d_params, s->n, s->wave_depth, needs_cons(s), s->d_float, s->dev, s->fdev, s->d_pid, s->W,
                                       a, s->contacts ? 1 : 0, s->d_overflow, s->stream));
        else if (s->float_tree)
            MW_HIP(mw::launch_float_run(s->d_params, s->n, s->topo, needs_cons(s), s->d_float, s->dev, s->fdev, pid,
                                        s->d_ws, s->W, a, s->contacts ? 1 : 0, s->stream));
        else
            MW_HIP(mw::launch_scenario_run(s->d_params, s->n, s->topo, needs_cons(s), needs_dual(s), baked_id(s),
                                           s->dev, pid, s->W, a, s->stream));
        a.first = 0;
        done += chunk;
    } while (!paused && done < spr);
    if (readback) {
        MW_HIP(hipMemcpyAsync(s->h_block, s->d_block, s->state_bytes, hipMemcpyDeviceToHost, s->stream));
        if (s->float_tree && (rc = read_base(s, paused))) return rc;
        if (s->h_overflow)
            MW_HIP(hipMemcpyAsync(s->h_overflow, s->d_overflow, 2 * sizeof(int), hipMemcpyDeviceToHost, s->stream));
        MW_HIP(hipMemcpyAsync(s->h_ndiv, s->dev.ndiv, sizeof(uint64_t), hipMemcpyDeviceToHost, s->stream));
        MW_HIP(hipStreamSynchronize(s->stream));
        s->contacts_stale = false;
    } else {
        s->host_stale = true;
        s->contacts_stale = s->float_tree && s->contacts;
    }
    // mirror the kernel's component semantics on the host copy
    std::memset(s->hcmd(), 0, s->nw * sizeof(float));
    std::memset(s->hrflag(), 0, s->nw);
    std::fill(s->cmd64.begin(), s->cmd64.end(), 0.0);
    if (!paused) {
        s->iterations += s->cfg.steps_per_run;
        s->stepped = true;
    }
    if (readback && s->h_overflow && *s->h_overflow > s->overflow_seen) {
        // DART keeps every contact: a run that dropped constraint rows fails
        // loudly (the state has advanced without them)
        const int64_t d = *s->h_overflow - s->overflow_seen;
        s->overflow_seen = *s->h_overflow;
        return fail(MW_ECAPACITY, "this run dropped " + std::to_string(d) +
                                      " constraint rows: a world exceeded the per-step capacity of the "
                                      "world-per-wavefront kernel (64 rows)");
    }
    return readback ? report_divergence(s) : MW_OK;
}

int mw_run(mw_sim* s, int paused) { return run_impl(s, paused, true); }

int mw_run_device(mw_sim* s, int32_t runs) {
    if (runs < 0) return fail(MW_EINVAL, "runs must be >= 0");
    for (int32_t k = 0; k < runs; ++k) {
        int rc = run_impl(s, 0, false);
        if (rc) return rc;
    }
    return MW_OK;
}

int mw_time(const mw_sim* s, double* t) {
    if (!s || !t) return fail(MW_EINVAL, "null argument");
    *t = static_cast<double>(s->iterations * s->dt_ns) / 1e9;
    return MW_OK;
}

int mw_set_gravity(mw_sim* s, const double g[3]) {
    if (!s || !g) return fail(MW_EINVAL, "null argument");
    if (s->stepped) return fail(MW_ESTATE, "the gravity can be changed only before the first run");
    std::memcpy(s->gravity, g, sizeof(s->gravity));
    if (s->initialized) return upload_params(s);
    if (s->loaded) build_params(s);
    return MW_OK;
}

int mw_gravity(const mw_sim* s, double g[3]) {
    if (!s || !g) return fail(MW_EINVAL, "null argument");
    std::memcpy(g, s->gravity, sizeof(s->gravity));
    return MW_OK;
}

int mw_n_worlds(const mw_sim* s, int32_t* n) {
    if (!s || !n) return fail(MW_EINVAL, "null argument");
    *n = s->W;
    return MW_OK;
}

int mw_dofs(const mw_sim* s, int32_t* n) {
    if (!s || !n) return fail(MW_EINVAL, "null argument");
    if (!s->loaded) return fail(MW_ESTATE, "no model loaded");
    *n = s->model.dofs();
    return MW_OK;
}

int mw_joint_name(const mw_sim* s, int32_t dof, char* buf, int32_t len) {
    if (!s || !s->loaded) return fail(MW_ESTATE, "no model loaded");
    if (dof < 0 || dof >= s->model.dofs()) return fail(MW_EINVAL, "dof out of range");
    return copy_str(s->model.bodies[dof].joint_name, buf, len);
}

int mw_link_name(const mw_sim* s, int32_t dof, char* buf, int32_t len) {
    if (!s || !s->loaded) return fail(MW_ESTATE, "no model loaded");
    if (dof < 0 || dof >= s->model.dofs()) return fail(MW_EINVAL, "dof out of range");
    return copy_str(s->model.bodies[dof].link_name, buf, len);
}

int mw_joint_index(const mw_sim* s, const char* name, int32_t* dof) {
    if (!s || !name || !dof) return fail(MW_EINVAL, "null argument");
    if (!s->loaded) return fail(MW_ESTATE, "no model loaded");
    for (int i = 0; i < s->model.dofs(); ++i)
        if (s->model.bodies[i].joint_name == name) {
            *dof = i;
            return MW_OK;
        }
    return fail(MW_ENOTFOUND, std::string("joint '") + name + "' not found");
}

int mw_joint_type(const mw_sim* s, int32_t dof, int32_t* type) {
    if (!s || !type) return fail(MW_EINVAL, "null argument");
    if (!s->loaded) return fail(MW_ESTATE, "no model loaded");
    if (dof < 0 || dof >= s->model.dofs()) return fail(MW_EINVAL, "dof out of range");
    const mw::ChainBody& b = s->model.bodies[dof];
    *type = b.ball ? MW_JOINT_BALL : ((b.type == mw::JType::Prismatic) ? MW_JOINT_PRISMATIC : MW_JOINT_REVOLUTE);
    return MW_OK;
}

int mw_model_name(const mw_sim* s, char* buf, int32_t len) {
    if (!s || !s->loaded) return fail(MW_ESTATE, "no model loaded");
    return copy_str(s->model_name, buf, len);
}

int mw_base_frame(const mw_sim* s, char* buf, int32_t len) {
    if (!s || !s->loaded) return fail(MW_ESTATE, "no model loaded");
    return copy_str(s->model.base_link, buf, len);
}

int mw_set_joint_param(mw_sim* s, int32_t dof, int32_t which, double value) {
    if (!s || !s->loaded) return fail(MW_ESTATE, "no model loaded");
    if (dof < 0 || dof >= s->model.dofs()) return fail(MW_EINVAL, "dof out of range");
    // Joint.cpp:262-266: parameters can change only while the model was just created
    if (s->stepped) return fail(MW_ESTATE, "The model has been already processed and its parameters cannot be modified");
    mw::ChainBody& b = s->model.bodies[dof];
    switch (which) {
    case MW_PARAM_COULOMB_FRICTION: b.friction = value; break;
    case MW_PARAM_VISCOUS_FRICTION:
        // a damped floating tree runs on the wave kernel (dual recursion);
        // before the first step a lane-kernel model can still switch
        if (s->float_tree && value != 0.0 && !s->wave) {
            if (!s->wave_depth_ok)
                return fail(MW_EPARSE, "joint damping on this floating-base model needs the world-per-wavefront "
                                       "kernel, whose depth limit the tree exceeds");
            if (s->initialized && !s->d_pid) {
                int rc = alloc_wave_buffers(s);
                if (rc) return rc;
                s->fdev.warm = s->d_warm;
                s->pid_dirty = true;
            }
            s->wave = true;
        }
        b.damping = value;
        break;
    case MW_PARAM_MAX_GENERALIZED_FORCE: b.effort = value; break;
    case MW_PARAM_POSITION_LIMIT_MIN: b.lower = value; break;
    case MW_PARAM_POSITION_LIMIT_MAX: b.upper = value; break;
    default: return fail(MW_EINVAL, "unknown joint parameter");
    }
    if (s->initialized) return upload_params(s);
    build_params(s);
    return MW_OK;
}

int mw_joint_param(const mw_sim* s, int32_t dof, int32_t which, double* value) {
    if (!s || !value) return fail(MW_EINVAL, "null argument");
    if (!s->loaded) return fail(MW_ESTATE, "no model loaded");
    if (dof < 0 || dof >= s->model.dofs()) return fail(MW_EINVAL, "dof out of range");
    const mw::ChainBody& b = s->model.bodies[dof];
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

int mw_model_export(const mw_sim* s, double* out, int32_t len) {
    if (!s || !out) return fail(MW_EINVAL, "null argument");
    if (!s->loaded) return fail(MW_ESTATE, "no model loaded");
    const int n = s->model.dofs();
    if (len < 34 * n + 3) return fail(MW_EINVAL, "export buffer too small");
    double* o = out;
    for (const mw::ChainBody& b : s->model.bodies) {
        *o++ = static_cast<double>(((b.type == mw::JType::Prismatic) ? 1 : 0) | (b.ball << 4));
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
    const auto& R = s->model.base_R;
    for (int k = 0; k < 3; ++k) *o++ = R[k] * s->gravity[0] + R[3 + k] * s->gravity[1] + R[6 + k] * s->gravity[2];
    return MW_OK;
}

int mw_model_export_base(const mw_sim* s, double* out) {
    if (!s || !out) return fail(MW_EINVAL, "null argument");
    if (!s->loaded) return fail(MW_ESTATE, "no model loaded");
    const mw::ChainModel& m = s->model;
    double* o = out;
    *o++ = m.floating ? 1.0 : 0.0;
    for (double v : m.base_R) *o++ = v;
    for (double v : m.base_p) *o++ = v;
    *o++ = m.base_mass;
    for (double v : m.base_com) *o++ = v;
    for (double v : m.base_Ic) *o++ = v;
    return MW_OK;
}

int mw_model_export_shapes(const mw_sim* s, int32_t body, double* out, int32_t max_shapes, int32_t* count) {
    if (!s || !count || (max_shapes > 0 && !out)) return fail(MW_EINVAL, "null argument");
    if (!s->loaded) return fail(MW_ESTATE, "no model loaded");
    if (body < -1 || body >= s->model.dofs()) return fail(MW_EINVAL, "body index out of range");
    const std::vector<mw::Shape>& sh = body < 0 ? s->model.base_shapes : s->model.bodies[body].shapes;
    *count = static_cast<int32_t>(sh.size());
    for (int32_t k = 0; k < std::min<int32_t>(max_shapes, *count); ++k) {
        double* o = out + 16 * k;
        *o++ = static_cast<double>(sh[k].type);
        for (double v : sh[k].size) *o++ = v;
        for (double v : sh[k].R) *o++ = v;
        for (double v : sh[k].p) *o++ = v;
    }
    return MW_OK;
}

int mw_compile_collisions(const char* model, const double pose[7], double* out, int32_t max_shapes, int32_t* count) {
    if (!model || !count || (max_shapes > 0 && !out)) return fail(MW_EINVAL, "null argument");
    const double ident[7] = {0, 0, 0, 1, 0, 0, 0};
    mw::ChainModel cm;
    try {
        cm = mw::compile_urdf(model, pose ? pose : ident);
    } catch (const std::exception& e) {
        return fail(MW_EPARSE, e.what());
    }
    std::vector<std::pair<int, const mw::Shape*>> all;
    for (const auto& sh : cm.base_shapes) all.push_back({-1, &sh});
    for (int b = 0; b < cm.dofs(); ++b)
        for (const auto& sh : cm.bodies[b].shapes) all.push_back({b, &sh});
    *count = static_cast<int32_t>(all.size());
    for (int32_t k = 0; k < std::min<int32_t>(max_shapes, *count); ++k) {
        const mw::Shape& sh = *all[k].second;
        double* o = out + MW_COLLISION_WORDS * k;
        std::fill(o, o + MW_COLLISION_WORDS, 0.0);
        *o++ = all[k].first;
        *o++ = static_cast<double>(sh.type);
        for (double v : sh.size) *o++ = v;
        for (double v : sh.R) *o++ = v;
        for (double v : sh.p) *o++ = v;
        *o++ = static_cast<double>(sh.points.size());
        for (const auto& pt : sh.points)
            for (double v : pt) *o++ = v;
    }
    return MW_OK;
}

int mw_get_joint_positions(const mw_sim* cs, int32_t w0, int32_t nw, const int32_t* d, int32_t nd, double* out) {
    mw_sim* s = const_cast<mw_sim*>(cs);
    return getter(s, w0, nw, d, nd, out, [&](int dof, int w) { return double(s->hq()[s->idx(dof, w)]); });
}
int mw_get_joint_velocities(const mw_sim* cs, int32_t w0, int32_t nw, const int32_t* d, int32_t nd, double* out) {
    mw_sim* s = const_cast<mw_sim*>(cs);
    return getter(s, w0, nw, d, nd, out, [&](int dof, int w) { return double(s->hqd()[s->idx(dof, w)]); });
}
int mw_get_joint_accelerations(const mw_sim* cs, int32_t w0, int32_t nw, const int32_t* d, int32_t nd, double* out) {
    mw_sim* s = const_cast<mw_sim*>(cs);
    return getter(s, w0, nw, d, nd, out, [&](int dof, int w) { return double(s->hqdd()[s->idx(dof, w)]); });
}
int mw_get_joint_forces(const mw_sim* cs, int32_t w0, int32_t nw, const int32_t* d, int32_t nd, double* out) {
    // DART clears the joint forces at the end of World::step (clearInternalForces),
    // so GetForce -- the JointForce component readback, Physics.cpp:2330-2345 -- is 0
    mw_sim* s = const_cast<mw_sim*>(cs);
    return getter(s, w0, nw, d, nd, out, [](int, int) { return 0.0; });
}
int mw_get_joint_force_targets(const mw_sim* cs, int32_t w0, int32_t nw, const int32_t* d, int32_t nd, double* out) {
    mw_sim* s = const_cast<mw_sim*>(cs);
    return getter(s, w0, nw, d, nd, out, [&](int dof, int w) { return s->cmd64[s->idx(dof, w)]; });
}
int mw_get_joint_velocity_targets(const mw_sim* cs, int32_t w0, int32_t nw, const int32_t* d, int32_t nd, double* out) {
    mw_sim* s = const_cast<mw_sim*>(cs);
    return getter(s, w0, nw, d, nd, out, [&](int dof, int w) { return double(s->hvt()[s->idx(dof, w)]); });
}
int mw_get_joint_position_targets(const mw_sim* cs, int32_t w0, int32_t nw, const int32_t* d, int32_t nd, double* out) {
    mw_sim* s = const_cast<mw_sim*>(cs);
    if (s && s->initialized) {
        int rc = pull_ptgt(s);
        if (rc) return rc;
    }
    return getter(s, w0, nw, d, nd, out, [&](int dof, int w) { return s->ptgt[s->idx(dof, w)]; });
}

int mw_set_joint_force_targets(mw_sim* s, int32_t w0, int32_t nw, const int32_t* d, int32_t nd, const double* v) {
    // Joint::setGeneralizedForceTarget, Joint.cpp:774-815: allowed in Force,
    // Position, PositionInterpolated and Velocity modes
    return setter(s, w0, nw, d, nd, v, [&](int dof, int w, double x, bool dry) {
        const int m = s->mode[s->idx(dof, w)];
        if (m != MW_MODE_FORCE && m != MW_MODE_POSITION && m != MW_MODE_POSITION_INTERPOLATED &&
            m != MW_MODE_VELOCITY)
            return fail(MW_ESTATE, "The active joint control mode does not accept a force target");
        if (!dry) {
            s->cmd64[s->idx(dof, w)] = x;
            s->hcmd()[s->idx(dof, w)] = static_cast<float>(x);
        }
        return MW_OK;
    });
}

int mw_set_joint_velocity_targets(mw_sim* s, int32_t w0, int32_t nw, const int32_t* d, int32_t nd, const double* v) {
    // Joint::setVelocityTarget, Joint.cpp:728-754
    return setter(s, w0, nw, d, nd, v, [&](int dof, int w, double x, bool dry) {
        const int m = s->mode[s->idx(dof, w)];
        if (m != MW_MODE_VELOCITY && m != MW_MODE_VELOCITY_FOLLOWER_DART && m != MW_MODE_FORCE)
            return fail(MW_ESTATE, "The active joint control mode does not accept a velocity target");
        if (!dry) s->hvt()[s->idx(dof, w)] = static_cast<float>(x);
        return MW_OK;
    });
}

int mw_set_joint_position_targets(mw_sim* s, int32_t w0, int32_t nw, const int32_t* d, int32_t nd, const double* v) {
    // Joint::setPositionTarget, Joint.cpp:694-726
    if (s && s->initialized) {
        int rc = pull_ptgt(s);
        if (rc) return rc;
    }
    return setter(s, w0, nw, d, nd, v, [&](int dof, int w, double x, bool dry) {
        const int m = s->mode[s->idx(dof, w)];
        if (m != MW_MODE_POSITION && m != MW_MODE_POSITION_INTERPOLATED && m != MW_MODE_IDLE &&
            m != MW_MODE_FORCE)
            return fail(MW_ESTATE, "The active joint control mode does not accept a position target");
        if (!dry) {
            s->ptgt[s->idx(dof, w)] = x;
            s->h_ptgt[s->idx(dof, w)] = static_cast<float>(x);
            s->ptgt_dirty = true;
        }
        return MW_OK;
    });
}

int mw_reset_joint_positions(mw_sim* s, int32_t w0, int32_t nw, const int32_t* d, int32_t nd, const double* v) {
    // Joint::resetPosition writes JointPositionReset, applied by the next run (Joint.cpp:132-156)
    const int rc = setter(s, w0, nw, d, nd, v, [&](int dof, int w, double x, bool dry) {
        if (!dry) {
            s->hrq()[s->idx(dof, w)] = static_cast<float>(x);
            s->hrflag()[s->idx(dof, w)] |= 1u | 4u;  // Joint::resetPosition also resets the PID
        }
        return MW_OK;
    });
    return rc ? rc : rearm_diverged(s, w0, nw);
}

int mw_reset_joint_velocities(mw_sim* s, int32_t w0, int32_t nw, const int32_t* d, int32_t nd, const double* v) {
    const int rc = setter(s, w0, nw, d, nd, v, [&](int dof, int w, double x, bool dry) {
        if (!dry) {
            s->hrqd()[s->idx(dof, w)] = static_cast<float>(x);
            s->hrflag()[s->idx(dof, w)] |= 2u | 4u;
        }
        return MW_OK;
    });
    return rc ? rc : rearm_diverged(s, w0, nw);
}

int mw_set_joint_control_mode(mw_sim* s, int32_t w0, int32_t nw, const int32_t* d, int32_t nd, int32_t mode) {
    int rc = check_sim(s);
    if (rc) return rc;
    // Joint::setControlMode, Joint.cpp:369-460
    if (mode == MW_MODE_POSITION_INTERPOLATED) return fail(MW_EINVAL, "PositionInterpolated not yet supported");
    if (mode != MW_MODE_IDLE && mode != MW_MODE_FORCE && mode != MW_MODE_VELOCITY_FOLLOWER_DART &&
        mode != MW_MODE_POSITION && mode != MW_MODE_VELOCITY)
        return fail(MW_EINVAL, "You cannot set the Invalid control mode");
    std::vector<int32_t> sel;
    if ((rc = selection(s, w0, nw, d, nd, sel))) return rc;
    if ((rc = pull_state(s))) return rc;
    if ((rc = pull_ptgt(s))) return rc;
    for (int32_t w = w0; w < w0 + nw; ++w)
        for (int32_t dof : sel) {
            const size_t i = s->idx(dof, w);
            s->mode[i] = mode;
            // targets are deleted and re-initialised from the current state (:418-446)
            s->hcmd()[i] = 0.f;
            s->cmd64[i] = 0.0;
            const bool vel = (mode == MW_MODE_VELOCITY_FOLLOWER_DART || mode == MW_MODE_VELOCITY);
            s->hvt()[i] = vel ? s->hqd()[i] : 0.f;
            s->ptgt[i] = s->hq()[i];
            s->h_ptgt[i] = s->hq()[i];
            uint8_t act = mw::kActForce;
            if (mode == MW_MODE_VELOCITY_FOLLOWER_DART) act = mw::kActServo;
            else if (mode == MW_MODE_POSITION) act = mw::kActPidPos;
            else if (mode == MW_MODE_VELOCITY) act = mw::kActPidVel;
            s->hact()[i] = act;
            s->hrflag()[i] |= 4u;  // pid.Reset() (:453-457)
        }
    if (mode == MW_MODE_VELOCITY_FOLLOWER_DART) s->servo_used = true;
    if (mode == MW_MODE_POSITION || mode == MW_MODE_VELOCITY || mode == MW_MODE_VELOCITY_FOLLOWER_DART)
        s->controller = true;
    s->cmd_dirty = true;
    s->ptgt_dirty = true;
    return MW_OK;
}

int mw_set_joint_pid(mw_sim* s, int32_t dof, const double gains[8]) {
    if (!s || !gains) return fail(MW_EINVAL, "null argument");
    if (!s->loaded) return fail(MW_ESTATE, "no model loaded");
    if (dof < 0 || dof >= s->n) return fail(MW_EINVAL, "dof out of range");
    // Joint::setPID, Joint.cpp:479-525: output limits less limiting than the
    // joint's maximum generalized force are replaced by +-effort
    std::array<double, 8> g;
    std::memcpy(g.data(), gains, sizeof(double) * 8);
    const double maxf = s->model.bodies[dof].effort;
    if (g[3] < -maxf || g[4] > maxf) {
        g[3] = -maxf;
        g[4] = maxf;
    }
    s->pid[dof] = g;
    s->pid_dirty = true;
    // a new ignition::math::PID starts from a reset state (before mw_initialize
    // the device state is zero-initialised anyway)
    if (s->initialized) {
        for (int32_t w = 0; w < s->W; ++w) s->hrflag()[s->idx(dof, w)] |= 4u;
        s->cmd_dirty = true;
    }
    return MW_OK;
}

int mw_joint_pid(const mw_sim* s, int32_t dof, double gains[8]) {
    if (!s || !gains) return fail(MW_EINVAL, "null argument");
    if (!s->loaded) return fail(MW_ESTATE, "no model loaded");
    if (dof < 0 || dof >= s->model.dofs()) return fail(MW_EINVAL, "dof out of range");
    std::memcpy(gains, s->pid[dof].data(), sizeof(double) * 8);
    return MW_OK;
}

int mw_set_controller_period(mw_sim* s, double period) {
    if (!s) return fail(MW_EINVAL, "null simulator handle");
    // Model::setControllerPeriod, Model.cpp:589-602 (doubleToSteadyClockDuration truncates)
    if (!(period > 0.0)) return fail(MW_EINVAL, "The controller period must be greater than zero");
    const double ns = period * 1e9;
    s->period_ns = ns >= 9.2e18 ? std::numeric_limits<int64_t>::max() : static_cast<int64_t>(ns);
    return MW_OK;
}

int mw_controller_period(const mw_sim* s, double* period) {
    if (!s || !period) return fail(MW_EINVAL, "null argument");
    *period = static_cast<double>(s->period_ns) / 1e9;
    return MW_OK;
}

int mw_joint_control_mode(const mw_sim* s, int32_t w, int32_t dof, int32_t* mode) {
    int rc = check_sim(s);
    if (rc) return rc;
    if (!mode) return fail(MW_EINVAL, "null argument");
    if (w < 0 || w >= s->W || dof < 0 || dof >= s->n) return fail(MW_EINVAL, "index out of range");
    *mode = s->mode[s->idx(dof, w)];
    return MW_OK;
}

// ------------------------------------------------- floating bodies ----

static int check_free(const mw_sim* s) {
    int rc = check_sim(s);
    if (rc) return rc;
    if (!s->floating) return fail(MW_ESTATE, "the model has a fixed base");
    return MW_OK;
}

int mw_is_floating(const mw_sim* s, int32_t* floating) {
    if (!s || !floating) return fail(MW_EINVAL, "null argument");
    if (!s->loaded) return fail(MW_ESTATE, "no model loaded");
    *floating = s->floating ? 1 : 0;
    return MW_OK;
}

static float* base_at(const mw_sim* s, int f, int w) { return s->h_base + static_cast<size_t>(f) * s->W + w; }

// the base of a fixed-base model is the model frame, at rest (Model::basePosition
// reads the model's Pose component, Model.cpp:976-994)
static int fixed_base_pose(const mw_sim* s, int32_t w0, int32_t nw, double* out, bool velocity) {
    if (!out || w0 < 0 || nw < 0 || w0 + nw > s->W) return fail(MW_EINVAL, "bad world range or null output");
    const auto& R = s->model.base_R;
    const double tr = R[0] + R[4] + R[8];
    double q[4];
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
    for (int32_t k = 0; k < nw; ++k) {
        if (velocity) {
            for (int f = 0; f < 6; ++f) out[6 * k + f] = 0.0;
        } else {
            for (int f = 0; f < 3; ++f) out[7 * k + f] = s->model.base_p[f];
            for (int f = 0; f < 4; ++f) out[7 * k + 3 + f] = q[f];
        }
    }
    return MW_OK;
}

int mw_get_base_pose(const mw_sim* cs, int32_t w0, int32_t nw, double* out) {
    mw_sim* s = const_cast<mw_sim*>(cs);
    int rc = check_sim(s);
    if (rc) return rc;
    if (!s->floating) return fixed_base_pose(s, w0, nw, out, false);
    if (!out || w0 < 0 || nw < 0 || w0 + nw > s->W) return fail(MW_EINVAL, "bad world range or null output");
    if ((rc = pull_state(s))) return rc;
    // Model::basePosition / baseOrientation (Model.cpp:976-994): x y z, qw qx qy qz
    for (int32_t k = 0; k < nw; ++k)
        for (int f = 0; f < 7; ++f) out[7 * k + f] = *base_at(s, f, w0 + k);
    return MW_OK;
}

int mw_get_base_velocity(const mw_sim* cs, int32_t w0, int32_t nw, double* out) {
    mw_sim* s = const_cast<mw_sim*>(cs);
    int rc = check_sim(s);
    if (rc) return rc;
    if (!s->floating) return fixed_base_pose(s, w0, nw, out, true);
    if (!out || w0 < 0 || nw < 0 || w0 + nw > s->W) return fail(MW_EINVAL, "bad world range or null output");
    if ((rc = pull_state(s))) return rc;
    // Model::baseWorldLinearVelocity / baseWorldAngularVelocity (Model.cpp:1024-1075):
    // the body-frame twist rotated into the world frame
    for (int32_t k = 0; k < nw; ++k) {
        const int w = w0 + k;
        const double qw = *base_at(s, 3, w), qx = *base_at(s, 4, w), qy = *base_at(s, 5, w), qz = *base_at(s, 6, w);
        const double R[9] = {1 - 2 * (qy * qy + qz * qz), 2 * (qx * qy - qw * qz), 2 * (qx * qz + qw * qy),
                             2 * (qx * qy + qw * qz), 1 - 2 * (qx * qx + qz * qz), 2 * (qy * qz - qw * qx),
                             2 * (qx * qz - qw * qy), 2 * (qy * qz + qw * qx), 1 - 2 * (qx * qx + qy * qy)};
        const double wb[3] = {*base_at(s, 7, w), *base_at(s, 8, w), *base_at(s, 9, w)};
        const double vb[3] = {*base_at(s, 10, w), *base_at(s, 11, w), *base_at(s, 12, w)};
        for (int r = 0; r < 3; ++r) {
            out[6 * k + r] = R[r * 3] * vb[0] + R[r * 3 + 1] * vb[1] + R[r * 3 + 2] * vb[2];
            out[6 * k + 3 + r] = R[r * 3] * wb[0] + R[r * 3 + 1] * wb[1] + R[r * 3 + 2] * wb[2];
        }
    }
    return MW_OK;
}

int mw_reset_base_pose(mw_sim* s, int32_t w0, int32_t nw, const double* in) {
    int rc = check_free(s);
    if (rc) return rc;
    if (!in || w0 < 0 || nw < 0 || w0 + nw > s->W) return fail(MW_EINVAL, "bad world range or null input");
    // Model::resetBasePose (Model.cpp:256-289): WorldPoseCmd, applied by the next run
    for (int32_t k = 0; k < nw; ++k) {
        const double* v = in + 7 * k;
        const double qn = std::sqrt(v[3] * v[3] + v[4] * v[4] + v[5] * v[5] + v[6] * v[6]);
        if (!(qn > 0.0)) return fail(MW_EINVAL, "the base orientation quaternion is zero");
    }
    const size_t W = static_cast<size_t>(s->W);
    for (int32_t k = 0; k < nw; ++k) {
        for (int f = 0; f < 7; ++f) s->h_rpose[f * W + w0 + k] = static_cast<float>(in[7 * k + f]);
        s->h_rflag[w0 + k] |= 1u;
    }
    s->free_dirty = true;
    return rearm_diverged(s, w0, nw);
}

int mw_reset_base_velocity(mw_sim* s, int32_t w0, int32_t nw, const double* in) {
    int rc = check_free(s);
    if (rc) return rc;
    if (!in || w0 < 0 || nw < 0 || w0 + nw > s->W) return fail(MW_EINVAL, "bad world range or null input");
    // Model::resetBaseWorldVelocity (Model.cpp:343-400): WorldVelocityCmd
    const size_t W = static_cast<size_t>(s->W);
    for (int32_t k = 0; k < nw; ++k) {
        for (int f = 0; f < 6; ++f) s->h_rvel[f * W + w0 + k] = static_cast<float>(in[6 * k + f]);
        s->h_rflag[w0 + k] |= 2u;
    }
    s->free_dirty = true;
    return rearm_diverged(s, w0, nw);
}

int mw_set_pgs_options(mw_sim* s, double tol, int32_t warm_start) {
    if (!s) return fail(MW_EINVAL, "null simulator handle");
    if (!(tol >= 0.0) || tol >= 1.0) return fail(MW_EINVAL, "the PGS velocity tolerance must be in [0, 1)");
    const bool warm = warm_start != 0;
    if (warm && s->initialized && !s->wave)
        return fail(MW_ESTATE, "warm-started PGS needs the world-per-wavefront kernel (articulated floating "
                               "bases / generic fixed trees); this model runs on another kernel");
    if (warm && !s->pgs_warm && s->d_warm) {
        // a fresh warm start: no stale impulses from before the option was off
        MW_HIP(hipMemsetAsync(s->d_warm, 0, static_cast<size_t>(mw::kWaveWarmWordsHost) * s->W * sizeof(float),
                              s->stream));
    }
    s->pgs_tol = tol;
    s->pgs_warm = warm;
    return MW_OK;
}

// Link::applyWorldWrench (Link.cpp:484-560) on the batched simulator: a
// world force at the link origin and a world torque (wrench[6 * nw]: f xyz,
// tau xyz per world), applied from the next physics step for max(1,
// ceil(duration / dt)) steps, as mw_scene_apply_world_wrench.  link -1 = the
// base.  The wave kernel carries them (articulated floating bases and generic
// fixed-base trees); other kernels fail with MW_ESTATE.
int mw_apply_link_wrench(mw_sim* s, int32_t link, int32_t w0, int32_t nw, const double* wrench, double duration) {
    if (!s || !s->loaded) return fail(MW_ESTATE, "no model loaded");
    if (!s->initialized) return fail(MW_ESTATE, "the simulator is not initialized");
    if (!wrench && nw > 0) return fail(MW_EINVAL, "null argument");
    if (w0 < 0 || nw < 0 || w0 + nw > s->W) return fail(MW_EINVAL, "world range out of bounds");
    if (!s->wave)
        return fail(MW_ESTATE, "world wrenches on mw_sim need the world-per-wavefront kernel (articulated floating "
                               "bases, generic fixed-base trees); fixed-base chains and free bodies take them "
                               "through a scene (mw_scene_apply_world_wrench)");
    if (link < -1 || link >= s->n) return fail(MW_EINVAL, "link index out of range");
    if (!(duration >= 0.0)) return fail(MW_EINVAL, "the wrench duration must be >= 0");
    const int nn = s->n + 1;
    const size_t W = static_cast<size_t>(s->W);
    if (!s->d_ext) {
        s->h_wr.assign(static_cast<size_t>(mw::kSimWrenchSlots) * 6 * nn * W, 0.f);
        s->h_wl.assign(static_cast<size_t>(mw::kSimWrenchSlots) * nn * W, -1);
        MW_HIP(hipMalloc(reinterpret_cast<void**>(&s->d_ext), 6 * nn * W * sizeof(float)));
        MW_HIP(hipHostMalloc(reinterpret_cast<void**>(&s->h_ext), 6 * nn * W * sizeof(float), hipHostMallocDefault));
        s->fdev.wrench = s->d_ext;
        s->fdev.wnodes = nn;
    }
    const int node = link + 1;
    const int64_t d_ns = static_cast<int64_t>(duration * 1e9);
    const int64_t k = std::max<int64_t>(1, (d_ns + s->dt_ns - 1) / s->dt_ns);
    const int64_t last = s->iterations + k;
    if (last > std::numeric_limits<int32_t>::max()) return fail(MW_EINVAL, "wrench expiry beyond the counter range");
    auto wl = [&](int sl, int w) -> int32_t& { return s->h_wl[(static_cast<size_t>(sl) * nn + node) * W + w]; };
    auto wr = [&](int sl, int e, int w) -> float& {
        return s->h_wr[((static_cast<size_t>(sl) * 6 + e) * nn + node) * W + w];
    };
    // validate first: a failing call changes nothing
    for (int w = w0; w < w0 + nw; ++w) {
        bool ok = false;
        for (int sl = 0; sl < mw::kSimWrenchSlots && !ok; ++sl) ok = wl(sl, w) == last || wl(sl, w) <= s->iterations;
        if (!ok) return fail(MW_ESTATE, "too many concurrent wrenches with different durations on one link");
    }
    for (int w = w0; w < w0 + nw; ++w) {
        int slot = -1;
        for (int sl = 0; sl < mw::kSimWrenchSlots && slot < 0; ++sl)
            if (wl(sl, w) == last) slot = sl;
        for (int sl = 0; sl < mw::kSimWrenchSlots && slot < 0; ++sl)
            if (wl(sl, w) <= s->iterations) {
                slot = sl;
                for (int e = 0; e < 6; ++e) wr(sl, e, w) = 0.f;
            }
        wl(slot, w) = static_cast<int32_t>(last);
        for (int e = 0; e < 6; ++e) wr(slot, e, w) += static_cast<float>(wrench[(w - w0) * 6 + e]);
    }
    s->wr_until = std::max(s->wr_until, last);
    return MW_OK;
}

int mw_set_lcp_solver(mw_sim* s, int32_t mode, int32_t max_solves) {
    if (!s) return fail(MW_EINVAL, "null simulator handle");
    if (mode != MW_LCP_PGS && mode != MW_LCP_EXACT) return fail(MW_EINVAL, "unknown LCP solver mode");
    if (mode == MW_LCP_EXACT && (max_solves < 1 || max_solves > 256))
        return fail(MW_EINVAL, "the exact solve's budget must be 1..256 linear solves per step");
    if (mode == MW_LCP_EXACT && s->loaded && s->floating && !s->wave)
        return fail(MW_ESTATE, "this model was loaded for the PGS-only lane kernel: select MW_LCP_EXACT before "
                               "mw_load_model (the exact solve runs on the world-per-wavefront kernel)");
    s->lcp_mode = mode;
    s->lcp_solves = (mode == MW_LCP_EXACT) ? max_solves : 0;
    return MW_OK;
}

int mw_lcp_solver(const mw_sim* s, int32_t* mode, int32_t* max_solves) {
    if (!s || !mode || !max_solves) return fail(MW_EINVAL, "null argument");
    // a floating model on a lane kernel runs the PGS sweeps only
    const bool pgs_kernel = s->loaded && s->floating && !s->wave;
    *mode = pgs_kernel ? MW_LCP_PGS : s->lcp_mode;
    *max_solves = pgs_kernel ? 0 : s->lcp_solves;
    return MW_OK;
}

int mw_pgs_options(const mw_sim* s, double* tol, int32_t* warm_start) {
    if (!s || !tol || !warm_start) return fail(MW_EINVAL, "null argument");
    *tol = s->pgs_tol;
    *warm_start = s->pgs_warm ? 1 : 0;
    return MW_OK;
}

int mw_set_ground_plane(mw_sim* s, int32_t enabled, double mu) {
    if (!s) return fail(MW_EINVAL, "null simulator handle");
    if (!(mu >= 0.0)) return fail(MW_EINVAL, "the friction coefficient must be >= 0");
    s->ground = enabled != 0;
    s->ground_mu = mu;
    if (s->fbase() && s->initialized) return upload_params(s);
    if (s->float_tree && s->loaded) build_float(s);
    else if (s->floating && s->loaded) build_free(s);
    return MW_OK;
}

int mw_enable_contacts(mw_sim* s, int32_t enable) {
    if (!s) return fail(MW_EINVAL, "null simulator handle");
    // Model::enableContacts (Model.cpp:686-700)
    s->contacts = enable != 0;
    if (!s->contacts && s->h_cmask) std::memset(s->h_cmask, 0, static_cast<size_t>(s->W) * sizeof(uint32_t));
    return MW_OK;
}

int mw_contacts_enabled(const mw_sim* s, int32_t* enabled) {
    if (!s || !enabled) return fail(MW_EINVAL, "null argument");
    *enabled = s->contacts ? 1 : 0;
    return MW_OK;
}

int mw_get_contacts(const mw_sim* s, int32_t w, double* out, int32_t cap, int32_t* n) {
    int rc = check_sim(s);
    if (rc) return rc;
    if (!n || (cap > 0 && !out)) return fail(MW_EINVAL, "null argument");
    if (w < 0 || w >= s->W) return fail(MW_EINVAL, "world index out of range");
    *n = 0;
    if (!s->fbase() || !s->contacts) return MW_OK;
    if (s->contacts_stale) {
        mw_sim* m = const_cast<mw_sim*>(s);
        const size_t Wc = static_cast<size_t>(s->W);
        MW_HIP(hipMemcpyAsync(m->h_cmask, s->fdev.cmask, Wc * sizeof(uint32_t), hipMemcpyDeviceToHost, s->stream));
        MW_HIP(hipMemcpyAsync(m->h_cdata, s->fdev.cdata, 7 * static_cast<size_t>(s->n_slots) * Wc * sizeof(float),
                              hipMemcpyDeviceToHost, s->stream));
        MW_HIP(hipStreamSynchronize(s->stream));
        m->contacts_stale = false;
    }
    // contacts of the last substep of the last run (Physics.cpp:2351-2540): per
    // point x y z, normal (into the body), force on the body (N), depth
    const size_t W = static_cast<size_t>(s->W);
    const uint32_t mask = s->h_cmask[w];
    int32_t k = 0;
    for (int slot = 0; slot < s->n_slots; ++slot) {
        if (!((mask >> slot) & 1u)) continue;
        if (k < cap) {
            const float* c = s->h_cdata + static_cast<size_t>(slot) * 7 * W + w;
            double* o = out + 10 * k;
            o[0] = c[0]; o[1] = c[W]; o[2] = c[2 * W];
            o[3] = 0.0; o[4] = 0.0; o[5] = 1.0;
            o[6] = c[3 * W]; o[7] = c[4 * W]; o[8] = c[5 * W];
            o[9] = c[6 * W];
        }
        ++k;
    }
    *n = k;
    return MW_OK;
}

int mw_get_contact_bodies(const mw_sim* s, int32_t w, int32_t* out, int32_t cap, int32_t* n) {
    int rc = check_sim(s);
    if (rc) return rc;
    if (!n || (cap > 0 && !out)) return fail(MW_EINVAL, "null argument");
    if (w < 0 || w >= s->W) return fail(MW_EINVAL, "world index out of range");
    double scratch[10];
    int32_t total = 0;
    // the same slot walk as mw_get_contacts (fills the host mirror if stale)
    if ((rc = mw_get_contacts(s, w, scratch, 0, &total))) return rc;
    const uint32_t mask = (s->fbase() && s->contacts) ? s->h_cmask[w] : 0u;
    int32_t k = 0;
    for (int slot = 0; slot < s->n_slots; ++slot) {
        if (!((mask >> slot) & 1u)) continue;
        if (k < cap) out[k] = s->float_tree ? s->slot_body[slot] : -1;
        ++k;
    }
    *n = k;
    return MW_OK;
}

int mw_device_ptr(mw_sim* s, const char* field, void** dptr, int64_t* stride) {
    int rc = check_sim(s);
    if (rc) return rc;
    if (!field || !dptr) return fail(MW_EINVAL, "null argument");
    const std::string f(field);
    if (f == "q") *dptr = s->dev.q;
    else if (f == "qd") *dptr = s->dev.qd;
    else if (f == "qdd") *dptr = s->dev.qdd;
    else if (f == "position_target") {
        // the caller drives the targets on the device from now on
        if ((rc = pull_ptgt(s))) return rc;
        if (s->ptgt_dirty) {
            MW_HIP(hipMemcpyAsync(s->d_aux, s->h_ptgt, s->nw * sizeof(float), hipMemcpyHostToDevice, s->stream));
            s->ptgt_dirty = false;
        }
        *dptr = s->dev.ptgt;
        if (stride) *stride = s->W;
        s->ptgt_stale = true;
        s->ptgt_view = true;
        return MW_OK;
    } else return fail(MW_ENOTFOUND, "unknown field '" + f + "'");
    if (stride) *stride = s->W;
    s->host_stale = true;  // the caller may write through the view
    return MW_OK;
}

// ------------------------------------------------ divergence, snapshots ----

int mw_diverged(mw_sim* s, int32_t w0, int32_t nw, uint8_t* flags, int64_t* count) {
    int rc = check_sim(s);
    if (rc) return rc;
    if (w0 < 0 || nw < 0 || w0 + nw > s->W) return fail(MW_EINVAL, "world range out of bounds");
    if (flags && nw) MW_HIP(hipMemcpyAsync(flags, s->dev.div + w0, nw, hipMemcpyDeviceToHost, s->stream));
    uint64_t n = 0;
    MW_HIP(hipMemcpyAsync(&n, s->dev.ndiv, sizeof(n), hipMemcpyDeviceToHost, s->stream));
    MW_HIP(hipStreamSynchronize(s->stream));
    if (count) *count = static_cast<int64_t>(n);
    return MW_OK;
}

int mw_clear_diverged(mw_sim* s, int32_t w0, int32_t nw) {
    int rc = check_sim(s);
    if (rc) return rc;
    if (w0 < 0 || nw < 0 || w0 + nw > s->W) return fail(MW_EINVAL, "world range out of bounds");
    if (nw) MW_HIP(hipMemsetAsync(s->dev.div + w0, 0, nw, s->stream));
    return MW_OK;
}

int mw_state_words(const mw_sim* s, int32_t* words) {
    int rc = check_sim(s);
    if (rc) return rc;
    if (!words) return fail(MW_EINVAL, "null argument");
    *words = state_words(s);
    return MW_OK;
}

int mw_get_state(mw_sim* s, int32_t w0, int32_t nw, float* out) {
    int rc = check_sim(s);
    if (rc) return rc;
    if (!out || w0 < 0 || nw < 0 || w0 + nw > s->W) return fail(MW_EINVAL, "bad argument");
    if (!nw) return MW_OK;
    const int K = state_words(s);
    std::vector<float> tmp(static_cast<size_t>(K) * nw);
    int row = 0;
    for (const auto& r : state_rows(s)) {
        MW_HIP(hipMemcpy2DAsync(tmp.data() + static_cast<size_t>(row) * nw, nw * sizeof(float), r.first + w0,
                                static_cast<size_t>(s->W) * sizeof(float), nw * sizeof(float), r.second,
                                hipMemcpyDeviceToHost, s->stream));
        row += r.second;
    }
    MW_HIP(hipStreamSynchronize(s->stream));
    for (int w = 0; w < nw; ++w)
        for (int k = 0; k < K; ++k) out[static_cast<size_t>(w) * K + k] = tmp[static_cast<size_t>(k) * nw + w];
    return MW_OK;
}

int mw_set_state(mw_sim* s, int32_t w0, int32_t nw, const float* in) {
    int rc = check_sim(s);
    if (rc) return rc;
    if (!in || w0 < 0 || nw < 0 || w0 + nw > s->W) return fail(MW_EINVAL, "bad argument");
    if (!nw) return MW_OK;
    const int K = state_words(s);
    std::vector<float> tmp(static_cast<size_t>(K) * nw);
    for (int w = 0; w < nw; ++w)
        for (int k = 0; k < K; ++k) tmp[static_cast<size_t>(k) * nw + w] = in[static_cast<size_t>(w) * K + k];
    int row = 0;
    for (const auto& r : state_rows(s)) {
        MW_HIP(hipMemcpy2DAsync(r.first + w0, static_cast<size_t>(s->W) * sizeof(float),
                                tmp.data() + static_cast<size_t>(row) * nw, nw * sizeof(float), nw * sizeof(float),
                                r.second, hipMemcpyHostToDevice, s->stream));
        row += r.second;
    }
    // the record replaces the worlds' state: their pending resets (joint,
    // base) are dropped and their divergence flags cleared
    for (int d = 0; d < s->n && s->nw; ++d)
        for (int w = w0; w < w0 + nw; ++w) s->hrflag()[s->idx(d, w)] = 0;
    for (int w = w0; w < w0 + nw && !s->h_rflag.empty(); ++w) s->h_rflag[w] = 0;
    MW_HIP(hipMemsetAsync(s->dev.div + w0, 0, nw, s->stream));
    MW_HIP(hipStreamSynchronize(s->stream));
    s->host_stale = true;
    s->contacts_stale = s->fbase() && s->contacts;
    return MW_OK;
}

int mw_copy_state(mw_sim* s, float* q, float* qd, int to_sim) {
    int rc = check_sim(s);
    if (rc) return rc;
    if (!q || !qd) return fail(MW_EINVAL, "null argument");
    const size_t bytes = s->nw * sizeof(float);
    if (to_sim) {
        MW_HIP(hipMemcpyAsync(s->dev.q, q, bytes, hipMemcpyDeviceToDevice, s->stream));
        MW_HIP(hipMemcpyAsync(s->dev.qd, qd, bytes, hipMemcpyDeviceToDevice, s->stream));
        MW_HIP(hipMemsetAsync(s->dev.qlo, 0, bytes, s->stream));
        s->host_stale = true;
    } else {
        MW_HIP(hipMemcpyAsync(q, s->dev.q, bytes, hipMemcpyDeviceToDevice, s->stream));
        MW_HIP(hipMemcpyAsync(qd, s->dev.qd, bytes, hipMemcpyDeviceToDevice, s->stream));
    }
    return MW_OK;
}

// ------------------------------------------------------------- VecEnv ----

int mw_vecenv_create(mw_sim* s, const mw_task_config* cfg, mw_vecenv** out) {
    int rc = check_sim(s);
    if (rc) return rc;
    if (!cfg || !out) return fail(MW_EINVAL, "null argument");
    *out = nullptr;
    const int n = s->n;
    // the batched env kernels step fixed-base chains only: a floating model
    // with a matching dof count would have its base and contacts ignored
    if (s->floating) return fail(MW_EINVAL, "the batched env tasks need a fixed-base model");
    // ... and a compiled chain topology: a generic fixed tree (wave kernel) or
    // a branched 1-2 dof model would be stepped as a serial chain
    if (s->fixed_tree || s->topo < 0)
        return fail(MW_EINVAL, "the batched env tasks need a serial-chain model (or the shipped Panda tree)");
    const bool cart = cfg->kind >= MW_TASK_CARTPOLE_DISCRETE && cfg->kind <= MW_TASK_CARTPOLE_CONTINUOUS_SWINGUP;
    const bool pidtask = cfg->kind == MW_TASK_PANDA_POSITION_TRACKING;
    if (cart && n != 2) return fail(MW_EINVAL, "CartPole tasks need the 2-dof cartpole model");
    if (cfg->kind == MW_TASK_PENDULUM_SWINGUP && n != 1) return fail(MW_EINVAL, "PendulumSwingUp needs the 1-dof pendulum model");
    if (pidtask && (n != 9 || s->topo != 1))
        return fail(MW_EINVAL, "PandaPositionTracking needs the 9-dof Panda model");
    if (pidtask && s->cfg.steps_per_run > 64) return fail(MW_EINVAL, "steps_per_run must be <= 64");
    if (!cart && !pidtask && cfg->kind != MW_TASK_PENDULUM_SWINGUP) return fail(MW_EINVAL, "unknown task kind");
    auto e = std::make_unique<mw_vecenv>();
    e->sim = s;
    e->cfg = *cfg;
    mw::TaskF& T = e->task;
    T.kind = cfg->kind;
    T.max_steps = cfg->max_episode_steps;
    T.reward_cart_at_center = cfg->reward_cart_at_center;
    T.n_obs = (cfg->kind == MW_TASK_PENDULUM_SWINGUP) ? 3 : (pidtask ? 2 * n : 4);
    T.seed_lo = static_cast<uint32_t>(cfg->seed);
    T.seed_hi = static_cast<uint32_t>(cfg->seed >> 32);
    if (cfg->world_offset < 0) return fail(MW_EINVAL, "world_offset must be >= 0");
    T.world_offset = static_cast<uint32_t>(cfg->world_offset);
    T.force_mag = 20.0f;  // cartpole_discrete_balancing.py:32
    const double pi = 3.14159265358979323846;
    switch (cfg->kind) {
    case MW_TASK_CARTPOLE_DISCRETE:
    case MW_TASK_CARTPOLE_CONTINUOUS_BALANCING:
        T.x_factor = (cfg->kind == MW_TASK_CARTPOLE_DISCRETE) ? 0.9f : 1.0f;
        T.hi[0] = 2.4f; T.hi[1] = 20.0f;
        T.hi[2] = static_cast<float>(12.0 * pi / 180.0);
        T.hi[3] = static_cast<float>(3.0 * 360.0 * pi / 180.0);
        break;
    case MW_TASK_CARTPOLE_CONTINUOUS_SWINGUP:
        T.x_factor = 0.8f;
        T.hi[0] = 2.4f; T.hi[1] = 20.0f;
        T.hi[2] = static_cast<float>(5.0 * 360.0 * pi / 180.0);
        T.hi[3] = static_cast<float>(3.0 * 360.0 * pi / 180.0);
        break;
    case MW_TASK_PENDULUM_SWINGUP:
        T.x_factor = 0.f;
        T.hi[0] = 1.f; T.hi[1] = 1.f; T.hi[2] = 10.f; T.hi[3] = 0.f;
        break;
    case MW_TASK_PANDA_POSITION_TRACKING: {
        // the Panda wrapper's initial configuration (models/panda.py:41-44) with
        // joints 1 and 6 at mid-range as test_pid_controllers.py:49-59 sets them
        // (so the config-4 sinusoids stay inside the limits) and the fingers
        // half open: no joint starts on a position limit
        const double wrapper[7] = {0.0, -0.785, 0.0, -2.356, 0.0, 1.571, 0.785};
        for (int d = 0; d < n; ++d) {
            const mw::ChainBody& b = s->model.bodies[d];
            double h = (d < 7) ? wrapper[d] : 0.5 * (b.lower + b.upper);
            if (d == 0 || d == 5) h = 0.5 * (b.lower + b.upper);
            T.home[d] = static_cast<float>(h);
        }
        T.home_noise = 0.05f;
        // the JointController runs every physics step (period = step size)
        s->period_ns = s->dt_ns;
        s->controller = true;
        break;
    }
    }
    if (cfg->randomize & ~(MW_RAND_MASS | MW_RAND_GRAVITY)) return fail(MW_EINVAL, "unknown randomisation bits");
    if (cfg->randomize && pidtask) return fail(MW_EINVAL, "randomisation is available for the CartPole / Pendulum tasks");
    if ((cfg->randomize & MW_RAND_MASS) && !(cfg->mass_high >= cfg->mass_low))
        return fail(MW_EINVAL, "mass_high must be >= mass_low");
    if ((cfg->randomize & MW_RAND_GRAVITY) && !(cfg->gravity_std >= 0.f))
        return fail(MW_EINVAL, "gravity_std must be >= 0");
    T.randomize = cfg->randomize;
    T.mass_lo = cfg->mass_low;
    T.mass_hi = cfg->mass_high;
    T.g_mean = cfg->gravity_mean;
    T.g_std = cfg->gravity_std;
    {
        // the world z axis in the base frame: R_base^T e_z
        const auto& R = s->model.base_R;
        for (int k = 0; k < 3; ++k) T.gdir[k] = static_cast<float>(R[6 + k]);
    }
    MW_HIP(hipSetDevice(s->cfg.device));
    if (cfg->randomize) {
        const size_t bytes = (static_cast<size_t>(n) + 1) * s->W * sizeof(float);
        MW_HIP(hipMalloc(&e->d_physics, bytes));
        MW_HIP(hipMemsetAsync(e->d_physics, 0, bytes, s->stream));
        e->dev.rmass = static_cast<float*>(e->d_physics);
        e->dev.rgz = e->dev.rmass + static_cast<size_t>(n) * s->W;
    }
    MW_HIP(hipMalloc(&e->d_counters, 2 * static_cast<size_t>(s->W) * sizeof(uint32_t)));
    MW_HIP(hipMemsetAsync(e->d_counters, 0, 2 * static_cast<size_t>(s->W) * sizeof(uint32_t), s->stream));
    e->dev.episode = static_cast<uint32_t*>(e->d_counters);
    e->dev.steps = e->dev.episode + s->W;
    *out = e.release();
    return MW_OK;
}

void mw_vecenv_destroy(mw_vecenv* e) {
    if (!e) return;
    if (e->sim && e->sim->stream) (void)hipStreamSynchronize(e->sim->stream);
    (void)hipFree(e->d_counters);
    (void)hipFree(e->d_physics);
    (void)hipFree(e->d_lane);
    delete e;
}

int mw_vecenv_obs_dim(const mw_vecenv* e, int32_t* n) {
    if (!e || !n) return fail(MW_EINVAL, "null argument");
    *n = e->task.n_obs;
    return MW_OK;
}

int mw_vecenv_reset(mw_vecenv* e, float* obs) {
    if (!e || !obs) return fail(MW_EINVAL, "null argument");
    mw_sim* s = e->sim;
    MW_HIP(mw::launch_vecenv_reset(s->d_params, s->n, e->task, s->dev, e->dev, obs, s->W, s->stream));
    s->host_stale = true;
    return MW_OK;
}

static int vec_common(mw_vecenv* e, int32_t T, const void* a, float* o, float* r, uint8_t* d, float* to) {
    if (!e || !a || !o || !r || !d || !to) return fail(MW_EINVAL, "null argument");
    if (e->task.n_obs == 4 &&
        ((reinterpret_cast<uintptr_t>(o) | reinterpret_cast<uintptr_t>(to)) & 15u))
        return fail(MW_EINVAL, "obs buffers must be 16-byte aligned");
    mw_sim* s = e->sim;
    if (e->task.kind == MW_TASK_PANDA_POSITION_TRACKING) {
        if (T > 0) return fail(MW_EINVAL, "the fused rollout is not available for position-target tasks");
        // one world per 16-lane row (group_kernel.hip) unless
        // MWSTEP_PANDA_KERNEL=lane asks for the one-world-per-lane kernel
        const char* kk = std::getenv("MWSTEP_PANDA_KERNEL");
        if (kk && std::strcmp(kk, "lane") == 0) {
            MW_HIP(mw::launch_vecenv_pid_step(s->d_params, s->n, s->topo, needs_cons(s), needs_dual(s), baked_id(s),
                                              e->task, s->dev, e->dev, pid_set(s), static_cast<const float*>(a), o,
                                              r, d, to, s->W, static_cast<float>(s->cfg.step_size),
                                              s->cfg.steps_per_run, s->cfg.pgs_iters, s->stream));
        } else {
            // per-dof gains and reset pose: uploaded when they change (a
            // pageable copy, complete when the call returns; never inside a
            // captured step, where the gains are fixed)
            const mw::PidSet ps = pid_set(s);
            mw::GLaneTask lt[mw::kMaxKernelDofs] = {};
            for (int k = 0; k < s->n; ++k) {
                lt[k].pid = ps.g[k];
                lt[k].home = e->task.home[k];
            }
            if (!e->d_lane) MW_HIP(hipMalloc(reinterpret_cast<void**>(&e->d_lane), sizeof(lt)));
            if (!e->lane_uploaded || std::memcmp(lt, e->h_lane, sizeof(lt)) != 0) {
                std::memcpy(e->h_lane, lt, sizeof(lt));
                MW_HIP(hipMemcpyAsync(e->d_lane, e->h_lane, sizeof(lt), hipMemcpyHostToDevice, s->stream));
                e->lane_uploaded = true;
            }
            MW_HIP(mw::launch_vecenv_pid_group(s->d_params, s->n, needs_cons(s), needs_dual(s), e->task, s->dev,
                                               e->dev, e->d_lane, static_cast<const float*>(a), o, r, d, to, s->W,
                                               static_cast<float>(s->cfg.step_size), s->cfg.steps_per_run,
                                               s->cfg.pgs_iters, s->stream));
        }
        s->host_stale = true;
        s->iterations += s->cfg.steps_per_run;
        s->stepped = true;
        return MW_OK;
    }
    MW_HIP(mw::launch_vecenv_step(s->d_params, s->n, needs_cons(s), needs_dual(s), baked_id(s), e->task, s->dev, e->dev,
                                  a, o, r, d, to, s->W, static_cast<float>(s->cfg.step_size),
                                  s->cfg.steps_per_run, s->cfg.pgs_iters, T, s->stream));
    s->host_stale = true;
    s->iterations += static_cast<int64_t>(s->cfg.steps_per_run) * (T > 0 ? T : 1);
    s->stepped = true;
    return MW_OK;
}

int mw_vecenv_step(mw_vecenv* e, const void* a, float* o, float* r, uint8_t* d, float* to) {
    return vec_common(e, 0, a, o, r, d, to);
}

int mw_vecenv_rollout(mw_vecenv* e, int32_t T, const void* a, float* o, float* r, uint8_t* d, float* to) {
    if (T <= 0) return fail(MW_EINVAL, "T must be positive");
    return vec_common(e, T, a, o, r, d, to);
}

int mw_vecenv_physics(mw_vecenv* e, float* mass, float* gz) {
    if (!e || !mass || !gz) return fail(MW_EINVAL, "null argument");
    if (!e->d_physics) return fail(MW_ESTATE, "the env was created without physics randomisation");
    const size_t nw = static_cast<size_t>(e->sim->n) * e->sim->W;
    MW_HIP(hipMemcpyAsync(mass, e->dev.rmass, nw * sizeof(float), hipMemcpyDeviceToDevice, e->sim->stream));
    MW_HIP(hipMemcpyAsync(gz, e->dev.rgz, e->sim->W * sizeof(float), hipMemcpyDeviceToDevice, e->sim->stream));
    return MW_OK;
}

int mw_vecenv_counters(mw_vecenv* e, uint32_t* episode, uint32_t* steps) {
    if (!e || !episode || !steps) return fail(MW_EINVAL, "null argument");
    const size_t bytes = static_cast<size_t>(e->sim->W) * sizeof(uint32_t);
    MW_HIP(hipMemcpyAsync(episode, e->dev.episode, bytes, hipMemcpyDeviceToDevice, e->sim->stream));
    MW_HIP(hipMemcpyAsync(steps, e->dev.steps, bytes, hipMemcpyDeviceToDevice, e->sim->stream));
    return MW_OK;
}

}  // extern "C"
