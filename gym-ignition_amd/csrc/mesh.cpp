// mesh.cpp -- mesh collision geometries for the model compiler.
//
// The reference attaches <mesh> collisions to DART as triangle meshes
// (cpp/scenario/plugins/Physics/Physics.cpp:897-931: MeshManager::Load of the
// resolved URI, AttachMeshShape with the collision pose and the SDF <scale>).
// Here a mesh becomes a Shape::Mesh: its contact points against the ground
// plane are support points of its vertex set (the vertices extreme along 26
// fixed directions, then along 136 Fibonacci-sphere directions while fewer
// than kMeshMaxPoints were found -- every one a vertex of the convex hull; a
// box-shaped mesh gives exactly its 8 corners, a mesh of at most 16 hull
// vertices all of them), and against the
// shapes of other models it collides as its bounding box in the mesh frame.
// The shape frame is the mesh frame moved to the bounding box centre, so the
// box half extents are Shape::size and the points are relative to the centre.
//
// Formats: STL (binary and ASCII), Wavefront OBJ (`v` records) and COLLADA
// (model.cpp dae_vertices).  Other formats throw: a collision that cannot be
// modelled fails loudly instead of silently dropping contacts.

#include <array>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "model.hpp"

namespace mw {

namespace {

using V3 = std::array<double, 3>;

bool ends_with_ci(const std::string& s, const char* suf) {
    const size_t n = std::strlen(suf);
    if (s.size() < n) return false;
    for (size_t i = 0; i < n; ++i) {
        char a = s[s.size() - n + i];
        if (a >= 'A' && a <= 'Z') a = static_cast<char>(a - 'A' + 'a');
        if (a != suf[i]) return false;
    }
    return true;
}

std::string read_file(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot open mesh file '" + path + "'");
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

std::vector<V3> stl_vertices(const std::string& path, const std::string& data) {
    std::vector<V3> v;
    // binary: 80-byte header, uint32 count, 50 bytes per triangle
    if (data.size() >= 84) {
        uint32_t n = 0;
        std::memcpy(&n, data.data() + 80, 4);
        if (data.size() == 84 + 50 * static_cast<size_t>(n)) {
            v.reserve(3 * n);
            for (uint32_t t = 0; t < n; ++t) {
                const char* rec = data.data() + 84 + 50 * static_cast<size_t>(t) + 12;  // skip the normal
                for (int k = 0; k < 3; ++k) {
                    float xyz[3];
                    std::memcpy(xyz, rec + 12 * k, 12);
                    v.push_back({xyz[0], xyz[1], xyz[2]});
                }
            }
            return v;
        }
    }
    // ASCII: "vertex x y z" records
    std::istringstream in(data);
    std::string tok;
    while (in >> tok) {
        if (tok == "vertex") {
            V3 p;
            if (!(in >> p[0] >> p[1] >> p[2])) throw std::runtime_error("malformed STL vertex in '" + path + "'");
            v.push_back(p);
        }
    }
    return v;
}

std::vector<V3> obj_vertices(const std::string& path, const std::string& data) {
    std::vector<V3> v;
    std::istringstream in(data);
    std::string line;
    while (std::getline(in, line)) {
        if (line.size() < 2 || line[0] != 'v' || (line[1] != ' ' && line[1] != '\t')) continue;
        std::istringstream ls(line.substr(2));
        V3 p;
        if (!(ls >> p[0] >> p[1] >> p[2])) throw std::runtime_error("malformed OBJ vertex in '" + path + "'");
        v.push_back(p);
    }
    return v;
}

bool exists(const std::string& p) {
    std::ifstream f(p);
    return static_cast<bool>(f);
}

}  // namespace

std::vector<std::array<double, 3>> load_mesh_vertices(const std::string& path) {
    const bool stl = ends_with_ci(path, ".stl"), obj = ends_with_ci(path, ".obj"), dae = ends_with_ci(path, ".dae");
    if (!stl && !obj && !dae)
        throw std::runtime_error("mesh '" + path + "': only STL, OBJ and COLLADA collision meshes are supported");
    const std::string data = read_file(path);
    const std::vector<V3> v = stl ? stl_vertices(path, data) : obj ? obj_vertices(path, data) : dae_vertices(path, data);
    if (v.empty()) throw std::runtime_error("mesh '" + path + "' has no vertices");
    return v;
}

// asFullPath(uri, filePath) of the reference: file:// and absolute paths as
// they are, model://<name>/<rest> and package://<name>/<rest> looked up under
// the resource path directories (GZ_SIM_RESOURCE_PATH, IGN_GAZEBO_RESOURCE_PATH,
// SDF_PATH, ROS_PACKAGE_PATH; ':'-separated) and then beside the model file,
// anything else relative to the directory of the model file.
std::string resolve_mesh_uri(const std::string& uri, const std::string& model_dir) {
    std::string u = uri;
    while (!u.empty() && (u.back() == ' ' || u.back() == '\n' || u.back() == '\t' || u.back() == '\r')) u.pop_back();
    size_t b = u.find_first_not_of(" \t\r\n");
    u = (b == std::string::npos) ? std::string() : u.substr(b);
    if (u.rfind("file://", 0) == 0) return u.substr(7);
    const bool model = u.rfind("model://", 0) == 0, package = u.rfind("package://", 0) == 0;
    if (model || package) {
        const std::string rest = u.substr(model ? 8 : 10);
        for (const char* var : {"GZ_SIM_RESOURCE_PATH", "IGN_GAZEBO_RESOURCE_PATH", "SDF_PATH", "ROS_PACKAGE_PATH"}) {
            const char* val = std::getenv(var);
            if (!val) continue;
            std::string list(val);
            size_t s = 0;
            while (s <= list.size()) {
                size_t e = list.find(':', s);
                if (e == std::string::npos) e = list.size();
                const std::string dir = list.substr(s, e - s);
                if (!dir.empty() && exists(dir + "/" + rest)) return dir + "/" + rest;
                s = e + 1;
            }
        }
        // model://<this model>/<rest> from a model directory: its parent holds <name>
        if (!model_dir.empty()) {
            const size_t sl = rest.find('/');
            if (sl != std::string::npos && exists(model_dir + "/" + rest.substr(sl + 1)))
                return model_dir + "/" + rest.substr(sl + 1);
        }
        throw std::runtime_error("cannot resolve mesh URI '" + u + "' (set GZ_SIM_RESOURCE_PATH)");
    }
    if (!u.empty() && u[0] == '/') return u;
    return model_dir.empty() ? u : model_dir + "/" + u;
}

// Directions of the support points, in selection order: the 8 cube corners,
// the 12 edge midpoints, the 6 faces.
static const int kDirs[26][3] = {
    {-1, -1, -1}, {-1, -1, 1}, {-1, 1, -1}, {-1, 1, 1}, {1, -1, -1}, {1, -1, 1}, {1, 1, -1}, {1, 1, 1},
    {-1, -1, 0},  {-1, 1, 0},  {1, -1, 0},  {1, 1, 0},  {-1, 0, -1}, {-1, 0, 1}, {1, 0, -1}, {1, 0, 1},
    {0, -1, -1},  {0, -1, 1},  {0, 1, -1},  {0, 1, 1},  {-1, 0, 0},  {1, 0, 0},  {0, -1, 0}, {0, 1, 0},
    {0, 0, -1},   {0, 0, 1}};

Shape mesh_shape(const std::vector<std::array<double, 3>>& verts, const std::array<double, 3>& scale,
                 const std::array<double, 9>& R, const std::array<double, 3>& p) {
    // scaled vertices (the STL / OBJ repeats are harmless: the first index of
    // the maximum is picked, so a repeated vertex always resolves to the same one)
    std::vector<V3> v;
    v.reserve(verts.size());
    for (const V3& a : verts) v.push_back({a[0] * scale[0], a[1] * scale[1], a[2] * scale[2]});
    V3 lo = v[0], hi = v[0];
    for (const V3& a : v)
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], a[k]);
            hi[k] = std::max(hi[k], a[k]);
        }
    Shape sh;
    sh.type = Shape::Mesh;
    V3 c;
    for (int k = 0; k < 3; ++k) {
        c[k] = 0.5 * (lo[k] + hi[k]);
        sh.size[k] = 0.5 * (hi[k] - lo[k]);
    }
    sh.R = R;
    for (int r = 0; r < 3; ++r) sh.p[r] = p[r] + R[3 * r] * c[0] + R[3 * r + 1] * c[1] + R[3 * r + 2] * c[2];
    std::vector<size_t> pick;
    for (const auto& d : kDirs) {
        size_t best = 0;
        double bv = d[0] * v[0][0] + d[1] * v[0][1] + d[2] * v[0][2];
        for (size_t i = 1; i < v.size(); ++i) {
            const double s = d[0] * v[i][0] + d[1] * v[i][1] + d[2] * v[i][2];
            if (s > bv) { bv = s; best = i; }
        }
        bool seen = false;
        for (size_t j : pick) seen = seen || j == best;
        if (!seen && pick.size() < static_cast<size_t>(kMeshMaxPoints)) pick.push_back(best);
    }
    // room left: the extremes along 136 Fibonacci-sphere directions (a mesh
    // with at most 16 hull vertices ends up with all of them)
    const double golden = M_PI * (3.0 - std::sqrt(5.0));
    for (int k = 0; k < 136 && pick.size() < static_cast<size_t>(kMeshMaxPoints); ++k) {
        const double z = 1.0 - (2.0 * k + 1.0) / 136.0;
        const double r = std::sqrt(1.0 - z * z), phi = golden * k;
        const double d[3] = {r * std::cos(phi), r * std::sin(phi), z};
        size_t best = 0;
        double bv = d[0] * v[0][0] + d[1] * v[0][1] + d[2] * v[0][2];
        for (size_t i = 1; i < v.size(); ++i) {
            const double s = d[0] * v[i][0] + d[1] * v[i][1] + d[2] * v[i][2];
            if (s > bv) { bv = s; best = i; }
        }
        bool seen = false;
        for (size_t j : pick) seen = seen || j == best;
        if (!seen) pick.push_back(best);
    }
    for (size_t i : pick) sh.points.push_back({v[i][0] - c[0], v[i][1] - c[1], v[i][2] - c[2]});
    return sh;
}

}  // namespace mw
