// model.hpp -- host-side model compiler: URDF or SDF -> flat kinematic tree.
//
// Mirrors what the reference does when a URDF is inserted
// (World::insertModel, cpp/scenario/gazebo/src/World.cpp:70-180 ->
// sdformat URDF import -> Physics::CreatePhysicsEntities,
// cpp/scenario/plugins/Physics/Physics.cpp:687-1219):
//   - links joined by fixed joints are lumped into one rigid body
//     (sdformat's URDF fixed-joint reduction),
//   - a root link named "world" fixes the model base to the world,
//   - joint axis / limits / effort / damping / friction come from
//     <axis>, <limit>, <dynamics> (ign-physics copies them into DART).
// The output is shared by all worlds of a simulator (topology and
// parameters are read-only on the device).
#pragma once

#include <array>
#include <string>
#include <vector>

namespace mw {

enum class JType : int { Revolute = 0, Prismatic = 1 };

struct ChainBody {
    std::string joint_name;
    std::string link_name;
    int parent = -1;               // parent body index (< own index), -1 = base
    JType type = JType::Revolute;
    bool continuous = false;       // URDF "continuous": revolute without limits
    bool limited = false;          // position limits enforced
    std::array<double, 9> E{};     // joint origin rotation in parent body frame
    std::array<double, 3> r{};     // joint origin translation in parent body frame
    std::array<double, 3> axis{};  // unit axis in the child (joint) frame
    double mass = 0.0;
    std::array<double, 3> com{};   // in body frame
    std::array<double, 6> Ic{};    // about COM: xx yy zz xy xz yz
    double damping = 0.0, friction = 0.0;
    double lower = -1e300, upper = 1e300;
    double effort = 1e300, vel_limit = 1e300;
    std::vector<struct Shape> shapes;  // collision shapes of the (lumped) link, body frame
    // 1..3: part of a ball joint, the rotation about x, y or z of the joint
    // frame (intrinsic X-Y-Z angles; parts 1 and 2 are massless, part 3
    // carries the child link); 0: a 1-dof joint
    int ball = 0;
};

// A collision shape in its body's frame: box (size = half extents), sphere
// (size[0] = radius), cylinder along z (size = {radius, half length}) or mesh
// (mesh.cpp: size = half extents of its bounding box, R / p = the mesh frame
// moved to the box centre, points = its ground-contact support points in that
// frame).  Other geometries are counted, not modelled.
constexpr int kMeshMaxPoints = 16;
struct Shape {
    enum Type : int { Box = 0, Sphere = 1, Cylinder = 2, Mesh = 3 } type = Box;
    std::array<double, 3> size{};
    std::array<double, 9> R{};
    std::array<double, 3> p{};
    std::vector<std::array<double, 3>> points;  // Mesh only
};

// mesh.cpp: vertices of an STL / OBJ file; URI -> file path (the reference's
// asFullPath); the Mesh shape of scaled vertices under collision pose (R, p).
std::vector<std::array<double, 3>> load_mesh_vertices(const std::string& path);
// model.cpp (it owns the XML reader): vertices of a COLLADA document
std::vector<std::array<double, 3>> dae_vertices(const std::string& path, const std::string& data);
std::string resolve_mesh_uri(const std::string& uri, const std::string& model_dir);
Shape mesh_shape(const std::vector<std::array<double, 3>>& verts, const std::array<double, 3>& scale,
                 const std::array<double, 9>& R, const std::array<double, 3>& p);

struct ChainModel {
    std::string name;              // robot name
    std::string base_link;         // canonical (base) link
    // floating base: the root link is not attached to "world"; it moves with a
    // 6-dof free joint (DART FreeJoint) and carries the lumped inertia below
    bool floating = false;
    double base_mass = 0.0;
    std::array<double, 3> base_com{};
    std::array<double, 6> base_Ic{};   // about the COM: xx yy zz xy xz yz
    std::vector<Shape> base_shapes;    // collision shapes of the base body
    int unsupported_shapes = 0;        // collision geometries other than box / sphere / cylinder
    std::array<double, 9> base_R{};  // base pose in world
    std::array<double, 3> base_p{};
    std::vector<ChainBody> bodies; // depth-first: bodies[i].parent < i (-1 = base)
    int dofs() const { return static_cast<int>(bodies.size()); }
};

// Parse a URDF or SDF model (file path or inline string).  pose =
// {x,y,z,qw,qx,qy,qz}; for SDF the identity keeps the model's <pose>
// (World::insertModel, World.cpp:169-177).
// Throws std::runtime_error with a message on unsupported / malformed input.
ChainModel compile_urdf(const std::string& path_or_xml, const double pose[7]);

}  // namespace mw
