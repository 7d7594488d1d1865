// model.cpp -- minimal XML reader + URDF / SDF -> tree compiler (see model.hpp).
#include "model.hpp"

#include <cctype>
#include <cmath>
#include <cstdlib>
#include <fstream>
#include <functional>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>

namespace mw {
namespace {

// ------------------------------------------------------------------ XML ----
struct XNode {
    std::string tag;
    std::string text;  // character data directly inside the element (SDF values)
    std::map<std::string, std::string> attr;
    std::vector<std::unique_ptr<XNode>> kids;

    const XNode* child(const std::string& t) const {
        for (auto& k : kids)
            if (k->tag == t) return k.get();
        return nullptr;
    }
    std::vector<const XNode*> children(const std::string& t) const {
        std::vector<const XNode*> out;
        for (auto& k : kids)
            if (k->tag == t) out.push_back(k.get());
        return out;
    }
    const std::string* get(const std::string& a) const {
        auto it = attr.find(a);
        return it == attr.end() ? nullptr : &it->second;
    }
};

class XmlReader {
public:
    explicit XmlReader(const std::string& s) : s_(s) {}

    std::unique_ptr<XNode> parse() {
        std::unique_ptr<XNode> root;
        while (skip_misc()) {
            if (root) fail("multiple root elements");
            root = element();
        }
        if (!root) fail("no root element");
        return root;
    }

private:
    const std::string& s_;
    size_t i_ = 0;

    [[noreturn]] void fail(const std::string& what) const {
        throw std::runtime_error("XML parse error at offset " + std::to_string(i_) + ": " + what);
    }
    bool eof() const { return i_ >= s_.size(); }
    bool starts(const char* p) const { return s_.compare(i_, std::char_traits<char>::length(p), p) == 0; }
    void ws() {
        while (!eof() && std::isspace(static_cast<unsigned char>(s_[i_]))) ++i_;
    }
    void skip_until(const char* end) {
        size_t k = s_.find(end, i_);
        if (k == std::string::npos) fail(std::string("unterminated construct, expected ") + end);
        i_ = k + std::char_traits<char>::length(end);
    }
    // skips whitespace, comments, PIs, doctype, text; returns true when an
    // element start tag follows
    bool skip_misc() {
        for (;;) {
            ws();
            if (eof()) return false;
            if (starts("<?")) { skip_until("?>"); continue; }
            if (starts("<!--")) { skip_until("-->"); continue; }
            if (starts("<!")) { skip_until(">"); continue; }
            if (s_[i_] == '<') return true;
            ++i_;  // stray text
        }
    }
    std::string name() {
        size_t b = i_;
        while (!eof() && (std::isalnum(static_cast<unsigned char>(s_[i_])) || s_[i_] == '_' ||
                          s_[i_] == ':' || s_[i_] == '-' || s_[i_] == '.'))
            ++i_;
        if (b == i_) fail("expected a name");
        return s_.substr(b, i_ - b);
    }
    std::unique_ptr<XNode> element() {
        if (s_[i_] != '<') fail("expected '<'");
        ++i_;
        auto n = std::make_unique<XNode>();
        n->tag = name();
        for (;;) {
            ws();
            if (eof()) fail("unterminated start tag");
            if (starts("/>")) { i_ += 2; return n; }
            if (s_[i_] == '>') { ++i_; break; }
            std::string a = name();
            ws();
            if (eof() || s_[i_] != '=') fail("expected '=' after attribute " + a);
            ++i_;
            ws();
            if (eof() || (s_[i_] != '"' && s_[i_] != '\'')) fail("expected quoted value");
            const char q = s_[i_++];
            size_t e = s_.find(q, i_);
            if (e == std::string::npos) fail("unterminated attribute value");
            n->attr[a] = s_.substr(i_, e - i_);
            i_ = e + 1;
        }
        // content
        for (;;) {
            if (eof()) fail("unterminated element <" + n->tag + ">");
            if (starts("</")) {
                i_ += 2;
                std::string t = name();
                if (t != n->tag) fail("mismatched </" + t + "> for <" + n->tag + ">");
                ws();
                if (eof() || s_[i_] != '>') fail("expected '>'");
                ++i_;
                return n;
            }
            if (starts("<!--")) { skip_until("-->"); continue; }
            if (starts("<![CDATA[")) { skip_until("]]>"); continue; }
            if (starts("<?")) { skip_until("?>"); continue; }
            if (s_[i_] == '<') { n->kids.push_back(element()); continue; }
            n->text.push_back(s_[i_++]);  // character data (SDF element values)
        }
    }
};

// ------------------------------------------------------------ math -----
using M3 = std::array<double, 9>;
using V3 = std::array<double, 3>;

M3 eye() { return {1, 0, 0, 0, 1, 0, 0, 0, 1}; }
M3 mul(const M3& a, const M3& b) {
    M3 c{};
    for (int r = 0; r < 3; ++r)
        for (int k = 0; k < 3; ++k)
            c[r * 3 + k] = a[r * 3] * b[k] + a[r * 3 + 1] * b[3 + k] + a[r * 3 + 2] * b[6 + k];
    return c;
}
V3 mul(const M3& a, const V3& v) {
    return {a[0] * v[0] + a[1] * v[1] + a[2] * v[2], a[3] * v[0] + a[4] * v[1] + a[5] * v[2],
            a[6] * v[0] + a[7] * v[1] + a[8] * v[2]};
}
M3 transpose(const M3& a) { return {a[0], a[3], a[6], a[1], a[4], a[7], a[2], a[5], a[8]}; }
V3 add(const V3& a, const V3& b) { return {a[0] + b[0], a[1] + b[1], a[2] + b[2]}; }
V3 sub(const V3& a, const V3& b) { return {a[0] - b[0], a[1] - b[1], a[2] - b[2]}; }
V3 scale(const V3& a, double s) { return {a[0] * s, a[1] * s, a[2] * s}; }

// URDF rpy: fixed-axis roll (x), pitch (y), yaw (z): R = Rz * Ry * Rx
M3 rpy(const V3& v) {
    const double cr = std::cos(v[0]), sr = std::sin(v[0]);
    const double cp = std::cos(v[1]), sp = std::sin(v[1]);
    const double cy = std::cos(v[2]), sy = std::sin(v[2]);
    const M3 Rx{1, 0, 0, 0, cr, -sr, 0, sr, cr};
    const M3 Ry{cp, 0, sp, 0, 1, 0, -sp, 0, cp};
    const M3 Rz{cy, -sy, 0, sy, cy, 0, 0, 0, 1};
    return mul(Rz, mul(Ry, Rx));
}

M3 quat_wxyz(double w, double x, double y, double z) {
    const double n = std::sqrt(w * w + x * x + y * y + z * z);
    if (n == 0.0) throw std::runtime_error("zero quaternion in model pose");
    w /= n; x /= n; y /= n; z /= n;
    return {1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
            2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
            2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)};
}

std::vector<double> numbers(const std::string& s) {
    std::vector<double> out;
    const char* p = s.c_str();
    char* end = nullptr;
    for (;;) {
        double v = std::strtod(p, &end);
        if (end == p) break;
        out.push_back(v);
        p = end;
    }
    return out;
}

V3 vec_attr(const XNode* n, const char* a, V3 dflt) {
    if (!n) return dflt;
    const std::string* s = n->get(a);
    if (!s) return dflt;
    auto v = numbers(*s);
    if (v.size() != 3) throw std::runtime_error(std::string("expected 3 numbers in attribute ") + a);
    return {v[0], v[1], v[2]};
}

double num_attr(const XNode* n, const char* a, double dflt) {
    if (!n) return dflt;
    const std::string* s = n->get(a);
    if (!s) return dflt;
    auto v = numbers(*s);
    if (v.size() != 1) throw std::runtime_error(std::string("expected a number in attribute ") + a);
    return v[0];
}

// --------------------------------------------------------------- URDF ---
struct Link {
    double mass = 0.0;
    V3 com{};
    M3 I{};  // about COM, link frame
    std::vector<Shape> shapes;  // collision shapes, link frame
    int unsupported = 0;
};

struct Joint {
    std::string name, type, parent, child;
    M3 R = eye();
    V3 p{};
    V3 axis{1, 0, 0};
    double lower = -1e300, upper = 1e300, effort = 1e300, velocity = 1e300;
    double damping = 0.0, friction = 0.0;
};

Link merge(const Link& a, const Link& b, const M3& R, const V3& p) {
    Link out;
    out.mass = a.mass + b.mass;
    if (out.mass <= 0.0) return out;
    const V3 cb = add(mul(R, b.com), p);
    for (int k = 0; k < 3; ++k) out.com[k] = (a.mass * a.com[k] + b.mass * cb[k]) / out.mass;
    const M3 Ib = mul(R, mul(b.I, transpose(R)));
    auto shift = [](const M3& I, double m, const V3& d) {
        M3 o = I;
        const double dd = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) o[r * 3 + c] += m * ((r == c ? dd : 0.0) - d[r] * d[c]);
        return o;
    };
    const M3 Ia = shift(a.I, a.mass, sub(a.com, out.com));
    const M3 Ib2 = shift(Ib, b.mass, sub(cb, out.com));
    for (int k = 0; k < 9; ++k) out.I[k] = Ia[k] + Ib2[k];
    return out;
}

// lump b (pose R, p in a) into a: inertia (merge) and collision shapes
Link lump(const Link& a, const Link& b, const M3& R, const V3& p) {
    Link out = (a.mass + b.mass > 0.0) ? merge(a, b, R, p) : Link{};
    out.shapes = a.shapes;
    for (const Shape& sh : b.shapes) {
        Shape t = sh;
        t.R = mul(R, sh.R);
        t.p = add(mul(R, sh.p), p);
        out.shapes.push_back(t);
    }
    out.unsupported = a.unsupported + b.unsupported;
    return out;
}

// directory of the model file being compiled (relative mesh URIs); empty for
// an inline model string (relative to the working directory)
thread_local std::string g_model_dir;

std::string read_source(const std::string& s) {
    size_t k = s.find_first_not_of(" \t\r\n");
    g_model_dir.clear();
    if (k != std::string::npos && s[k] == '<') return s;
    const size_t sl = s.rfind('/');
    g_model_dir = (sl == std::string::npos) ? std::string(".") : s.substr(0, sl);
    std::ifstream f(s);
    if (!f) throw std::runtime_error("cannot open model file '" + s + "'");
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

// The front-ends below describe a model the way URDF does: link contents in
// the link frame, joint origins in the parent link frame, the child link frame
// = the joint frame.  compile_description() then lumps fixed joints and numbers
// the moving joints depth-first.
struct Description {
    std::string name;
    std::map<std::string, Link> links;
    std::vector<std::string> link_order;
    std::vector<Joint> joints;
    M3 R = eye();  // model pose in the world
    V3 p{};
};

// ------------------------------------------------------------ URDF -----
Description describe_urdf(const XNode* root, const double pose[7]) {
    Description D;
    D.name = root->get("name") ? *root->get("name") : "model";
    D.R = quat_wxyz(pose[3], pose[4], pose[5], pose[6]);
    D.p = {pose[0], pose[1], pose[2]};
    std::map<std::string, Link>& links = D.links;
    for (const XNode* le : root->children("link")) {
        const std::string* nm = le->get("name");
        if (!nm) throw std::runtime_error("<link> without name");
        if (links.count(*nm)) throw std::runtime_error("duplicate link '" + *nm + "'");
        Link L;
        if (const XNode* ine = le->child("inertial")) {
            const XNode* o = ine->child("origin");
            const M3 Ro = rpy(vec_attr(o, "rpy", {0, 0, 0}));
            L.com = vec_attr(o, "xyz", {0, 0, 0});
            const XNode* ms = ine->child("mass");
            if (!ms) throw std::runtime_error("<inertial> without <mass> in link " + *nm);
            L.mass = num_attr(ms, "value", 0.0);
            const XNode* ie = ine->child("inertia");
            M3 Iin{};
            if (ie) {
                const double ixx = num_attr(ie, "ixx", 0), iyy = num_attr(ie, "iyy", 0),
                             izz = num_attr(ie, "izz", 0), ixy = num_attr(ie, "ixy", 0),
                             ixz = num_attr(ie, "ixz", 0), iyz = num_attr(ie, "iyz", 0);
                Iin = {ixx, ixy, ixz, ixy, iyy, iyz, ixz, iyz, izz};
            }
            L.I = mul(Ro, mul(Iin, transpose(Ro)));
        }
        for (const XNode* ce : le->children("collision")) {
            const XNode* o = ce->child("origin");
            const XNode* ge = ce->child("geometry");
            const XNode* box = ge ? ge->child("box") : nullptr;
            const XNode* sph = ge ? ge->child("sphere") : nullptr;
            const XNode* cyl = ge ? ge->child("cylinder") : nullptr;
            Shape sh;
            sh.R = rpy(vec_attr(o, "rpy", {0, 0, 0}));
            sh.p = vec_attr(o, "xyz", {0, 0, 0});
            if (box) {
                sh.type = Shape::Box;
                sh.size = scale(vec_attr(box, "size", {0, 0, 0}), 0.5);
            } else if (sph) {
                sh.type = Shape::Sphere;
                sh.size = {num_attr(sph, "radius", 0.0), 0.0, 0.0};
            } else if (cyl) {
                sh.type = Shape::Cylinder;
                sh.size = {num_attr(cyl, "radius", 0.0), 0.5 * num_attr(cyl, "length", 0.0), 0.0};
            } else if (const XNode* me = ge ? ge->child("mesh") : nullptr) {
                const std::string* fn = me->get("filename");
                if (!fn) throw std::runtime_error("<mesh> without filename in link " + *nm);
                sh = mesh_shape(load_mesh_vertices(resolve_mesh_uri(*fn, g_model_dir)),
                                vec_attr(me, "scale", {1, 1, 1}), sh.R, sh.p);
            } else {
                ++L.unsupported;
                continue;
            }
            L.shapes.push_back(sh);
        }
        links[*nm] = L;
        D.link_order.push_back(*nm);
    }

    for (const XNode* je : root->children("joint")) {
        Joint J;
        const std::string* nm = je->get("name");
        const std::string* ty = je->get("type");
        const XNode* pa = je->child("parent");
        const XNode* ch = je->child("child");
        if (!nm || !ty || !pa || !ch || !pa->get("link") || !ch->get("link"))
            throw std::runtime_error("malformed <joint>");
        J.name = *nm;
        J.type = *ty;
        J.parent = *pa->get("link");
        J.child = *ch->get("link");
        const XNode* o = je->child("origin");
        J.R = rpy(vec_attr(o, "rpy", {0, 0, 0}));
        J.p = vec_attr(o, "xyz", {0, 0, 0});
        V3 ax = vec_attr(je->child("axis"), "xyz", {1, 0, 0});
        const double an = std::sqrt(ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2]);
        if (an == 0.0) throw std::runtime_error("zero joint axis in " + J.name);
        J.axis = scale(ax, 1.0 / an);
        if (const XNode* lim = je->child("limit")) {
            J.effort = num_attr(lim, "effort", 1e300);
            J.velocity = num_attr(lim, "velocity", 1e300);
            if (J.type == "revolute" || J.type == "prismatic") {
                J.lower = num_attr(lim, "lower", 0.0);
                J.upper = num_attr(lim, "upper", 0.0);
            }
        }
        if (const XNode* dyn = je->child("dynamics")) {
            J.damping = num_attr(dyn, "damping", 0.0);
            J.friction = num_attr(dyn, "friction", 0.0);
        }
        if (J.type != "fixed" && J.type != "revolute" && J.type != "continuous" &&
            J.type != "prismatic")
            throw std::runtime_error("unsupported joint type '" + J.type + "' (" + J.name + ")");
        if (!links.count(J.parent) || !links.count(J.child))
            throw std::runtime_error("joint " + J.name + " references an unknown link");
        D.joints.push_back(J);
    }
    return D;
}

// ------------------------------------------------------------- SDF -----
// SDF 1.6 / 1.7 frame semantics (sdformat, as read by World::insertModel ->
// utils::getSdfRootFromString, cpp/scenario/gazebo/src/World.cpp:70-180):
// <link><pose> is the link frame in the model frame, <joint><pose> the joint
// frame in the CHILD link frame, <axis><xyz> is expressed in the joint frame
// (or the model frame with <use_parent_model_frame> / expressed_in="__model__"),
// <limit> and <dynamics> live inside <axis>; <inertial><pose> and
// <collision><pose> are in the link frame.  A joint whose parent is "world"
// attaches the model to the world where the model frame is placed.
struct Pose3 {
    M3 R = eye();
    V3 p{};
};
Pose3 compose(const Pose3& a, const Pose3& b) { return {mul(a.R, b.R), add(mul(a.R, b.p), a.p)}; }
Pose3 inverse(const Pose3& a) {
    const M3 Rt = transpose(a.R);
    return {Rt, scale(mul(Rt, a.p), -1.0)};
}

std::string trimmed(const std::string& s) {
    const size_t b = s.find_first_not_of(" \t\r\n");
    if (b == std::string::npos) return "";
    const size_t e = s.find_last_not_of(" \t\r\n");
    return s.substr(b, e - b + 1);
}

std::vector<double> sdf_numbers(const XNode* el, const char* tag, size_t n) {
    const XNode* c = el ? el->child(tag) : nullptr;
    if (!c) return {};
    auto v = numbers(c->text);
    if (v.size() != n)
        throw std::runtime_error("expected " + std::to_string(n) + " numbers in <" + tag + ">");
    return v;
}

double sdf_num(const XNode* el, const char* tag, double dflt) {
    auto v = sdf_numbers(el, tag, 1);
    return v.empty() ? dflt : v[0];
}

bool sdf_bool(const XNode* el, const char* tag, bool dflt) {
    const XNode* c = el ? el->child(tag) : nullptr;
    if (!c) return dflt;
    const std::string t = trimmed(c->text);
    return t == "1" || t == "true";
}

// <pose>x y z roll pitch yaw</pose> of `el` (identity when absent)
Pose3 sdf_pose(const XNode* el, const std::string& what) {
    const XNode* c = el ? el->child("pose") : nullptr;
    if (!c) return {};
    for (const char* a : {"relative_to", "frame"}) {
        const std::string* rel = c->get(a);
        if (rel && !rel->empty())
            throw std::runtime_error("<pose " + std::string(a) + "=\"" + *rel + "\"> of " + what +
                                     " is not supported (poses must use the default frames)");
    }
    auto v = numbers(c->text);
    if (v.size() != 6) throw std::runtime_error("expected 6 numbers in the <pose> of " + what);
    return {rpy({v[3], v[4], v[5]}), {v[0], v[1], v[2]}};
}

Description describe_sdf(const XNode* root, const double pose[7]) {
    auto models = root->children("model");
    if (models.empty())
        throw std::runtime_error(root->child("world") ? "the SDF holds a <world>, not a <model>"
                                                      : "The SDF does not contain a <model>");
    if (models.size() > 1) throw std::runtime_error("the SDF holds several models");
    const XNode* me = models[0];
    if (me->child("model") || me->child("include"))
        throw std::runtime_error("nested models and <include> are not supported");
    Description D;
    D.name = me->get("name") ? *me->get("name") : "model";
    // World::insertModel: a non-identity insertion pose replaces the model's
    // <pose> (World.cpp:169-177), the identity keeps it
    const bool identity = pose[0] == 0.0 && pose[1] == 0.0 && pose[2] == 0.0 && pose[3] == 1.0 &&
                          pose[4] == 0.0 && pose[5] == 0.0 && pose[6] == 0.0;
    if (identity) {
        const Pose3 X = sdf_pose(me, "model '" + D.name + "'");
        D.R = X.R;
        D.p = X.p;
    } else {
        D.R = quat_wxyz(pose[3], pose[4], pose[5], pose[6]);
        D.p = {pose[0], pose[1], pose[2]};
    }

    // links: contents in the SDF link frame
    std::map<std::string, Pose3> X_link;  // link frame in the model frame
    std::map<std::string, Link> raw;
    for (const XNode* le : me->children("link")) {
        const std::string* nm = le->get("name");
        if (!nm) throw std::runtime_error("<link> without name");
        if (*nm == "world") throw std::runtime_error("a link may not be named 'world'");
        if (raw.count(*nm)) throw std::runtime_error("duplicate link '" + *nm + "'");
        X_link[*nm] = sdf_pose(le, "link '" + *nm + "'");
        Link L;
        // sdformat's defaults: mass 1, unit principal moments
        L.mass = 1.0;
        M3 Iin = eye();
        Pose3 Xi;
        if (const XNode* ine = le->child("inertial")) {
            Xi = sdf_pose(ine, "the inertial of link '" + *nm + "'");
            L.mass = sdf_num(ine, "mass", 1.0);
            if (const XNode* ie = ine->child("inertia")) {
                const double ixx = sdf_num(ie, "ixx", 1.0), iyy = sdf_num(ie, "iyy", 1.0),
                             izz = sdf_num(ie, "izz", 1.0), ixy = sdf_num(ie, "ixy", 0.0),
                             ixz = sdf_num(ie, "ixz", 0.0), iyz = sdf_num(ie, "iyz", 0.0);
                Iin = {ixx, ixy, ixz, ixy, iyy, iyz, ixz, iyz, izz};
            }
        }
        L.com = Xi.p;
        L.I = mul(Xi.R, mul(Iin, transpose(Xi.R)));
        for (const XNode* ce : le->children("collision")) {
            const Pose3 Xc = sdf_pose(ce, "a collision of link '" + *nm + "'");
            const XNode* ge = ce->child("geometry");
            const XNode* box = ge ? ge->child("box") : nullptr;
            const XNode* sph = ge ? ge->child("sphere") : nullptr;
            const XNode* cyl = ge ? ge->child("cylinder") : nullptr;
            Shape sh;
            sh.R = Xc.R;
            sh.p = Xc.p;
            if (box) {
                auto v = sdf_numbers(box, "size", 3);
                if (v.empty()) v = {1.0, 1.0, 1.0};
                sh.type = Shape::Box;
                sh.size = {0.5 * v[0], 0.5 * v[1], 0.5 * v[2]};
            } else if (sph) {
                sh.type = Shape::Sphere;
                sh.size = {sdf_num(sph, "radius", 1.0), 0.0, 0.0};
            } else if (cyl) {  // sdformat defaults: radius 0.5, length 1
                sh.type = Shape::Cylinder;
                sh.size = {sdf_num(cyl, "radius", 0.5), 0.5 * sdf_num(cyl, "length", 1.0), 0.0};
            } else if (const XNode* me = ge ? ge->child("mesh") : nullptr) {
                const XNode* uri = me->child("uri");
                if (!uri) throw std::runtime_error("<mesh> without <uri> in link '" + *nm + "'");
                auto sc = sdf_numbers(me, "scale", 3);
                if (sc.empty()) sc = {1.0, 1.0, 1.0};
                sh = mesh_shape(load_mesh_vertices(resolve_mesh_uri(uri->text, g_model_dir)), {sc[0], sc[1], sc[2]},
                                sh.R, sh.p);
            } else {
                ++L.unsupported;
                continue;
            }
            L.shapes.push_back(sh);
        }
        raw[*nm] = L;
        D.link_order.push_back(*nm);
    }
    if (raw.empty()) throw std::runtime_error("model '" + D.name + "' has no links");

    // joints: the joint frame X_J is given in the child link frame; the
    // description's child link frame becomes the joint frame F(C) = X_C X_J
    struct SJ {
        Joint J;
        Pose3 XJ;        // joint frame in the child link frame
        V3 axis_raw{};   // as written
        bool axis_model = false;
    };
    std::vector<SJ> sjs;
    bool world_used = false;
    for (const XNode* je : me->children("joint")) {
        SJ s;
        Joint& J = s.J;
        const std::string* nm = je->get("name");
        const std::string* ty = je->get("type");
        if (!nm || !ty) throw std::runtime_error("malformed <joint>");
        J.name = *nm;
        J.type = *ty;
        const XNode* pa = je->child("parent");
        const XNode* ch = je->child("child");
        if (!pa || !ch) throw std::runtime_error("joint " + J.name + " needs <parent> and <child>");
        J.parent = trimmed(pa->text);
        J.child = trimmed(ch->text);
        if (J.parent == "world") world_used = true;
        else if (!raw.count(J.parent)) throw std::runtime_error("joint " + J.name + " references an unknown link");
        if (!raw.count(J.child)) throw std::runtime_error("joint " + J.name + " references an unknown link");
        if (J.type != "fixed" && J.type != "revolute" && J.type != "continuous" && J.type != "prismatic" &&
            J.type != "ball")
            throw std::runtime_error("unsupported joint type '" + J.type + "' (" + J.name + ")");
        s.XJ = sdf_pose(je, "joint '" + J.name + "'");
        const XNode* ax = je->child("axis");
        if (J.type != "fixed") {
            auto v = sdf_numbers(ax, "xyz", 3);
            s.axis_raw = v.empty() ? V3{0, 0, 1} : V3{v[0], v[1], v[2]};
            const XNode* xe = ax ? ax->child("xyz") : nullptr;
            const std::string* ei = xe ? xe->get("expressed_in") : nullptr;
            s.axis_model = sdf_bool(ax, "use_parent_model_frame", false) || (ei && *ei == "__model__");
            if (ei && !ei->empty() && *ei != "__model__" && *ei != J.name)
                throw std::runtime_error("joint " + J.name + ": axis expressed_in=\"" + *ei + "\" is not supported");
            if (const XNode* lim = ax ? ax->child("limit") : nullptr) {
                J.effort = sdf_num(lim, "effort", -1.0);
                J.velocity = sdf_num(lim, "velocity", -1.0);
                J.lower = sdf_num(lim, "lower", -1e16);
                J.upper = sdf_num(lim, "upper", 1e16);
            } else {
                J.effort = J.velocity = -1.0;
                J.lower = -1e16;
                J.upper = 1e16;
            }
            // a negative effort / velocity is not enforced (SDF spec)
            if (J.effort < 0.0) J.effort = 1e300;
            if (J.velocity < 0.0) J.velocity = 1e300;
            if (J.type == "revolute" && J.lower <= -1e16 && J.upper >= 1e16) J.type = "continuous";
            // a ball joint has no position limits (Joint.cpp:876-880)
            if (J.type == "continuous" || J.type == "ball") { J.lower = -1e300; J.upper = 1e300; }
            if (J.type == "prismatic") {
                if (J.lower <= -1e16) J.lower = -1e300;
                if (J.upper >= 1e16) J.upper = 1e300;
            }
            if (const XNode* dyn = ax ? ax->child("dynamics") : nullptr) {
                J.damping = sdf_num(dyn, "damping", 0.0);
                J.friction = sdf_num(dyn, "friction", 0.0);
            }
        }
        sjs.push_back(s);
    }

    // <static>true</static> (World::insertModel -> a static model in the
    // physics engine): every root link is welded to the world where the model
    // frame is placed
    if (sdf_bool(me, "static", false)) {
        for (const SJ& s : sjs)
            if (s.J.type != "fixed")
                throw std::runtime_error("static models with moving joints are not supported (joint " + s.J.name + ")");
        std::map<std::string, int> has_parent;
        for (const SJ& s : sjs) has_parent[s.J.child] = 1;
        for (auto& n : D.link_order) {
            if (has_parent.count(n)) continue;
            SJ s;
            s.J.name = "__static_" + n;
            s.J.type = "fixed";
            s.J.parent = "world";
            s.J.child = n;
            s.XJ = Pose3{};
            sjs.push_back(s);
            world_used = true;
        }
    }
    // the description frame of every link: the joint frame for a child link,
    // the model frame for the root (its contents move by its link pose)
    std::map<std::string, Pose3> F;
    std::map<std::string, int> parent_joint;
    for (size_t k = 0; k < sjs.size(); ++k) {
        const SJ& s = sjs[k];
        if (parent_joint.count(s.J.child))
            throw std::runtime_error("link '" + s.J.child + "' is the child of several joints");
        parent_joint[s.J.child] = static_cast<int>(k);
        F[s.J.child] = compose(X_link[s.J.child], s.XJ);
    }
    for (auto& n : D.link_order)
        if (!F.count(n)) F[n] = Pose3{};
    F["world"] = Pose3{};

    if (world_used) {
        D.links["world"] = Link{};
        D.link_order.insert(D.link_order.begin(), "world");
    }
    for (auto& n : D.link_order) {
        if (n == "world") continue;
        const Pose3 Xc = compose(inverse(F[n]), X_link[n]);  // SDF link frame in F(n)
        D.links[n] = lump(Link{}, raw[n], Xc.R, Xc.p);
    }
    for (SJ& s : sjs) {
        Joint J = s.J;
        const Pose3 O = compose(inverse(F[J.parent]), F[J.child]);
        J.R = O.R;
        J.p = O.p;
        if (J.type != "fixed") {
            V3 a = s.axis_model ? mul(transpose(F[J.child].R), s.axis_raw) : s.axis_raw;
            const double an = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
            if (an == 0.0) throw std::runtime_error("zero joint axis in " + J.name);
            J.axis = scale(a, 1.0 / an);
        }
        D.joints.push_back(J);
    }
    return D;
}

ChainModel compile_description(Description D) {
    ChainModel out;
    out.name = D.name;
    std::map<std::string, Link>& links = D.links;
    const std::vector<std::string>& link_order = D.link_order;
    std::vector<Joint>& joints = D.joints;

    // root link
    std::map<std::string, int> is_child;
    for (auto& j : joints) is_child[j.child]++;
    std::vector<std::string> roots;
    for (auto& n : link_order)
        if (!is_child.count(n)) roots.push_back(n);
    if (roots.size() != 1) throw std::runtime_error("the model must have exactly one root link");

    M3 baseR = D.R;
    V3 baseP = D.p;
    std::string base = roots[0];
    if (base == "world") {
        int found = -1, attached = 0;
        for (size_t k = 0; k < joints.size(); ++k)
            if (joints[k].parent == "world") {
                ++attached;
                found = static_cast<int>(k);
            }
        if (attached == 0) throw std::runtime_error("nothing is attached to the 'world' link");
        if (attached == 1 && joints[found].type == "fixed") {
            // the usual fixed base: the welded link is the base body
            baseP = add(baseP, mul(baseR, joints[found].p));
            baseR = mul(baseR, joints[found].R);
            base = joints[found].child;
            joints.erase(joints.begin() + found);
        }
        // otherwise the massless 'world' link itself is the fixed base and the
        // joints attached to it hang from the model frame
    } else {
        // floating base: the root link moves with a free joint; its world pose is
        // the insertion pose (World::insertModel, World.cpp:70-180)
        out.floating = true;
    }

    // lump fixed joints into their parent body
    std::map<std::string, std::string> owner;
    std::map<std::string, M3> offR;
    std::map<std::string, V3> offP;
    for (auto& n : link_order) { owner[n] = n; offR[n] = eye(); offP[n] = {0, 0, 0}; }
    for (bool changed = true; changed;) {
        changed = false;
        for (size_t k = 0; k < joints.size(); ++k) {
            if (joints[k].type != "fixed") continue;
            const Joint j = joints[k];
            const std::string po = owner[j.parent];
            const M3 R = mul(offR[j.parent], j.R);
            const V3 p = add(mul(offR[j.parent], j.p), offP[j.parent]);
            links[po] = lump(links[po], links[j.child], R, p);
            for (auto& n : link_order)
                if (owner[n] == j.child) {
                    owner[n] = po;
                    offP[n] = add(mul(R, offP[n]), p);
                    offR[n] = mul(R, offR[n]);
                }
            joints.erase(joints.begin() + static_cast<long>(k));
            changed = true;
            break;
        }
    }

    // the moving joints form a tree hanging from the base body; bodies are
    // numbered depth-first (children in declaration order), so parent < child
    std::vector<const Joint*> order;
    std::vector<int> parent_of;
    {
        std::vector<std::pair<const Joint*, int>> st;  // (joint, parent body index)
        auto push_children = [&](const std::string& link, int pidx) {
            std::vector<const Joint*> kids;
            for (auto& j : joints)
                if (owner[j.parent] == link) kids.push_back(&j);
            for (auto it = kids.rbegin(); it != kids.rend(); ++it) st.push_back({*it, pidx});
        };
        push_children(base, -1);
        while (!st.empty()) {
            const auto [j, pidx] = st.back();
            st.pop_back();
            const int me = static_cast<int>(order.size());
            if (order.size() >= joints.size())
                throw std::runtime_error("the model's joints do not form a tree (a link has several parents)");
            order.push_back(j);
            parent_of.push_back(pidx);
            push_children(j->child, me);
        }
    }
    if (order.size() != joints.size())
        throw std::runtime_error("the model's moving joints are not all connected to the base link");
    std::vector<Joint> chain;
    for (const Joint* j : order) chain.push_back(*j);

    out.base_link = base;
    out.base_R = baseR;
    out.base_p = baseP;
    // a ball joint (SDF "ball", 3 dofs, Joint.cpp:318-331) becomes three
    // revolute joints about the x, y and z axes of its frame at one point, the
    // first two carrying massless bodies: the same rigid motion (a spherical
    // pair), parameterised by intrinsic X-Y-Z angles instead of DART's
    // rotation vector -- the ScenarI/O layer converts positions, velocities,
    // forces and resets (scenario/gazebo.py BallJoint)
    std::vector<int> last_body(chain.size(), -1);  // the body carrying joint k's child link
    for (size_t k = 0; k < chain.size(); ++k) {
        const Joint& j = chain[k];
        const bool ball = (j.type == "ball");
        const int parts = ball ? 3 : 1;
        for (int part = 0; part < parts; ++part) {
            const bool carrier = (part == parts - 1);
            ChainBody b;
            b.parent = (part > 0) ? static_cast<int>(out.bodies.size()) - 1
                                  : (parent_of[k] >= 0 ? last_body[parent_of[k]] : -1);
            b.joint_name = ball ? j.name + (part == 0 ? "#x" : (part == 1 ? "#y" : "#z")) : j.name;
            b.link_name = carrier ? j.child : j.name + (part == 0 ? "#x" : "#y");
            b.type = (j.type == "prismatic") ? JType::Prismatic : JType::Revolute;
            b.continuous = (j.type == "continuous" || ball);
            b.limited = (j.type == "revolute" || j.type == "prismatic");
            if (part == 0) {
                b.E = mul(offR[j.parent], j.R);
                b.r = add(mul(offR[j.parent], j.p), offP[j.parent]);
            } else {
                b.E = eye();
                b.r = {0, 0, 0};
            }
            b.axis = ball ? std::array<double, 3>{part == 0 ? 1.0 : 0.0, part == 1 ? 1.0 : 0.0, part == 2 ? 1.0 : 0.0}
                          : j.axis;
            b.ball = ball ? part + 1 : 0;
            if (carrier) {
                const Link& L = links[j.child];
                b.mass = L.mass;
                b.com = L.com;
                b.Ic = {L.I[0], L.I[4], L.I[8], L.I[1], L.I[2], L.I[5]};
                b.shapes = L.shapes;
                if (b.mass <= 0.0) throw std::runtime_error("moving link '" + j.child + "' has no mass");
            }
            b.damping = j.damping;
            b.friction = j.friction;
            b.lower = j.lower;
            b.upper = j.upper;
            b.effort = j.effort;
            b.vel_limit = j.velocity;
            out.bodies.push_back(b);
        }
        last_body[k] = static_cast<int>(out.bodies.size()) - 1;
    }
    if (out.floating) {
        const Link& B = links[base];
        if (B.mass <= 0.0) throw std::runtime_error("the floating base link '" + base + "' has no mass");
        out.base_mass = B.mass;
        out.base_com = B.com;
        out.base_Ic = {B.I[0], B.I[4], B.I[8], B.I[1], B.I[2], B.I[5]};
        out.base_shapes = B.shapes;
    } else {
        // a welded base (incl. static models) is a collider for the other models
        out.base_shapes = links[base].shapes;
    }
    for (auto& kv : links)
        if (owner[kv.first] == kv.first) out.unsupported_shapes += kv.second.unsupported;
    if (out.bodies.empty() && !out.floating && out.base_shapes.empty())
        throw std::runtime_error("the model has no moving joints and no collision shapes");
    return out;
}

}  // namespace

// COLLADA (.dae) collision meshes, as ign-common's ColladaLoader reads them
// for MeshManager::Load (Physics.cpp:905): the POSITION sources of the
// geometries instantiated by the visual scene's nodes (<instance_geometry>),
// each under its node chain's transform (<matrix> row-major, <translate>,
// <rotate> axis + degrees, <scale>, composed in document order), scaled by
// <asset><unit meter>; without instantiating nodes, every geometry as stored.
// <up_axis> is not applied (vertices stay in the file's frame).
std::vector<std::array<double, 3>> dae_vertices(const std::string& path, const std::string& data) {
    XmlReader rd(data);
    auto root = rd.parse();
    if (root->tag != "COLLADA") throw std::runtime_error("mesh '" + path + "' is not a COLLADA document");
    double unit = 1.0;
    if (const XNode* as = root->child("asset"))
        if (const XNode* u = as->child("unit")) unit = num_attr(u, "meter", 1.0);
    std::vector<std::pair<std::string, std::vector<V3>>> geoms;
    if (const XNode* lg = root->child("library_geometries"))
        for (const XNode* g : lg->children("geometry")) {
            const XNode* me = g->child("mesh");
            const XNode* vt = me ? me->child("vertices") : nullptr;
            if (!vt) continue;
            std::string src;
            for (const XNode* in : vt->children("input"))
                if (in->get("semantic") && *in->get("semantic") == "POSITION" && in->get("source"))
                    src = in->get("source")->substr(1);
            std::vector<V3> v;
            for (const XNode* so : me->children("source")) {
                if (!so->get("id") || *so->get("id") != src) continue;
                const XNode* fa = so->child("float_array");
                if (!fa) continue;
                int stride = 3;
                if (const XNode* tc = so->child("technique_common"))
                    if (const XNode* ac = tc->child("accessor")) stride = static_cast<int>(num_attr(ac, "stride", 3));
                if (stride < 3) throw std::runtime_error("mesh '" + path + "': POSITION stride below 3");
                const std::vector<double> f = numbers(fa->text);
                for (size_t k = 0; k + 2 < f.size(); k += stride) v.push_back({f[k], f[k + 1], f[k + 2]});
            }
            geoms.push_back({g->get("id") ? *g->get("id") : std::string(), v});
        }
    using M4 = std::array<double, 16>;
    auto mul4 = [](const M4& a, const M4& b) {
        M4 c{};
        for (int r = 0; r < 4; ++r)
            for (int k = 0; k < 4; ++k)
                c[r * 4 + k] = a[r * 4] * b[k] + a[r * 4 + 1] * b[4 + k] + a[r * 4 + 2] * b[8 + k] + a[r * 4 + 3] * b[12 + k];
        return c;
    };
    const M4 I4 = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    std::vector<V3> out;
    bool instanced = false;
    std::function<void(const XNode*, M4)> walk = [&](const XNode* nd, M4 M) {
        for (const auto& k : nd->kids) {
            const std::vector<double> f = numbers(k->text);
            M4 T = I4;
            if (k->tag == "matrix" && f.size() == 16) {
                for (int i = 0; i < 16; ++i) T[i] = f[i];
            } else if (k->tag == "translate" && f.size() == 3) {
                T[3] = f[0]; T[7] = f[1]; T[11] = f[2];
            } else if (k->tag == "scale" && f.size() == 3) {
                T[0] = f[0]; T[5] = f[1]; T[10] = f[2];
            } else if (k->tag == "rotate" && f.size() == 4) {
                const double n = std::sqrt(f[0] * f[0] + f[1] * f[1] + f[2] * f[2]);
                const double x = f[0] / n, y = f[1] / n, z = f[2] / n, a = f[3] * M_PI / 180.0;
                const double c = std::cos(a), s = std::sin(a), t = 1.0 - c;
                T = {t * x * x + c, t * x * y - s * z, t * x * z + s * y, 0, t * x * y + s * z, t * y * y + c,
                     t * y * z - s * x, 0, t * x * z - s * y, t * y * z + s * x, t * z * z + c, 0, 0, 0, 0, 1};
            } else {
                continue;
            }
            M = mul4(M, T);
        }
        for (const XNode* ig : nd->children("instance_geometry")) {
            const std::string* url = ig->get("url");
            if (!url || url->empty()) continue;
            for (const auto& g : geoms)
                if (g.first == url->substr(1)) {
                    instanced = true;
                    for (const V3& p : g.second)
                        out.push_back({M[0] * p[0] + M[1] * p[1] + M[2] * p[2] + M[3],
                                       M[4] * p[0] + M[5] * p[1] + M[6] * p[2] + M[7],
                                       M[8] * p[0] + M[9] * p[1] + M[10] * p[2] + M[11]});
                }
        }
        for (const XNode* ch : nd->children("node")) walk(ch, M);
    };
    const XNode* vs = nullptr;
    if (const XNode* lv = root->child("library_visual_scenes")) {
        std::string want;
        if (const XNode* sc = root->child("scene"))
            if (const XNode* iv = sc->child("instance_visual_scene"))
                if (iv->get("url")) want = iv->get("url")->substr(1);
        for (const XNode* v : lv->children("visual_scene"))
            if (!vs || (v->get("id") && *v->get("id") == want)) vs = v;
    }
    if (vs) walk(vs, I4);
    if (!instanced) {
        out.clear();
        for (const auto& g : geoms) out.insert(out.end(), g.second.begin(), g.second.end());
    }
    for (V3& p : out)
        for (double& x : p) x *= unit;
    return out;
}

ChainModel compile_urdf(const std::string& path_or_xml, const double pose[7]) {
    const std::string text = read_source(path_or_xml);
    XmlReader rd(text);
    auto root = rd.parse();
    if (root->tag == "robot") return compile_description(describe_urdf(root.get(), pose));
    if (root->tag == "sdf") return compile_description(describe_sdf(root.get(), pose));
    throw std::runtime_error("expected a URDF <robot> or an SDF <sdf> model (got <" + root->tag + ">)");
}

}  // namespace mw
