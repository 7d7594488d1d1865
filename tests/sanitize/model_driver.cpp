// Test-only: the C-ABI library's host-side model compiler (csrc/model.cpp,
// csrc/mesh.cpp: URDF / SDF parsing, fixed-joint lumping, mesh readers) under
// AddressSanitizer + UndefinedBehaviorSanitizer (tests/test_sanitizers.py,
// SURVEY.md §5).
//
//   model_san <model file>...
//
// Prints one line per file: the compiled tree's body count, floating flag,
// total moving mass, shape count and joint names -- or the compiler's error
// message (a rejected model is an expected outcome, not a sanitizer failure).
#include <cstdio>
#include <exception>

#include "model.hpp"

int main(int argc, char** argv) {
    const double pose[7] = {0, 0, 0, 1, 0, 0, 0};
    for (int a = 1; a < argc; ++a) {
        try {
            const mw::ChainModel m = mw::compile_urdf(argv[a], pose);
            double mass = m.base_mass;
            size_t shapes = m.base_shapes.size();
            for (const auto& b : m.bodies) {
                mass += b.mass;
                shapes += b.shapes.size();
            }
            std::printf("ok %zu %d %.9g %zu", m.bodies.size(), m.floating ? 1 : 0, mass, shapes);
            for (const auto& b : m.bodies) std::printf(" %s", b.joint_name.c_str());
            std::printf("\n");
        } catch (const std::exception& e) {
            std::printf("error %s\n", e.what());
        }
    }
    return 0;
}
