// Test-only: the device dynamics code compiled for the host (the same
// tests/host_dyn/harness.cpp the CPU suite loads) under AddressSanitizer +
// UndefinedBehaviorSanitizer (tests/test_sanitizers.py).
//
//   hostdyn_san chain <ChainF file> <case file> <out file>
//       case: int32 n, int32 pgs, int32 cons, int32 dual, float dt,
//             float q[n], qd[n], tau[n], uint8 act[n], float vcmd[n]
//       out:  float q[n], qd[n], qdd[n]
//   hostdyn_san float <ChainF file> <FloatF file> <case file> <out file>
//       case: int32 n, int32 pgs, int32 cons, float dt,
//             float base[13], q[n], qd[n], tau[n]
//       out:  float base[13], q[n], qd[n], uint32 active
// The parameter blocks are the exact bytes the library uploads
// (mw_device_params / mw_device_float_params).
#include "../host_dyn/harness.cpp"

#include <cstdio>
#include <cstring>
#include <vector>

static std::vector<char> slurp(const char* path) {
    std::vector<char> out;
    FILE* f = std::fopen(path, "rb");
    if (!f) return out;
    char buf[4096];
    size_t k;
    while ((k = std::fread(buf, 1, sizeof buf, f)) > 0) out.insert(out.end(), buf, buf + k);
    std::fclose(f);
    return out;
}

template <typename T>
static bool take(const std::vector<char>& s, size_t& at, T* dst, size_t n) {
    if (at + sizeof(T) * n > s.size()) return false;
    std::memcpy(dst, s.data() + at, sizeof(T) * n);
    at += sizeof(T) * n;
    return true;
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const bool flt = std::strcmp(argv[1], "float") == 0;
    if ((!flt && argc != 5) || (flt && argc != 6)) return 2;
    const std::vector<char> pblk = slurp(argv[2]);
    if (pblk.size() != sizeof(ChainF)) return 3;
    // heap copies of exactly the struct size: an out-of-bounds read trips ASan
    ChainF* P = new ChainF;
    std::memcpy(static_cast<void*>(P), pblk.data(), sizeof(ChainF));
    FloatF* F = nullptr;
    if (flt) {
        const std::vector<char> fblk = slurp(argv[3]);
        if (fblk.size() != sizeof(FloatF)) return 3;
        F = new FloatF;
        std::memcpy(static_cast<void*>(F), fblk.data(), sizeof(FloatF));
    }
    const std::vector<char> c = slurp(argv[flt ? 4 : 3]);
    size_t at = 0;
    int32_t hdr[4] = {0, 0, 0, 0};
    float dt = 0.f;
    if (!take(c, at, hdr, flt ? 3 : 4) || !take(c, at, &dt, 1)) return 3;
    const int n = hdr[0];
    if (n < 1 || n > 48) return 3;
    std::vector<float> q(n), qd(n), tau(n), vc(n), qdd(n), base(13);
    std::vector<unsigned char> act(n);
    FILE* o = std::fopen(argv[flt ? 5 : 4], "wb");
    if (!o) return 2;
    int rc;
    if (!flt) {
        if (!take(c, at, q.data(), n) || !take(c, at, qd.data(), n) || !take(c, at, tau.data(), n) ||
            !take(c, at, act.data(), n) || !take(c, at, vc.data(), n))
            return 3;
        rc = hd_substep(P, q.data(), qd.data(), tau.data(), act.data(), vc.data(), dt, hdr[1], hdr[2], hdr[3],
                        qdd.data());
        std::fwrite(q.data(), sizeof(float), n, o);
        std::fwrite(qd.data(), sizeof(float), n, o);
        std::fwrite(qdd.data(), sizeof(float), n, o);
    } else {
        if (!take(c, at, base.data(), 13) || !take(c, at, q.data(), n) || !take(c, at, qd.data(), n) ||
            !take(c, at, tau.data(), n))
            return 3;
        std::vector<float> ws(4096, 0.f);
        unsigned active = 0;
        rc = hd_float_step(P, F, base.data(), q.data(), qd.data(), tau.data(), dt, hdr[1], hdr[2], ws.data(),
                           &active);
        std::fwrite(base.data(), sizeof(float), 13, o);
        std::fwrite(q.data(), sizeof(float), n, o);
        std::fwrite(qd.data(), sizeof(float), n, o);
        std::fwrite(&active, sizeof active, 1, o);
    }
    std::fclose(o);
    delete P;
    delete F;
    return rc == 0 ? 0 : 10 + rc;
}
