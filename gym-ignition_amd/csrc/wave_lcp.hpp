// wave_lcp.hpp -- exact solve of the world-per-wavefront kernel's boxed LCP
// (contact normal rows x_n >= 0, friction rows boxed by mu x_n, joint rows in
// [lo, hi]) as DART solves it: BoxedLcpConstraintSolver -> DantzigBoxedLcpSolver
// -> ODE's dSolveLCP [EXT: dart/external/odelcpsolver], reached from
// ForwardStep at /root/reference/cpp/scenario/plugins/Physics/Physics.cpp:1824-1835.
// ODE's friction-index handling moves the friction rows to the end, solves
// the other rows first and, on reaching the first friction row, sets every
// friction box once to +-mu x_n from the normals solved so far.  A is
// symmetric positive definite (the CFM), so the result is the unique pair of
// strictly convex box-QP minimisers (specification: oracle.c lcp_dantzig):
//
//   stage 1  the normal and joint rows, friction impulses pinned at 0;
//   stage 2  all rows, every friction row boxed by +-mu x_n of its contact's
//            STAGE-1 normal (fixed during the stage).
//
// Lane r owns row r: its Delassus row a[c] = A[r][c] (the PGS registers of
// wave_step), its impulse x_r and its row data.  Each stage is a box QP with
// fixed bounds, solved by the primal active-set method (wave_boxqp): the held
// rows sit on a bound, the reduced system A_FF d_F = -g_F over the free rows is
// symmetric positive definite and is eliminated in lane order without a pivot
// search, one bound joins or leaves the working set per linear solve (monotone
// and finite for a strictly convex QP), the residual b - A x accumulated
// compensated (Dot2).  The working set starts from the previous step's (a row
// on a bound last step starts held there), so a steady contact state costs one
// linear solve per stage; PGS sweeps on the stage's box problem place the rows
// without a record (new contacts).  A semismooth Newton start (every bound
// change at once) was measured and dropped: on the standing humanoid's
// redundant foot corners (cond(A) ~1e7) its steps raise the residual by 1e4
// and fail their line search (scripts/proto_dantzig.py).
//
// within a budget of linear solves per world-step (both stages).  Converged =
// every row's complementarity residual (oracle lcp_residual, velocity units)
// within fp32 round-off of its own terms, in both stages.  A world that runs
// out of budget keeps iterates that never leave the boxes of their stage
// (x_n >= 0, box rows in [lo, hi], friction within +-mu x_n of the stage-1
// normal) and is counted.
#pragma once

namespace mw {
namespace dev {

// residual <= kLcpRelTol (|b| + sum |A_rc x_c|) + kLcpAbsTol: 16 fp32 ulps of
// the row's terms (the compensated residual is accurate to ~1 ulp; rounding x
// to fp32 moves it by ~1 ulp of mag).  At 4e-6 (r04c) a resting cube kept
// 1.5e-4 N of tangential force and a redundant corner could stay unloaded
// (its multiplier, set by DART's CFM, sat inside the tolerance).
#ifndef MW_LCP_REL_TOL
#define MW_LCP_REL_TOL 1e-6f  // A/B builds: EXTRA=-DMW_LCP_REL_TOL=...
#endif
constexpr float kLcpRelTol = MW_LCP_REL_TOL;
#ifndef MW_LCP_ABS_TOL
#define MW_LCP_ABS_TOL 1e-8f
#endif
constexpr float kLcpAbsTol = MW_LCP_ABS_TOL;   // m/s or rad/s
// a refinement solve that moves no impulse by more than this (relative to
// 1 + max |x|) has reached the fp32 floor of its working set
constexpr float kLcpStall = 1e-7f;
// at the floor a stage counts as converged when its residual is within this
// factor of the tolerance
constexpr float kLcpFloorAccept = 64.f;
// Which register widths solve on the matrix cores (bit 0: <= 16 rows, bit 1:
// <= 32, bit 2: <= 64; the rest eliminate over the lanes).  The choice is per
// kernel: the solve's tiles (16 / 48 accumulators) add to the kernel's peak
// register pressure, and the wave kernels sit at 512 registers with spills
// (A/B on the legs, gpurun_out r05d: humanoid_c5 131.8 -> 109.2 us with the
// 32-row tile, the scene 1.74 -> 1.10 ms with the 64-row tiles; the 64-row
// tiles in the wave kernels and any tile in the <= 16-body instance made
// their legs slower through the spills; once the wave kernels ran without
// scratch, every width in the <= 16-body instance measured faster:
// kWaveLcpMfmaSmall, wave_tree.hpp)
constexpr int kLcpMfma32 = 2, kLcpMfmaAll = 7;

// Wave reductions on DPP (no LDS round trip: a __shfl_xor butterfly is six
// ds_bpermute): row prefix by row_shr 1/2/4/8, then row_bcast 15 / 31 carry
// the row results up; lane 63 ends with the wave's result, read as a scalar.
// Every lane of the wave must be active.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ float dpp_f(float v) {
#ifdef MW_HOST_TEST
    return v;
#else
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, ROWMASK, 0xf, false));
#endif
}

__device__ __forceinline__ float wave_fmax(float v) {
    v = fmaxf(v, dpp_f<0x111, 0xf>(v));  // row_shr:1
    v = fmaxf(v, dpp_f<0x112, 0xf>(v));  // row_shr:2
    v = fmaxf(v, dpp_f<0x114, 0xf>(v));  // row_shr:4
    v = fmaxf(v, dpp_f<0x118, 0xf>(v));  // row_shr:8 -> lane 15 of a row holds its max
    v = fmaxf(v, dpp_f<0x142, 0xa>(v));  // row_bcast:15 into rows 1 and 3
    v = fmaxf(v, dpp_f<0x143, 0xc>(v));  // row_bcast:31 into rows 2 and 3
    return read_lane(v, 63);
}

__device__ __forceinline__ float wave_fmin(float v) {
    v = fminf(v, dpp_f<0x111, 0xf>(v));
    v = fminf(v, dpp_f<0x112, 0xf>(v));
    v = fminf(v, dpp_f<0x114, 0xf>(v));
    v = fminf(v, dpp_f<0x118, 0xf>(v));
    v = fminf(v, dpp_f<0x142, 0xa>(v));
    v = fminf(v, dpp_f<0x143, 0xc>(v));
    return read_lane(v, 63);
}

// bitwise OR over the wave (the same DPP steps)
template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint32_t dpp_u(uint32_t v) {
#ifdef MW_HOST_TEST
    return v;
#else
    return static_cast<uint32_t>(
        __builtin_amdgcn_update_dpp(static_cast<int>(v), static_cast<int>(v), CTRL, ROWMASK, 0xf, false));
#endif
}
__device__ __forceinline__ uint32_t wave_or32(uint32_t v) {
    v |= dpp_u<0x111, 0xf>(v);
    v |= dpp_u<0x112, 0xf>(v);
    v |= dpp_u<0x114, 0xf>(v);
    v |= dpp_u<0x118, 0xf>(v);
    v |= dpp_u<0x142, 0xa>(v);
    v |= dpp_u<0x143, 0xc>(v);
    return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 63));
}

// first lane holding the wave maximum of v
__device__ __forceinline__ int wave_argmax(float v) {
    const float m = wave_fmax(v);
    return __builtin_ctzll(static_cast<unsigned long long>(__ballot(v == m)));
}

// Orders one wave's LDS stores before its later loads as seen by the other
// lanes (a wavefront-scope release / acquire around the wave barrier): the
// compiler otherwise reasons per lane and may move a load of data another lane
// stores above that store.
__device__ __forceinline__ void wave_lds_sync() {
#ifndef MW_HOST_TEST
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#endif
}

__device__ __forceinline__ bool mask_bit(uint64_t m, int i) { return ((m >> i) & 1ull) != 0ull; }

// Row data of lane r (r < n): rhs b, kind, bounds of box rows, the contact's
// normal row for friction rows.
struct LcpRow {
    float b, lo, hi;
    int kind;   // 0 normal, 1 friction, 2 box (joint limit / servo / Coulomb)
    int nrow;   // friction: lane of its normal row; else the lane itself
    bool live;  // r < n
};

// w_r = sum_c A[r][c] x_c, compensated (Ogita-Rump-Oishi Dot2: the product
// error by an FMA, the sum error by TwoSum, both carried in c), and
// mag = sum_c |A[r][c] x_c| (the round-off scale of the residual test).  A
// plain fp32 sum errs by ~R eps mag, a sizeable share of the tolerance, so
// the last refinement solves would chase the matvec's own rounding.
template <int RC>
__device__ __forceinline__ float lcp_matvec(const float (&a)[kWaveMaxRows], float xl, int n, float& mag) {
#pragma clang fp contract(off)
    float w = 0.f, c = 0.f, m = 0.f;
#pragma unroll
    for (int k = 0; k < RC; ++k) {
        if ((k & 7) == 0 && k >= n) break;
        const float xk = read_lane(xl, k);
        const float p = a[k] * xk;
        const float pe = fmaf(a[k], xk, -p);
        const float t = w + p;
        const float z = t - w;
        c += ((w - (t - z)) + (p - z)) + pe;
        w = t;
        m += fabsf(p);
    }
    mag = m;
    return w + c;
}

// v of the row's contact normal (friction rows; every other row: its own v),
// by lane reads of the normal rows (every third row of the contact block)
template <int RC>
__device__ __forceinline__ float gather_normal(float v, const LcpRow& R, int n) {
    float out = v;
#pragma unroll
    for (int c = 0; c < RC; c += 3) {
        if (c >= n) break;
        const float vc = read_lane(v, c);
        out = (R.kind == 1 && R.nrow == c) ? vc : out;
    }
    return out;
}

// complementarity residual of a row with box [L, U] (oracle lcp_residual,
// velocity units), relative to its round-off scale: <= 1 is converged
__device__ __forceinline__ float lcp_row_residual(bool live, float b, float xl, float w, float mag, float arr, float L,
                                                  float U, float tolx, float& e_abs) {
    if (!live) {
        e_abs = 0.f;
        return 0.f;
    }
    const float s = b - w;
    float e;
    if (xl < L - tolx || xl > U + tolx)
        e = ((xl < L) ? (L - xl) : (xl - U)) * arr;
    else if (U - L <= tolx)
        e = 0.f;
    else if (xl <= L + tolx)
        e = fmaxf(s, 0.f);
    else if (xl >= U - tolx)
        e = fmaxf(-s, 0.f);
    else
        e = fabsf(s);
    e_abs = e;
    return e * rcp(kLcpRelTol * (fabsf(b) + mag) + kLcpAbsTol);
}

// Gaussian elimination with partial pivoting, lane = row: k[c] = K[lane][c],
// rhs = rhs[lane], rows / columns >= n are ignored.  Returns d[lane].
// Column j is eliminated at step j; the registers shift by one column per
// step (k[0] is always the current column), so no register is indexed at run
// time.  The pivot row of step j goes to LDS (U, kLcpUStride floats per row:
// the row's columns j.. at 0.., its rhs at kLcpRhs) and comes back to every
// lane as uniform-address ds_read_b128 (a broadcast: one read per 4 columns,
// where a v_readlane per column stalled the FMA on its SGPR); the rows stay
// there for the back substitution, where lane l gathers U[l][j - l]
// (stride - 1 odd: the 64 lanes hit 64 banks).  U: 16-byte aligned,
// kLcpUStride * 65 floats (a scratch row for the paired steps).
constexpr int kLcpUStride = 68;
constexpr int kLcpRhs = 64;
constexpr int kLcpScratchRow = 64;  // the unreduced second row of a paired step
constexpr int kLcpWorkFloats = 65 * kLcpUStride;  // the workspace the caller provides
// the second row of a paired step starts at this offset (its rhs at 0), so
// that its columns from j + 2 go out as aligned float4 stores
constexpr int kLcpBOff = 3;

// LongRows (the scene kernel's LCPs: up to 96 rows, 20-60 of them live)
// eliminates two columns per step (pivot = false: one LDS round trip and one
// dependent rcp chain per pair of rows; the same FMA sequence as two single
// steps, so the same bits), and each column loop stops at the live columns.
// Otherwise (the wave kernels' LCPs, <= 32 rows in the common case): single
// steps over the whole register row with no exit -- an exit from the unrolled
// loop costs a copy of the register row on every exit edge (the compiler's
// phi resolution), more than the dead columns' FMAs.  Measured on the legs
// (gpurun_out r04t / r04v): scene 1.965 (single, exits) -> 1.728 ms
// (LongRows) vs 1.886 (pairs without exits); humanoid_c5 132.6 (single,
// exits) -> 128.9 us (no exits) vs 141.7 (pairs without exits).

// pivot = false: the system is symmetric positive definite (the staggered
// rounds' principal submatrices A_FF, identity rows elsewhere), eliminated in
// lane order without the pivot search -- the argmax's DPP chain is most of an
// elimination step's dependent latency
//
// cols (pivot = false): the rows / columns that take part; row j outside it is
// an identity row whose column is zero in every other row (a held row of the
// active-set solve), so its step only shifts the registers and its d is 0.
// c - f * b as a three-address v_fma_f32: the elimination's register shift
// k[c] = k[c + 1] - f u[c + 1] then writes k[c]'s own register (the compiler's
// two-address v_fmac would land in k[c + 1]'s and add a v_mov per column to
// rotate the loop-carried registers back)
__device__ __forceinline__ float ge_fnma(float f, float b, float c) {
    float d;
    asm("v_fma_f32 %0, -%1, %2, %3" : "=v"(d) : "v"(f), "v"(b), "v"(c));
    return d;
}

template <int RC, bool LongRows = false>
__device__ __forceinline__ float lcp_ge_solve(float (&k)[RC], float rhs, int n, float* __restrict__ U, bool pivot,
                                              uint64_t cols = ~0ull) {
    static_assert(RC % 8 == 0, "row blocks of 8");
    const int lane = lane_id();
    if (pivot) cols = ~0ull;
    bool used = lane >= n;
    int boff = 0;  // offset of the lane's row in U (kLcpBOff: stored by a paired step)
    for (int j = 0; j < n; ++j) {
        const int left = n - j;  // live columns
        if (!mask_bit(cols, j)) {
#pragma unroll
            for (int c = 0; c < RC - 1; ++c) {
                if (LongRows && (c & 7) == 0 && c >= left) break;
                k[c] = k[c + 1];
            }
            continue;
        }
        if (LongRows && !pivot && j + 1 < n && mask_bit(cols, j + 1)) {
            // rows j (A) and j + 1 (S, unreduced) to LDS; every lane then
            // forms the reduced row B = S - g A (g = S0 / A0) on the fly and
            // takes both multiples: f1 = k0 / A0, f2 = (k1 - f1 A1) / B1.
            // Lane j + 1 takes f1 = g, f2 = 0, i.e. ends holding B from its
            // column 2, and stores it after the loop at the row offset kLcpBOff
            // (16-byte aligned stores; no LDS store inside the column loop,
            // which would serialise its loads)
            float* rowA = U + j * kLcpUStride;
            float* rowB = rowA + kLcpUStride;
            float* rowS = U + kLcpScratchRow * kLcpUStride;
            if (lane == j || lane == j + 1) {
                float* dst = (lane == j) ? rowA : rowS;
                float4* u = reinterpret_cast<float4*>(dst);
#pragma unroll
                for (int c = 0; c < RC; c += 4) {
                    if (LongRows && (c & 7) == 0 && c >= left) break;
                    u[c / 4] = make_float4(k[c], k[c + 1], k[c + 2], k[c + 3]);
                }
                dst[kLcpRhs] = rhs;
            }
            wave_lds_sync();
            const float4* ua = reinterpret_cast<const float4*>(rowA);
            const float4* us = reinterpret_cast<const float4*>(rowS);
            float4 a = ua[0], sv = us[0];
            const float arhs = rowA[kLcpRhs], srhs = rowS[kLcpRhs];
            const float pa = (fabsf(a.x) < 1e-30f) ? 1e-30f : a.x;
            const float g = sv.x * rcp(pa);
            const float b1 = fmaf(-g, a.y, sv.y);
            const float pb = (fabsf(b1) < 1e-30f) ? 1e-30f : b1;
            const float brhs = fmaf(-g, arhs, srhs);
            const bool wb = lane == j + 1;
            const bool act = !(used || lane == j || wb);
            const float f1 = act ? k[0] * rcp(pa) : (wb ? g : 0.f);
            const float f2 = act ? fmaf(-f1, a.y, k[1]) * rcp(pb) : 0.f;
#pragma unroll
            for (int c = 0; c < RC; c += 4) {
                if (LongRows && (c & 7) == 0 && c >= left) break;
                const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
                const float4 an = (c + 4 < RC) ? ua[c / 4 + 1] : z;
                const float4 sn = (c + 4 < RC) ? us[c / 4 + 1] : z;
                // B at columns c + 2 .. c + 5
                const float e0 = fmaf(-g, a.z, sv.z), e1 = fmaf(-g, a.w, sv.w);
                const float e2 = fmaf(-g, an.x, sn.x), e3 = fmaf(-g, an.y, sn.y);
                k[c] = ge_fnma(f2, e0, ge_fnma(f1, a.z, k[c + 2]));
                k[c + 1] = ge_fnma(f2, e1, ge_fnma(f1, a.w, k[c + 3]));
                if (c + 4 < RC) {
                    k[c + 2] = ge_fnma(f2, e2, ge_fnma(f1, an.x, k[c + 4]));
                    k[c + 3] = ge_fnma(f2, e3, ge_fnma(f1, an.y, k[c + 5]));
                }
                a = an;
                sv = sn;
            }
            rhs = fmaf(-f2, brhs, fmaf(-f1, arhs, rhs));
            if (wb) {
                // row j + 1 from its pivot B1: rhs at 0, B1 at kLcpBOff, columns
                // j + 2 .. at kLcpBOff + 1 ..
                float4* u = reinterpret_cast<float4*>(rowB + kLcpBOff + 1);
#pragma unroll
                for (int c = 0; c < RC; c += 4) {
                    if (LongRows && (c & 7) == 0 && c + 2 >= left) break;
                    u[c / 4] = make_float4(k[c], k[c + 1], k[c + 2], k[c + 3]);
                }
                rowB[kLcpBOff] = b1;
                rowB[0] = rhs;
                boff = kLcpBOff;
            }
            used = used || lane == j || wb;
            ++j;
            continue;
        }
        const int p = pivot ? wave_argmax(used ? -1.f : fabsf(k[0])) : j;
        float* row = U + j * kLcpUStride;
        if (lane == p) {
            float4* u = reinterpret_cast<float4*>(row);
#pragma unroll
            for (int c = 0; c < RC; c += 4) {
                if (LongRows && (c & 7) == 0 && c >= left) break;
                u[c / 4] = make_float4(k[c], k[c + 1], k[c + 2], k[c + 3]);
            }
            row[kLcpRhs] = rhs;
        }
        // lane p's row is read by the other lanes: without the fence the
        // compiler forwards lane p's own values and hoists the other lanes'
        // loads into the store's else-branch, which runs first
        wave_lds_sync();
        // the pivot row back to every lane, 4 columns per read, as the update
        // walks the columns (one wave: its LDS accesses are in order; the
        // columns >= left are dead)
        const float4* ur = reinterpret_cast<const float4*>(row);
        float4 cur = ur[0];
        const float prhs = row[kLcpRhs];
        const float piv = (fabsf(cur.x) < 1e-30f) ? 1e-30f : cur.x;
        const float f = (used || lane == p) ? 0.f : k[0] * rcp(piv);
#pragma unroll
        for (int c = 0; c < RC; c += 4) {
            if (LongRows && (c & 7) == 0 && c >= left) break;
            const float4 nxt = (c + 4 < RC) ? ur[c / 4 + 1] : make_float4(0.f, 0.f, 0.f, 0.f);
            k[c] = ge_fnma(f, cur.y, k[c + 1]);
            k[c + 1] = ge_fnma(f, cur.z, k[c + 2]);
            k[c + 2] = ge_fnma(f, cur.w, k[c + 3]);
            if (c + 4 < RC) k[c + 3] = ge_fnma(f, nxt.x, k[c + 4]);
            cur = nxt;
        }
        rhs = fmaf(-f, prhs, rhs);
        used = used || lane == p;
    }
    // back substitution, right-looking: lane l holds row l (pivot of step l)
    wave_lds_sync();
    float acc = 0.f, rdiag = 1.f;
    if (lane < n && mask_bit(cols, lane)) {
        acc = U[lane * kLcpUStride + (boff ? 0 : kLcpRhs)];
        float dg = U[lane * kLcpUStride + boff];
        dg = (fabsf(dg) < 1e-30f) ? 1e-30f : dg;
        rdiag = rcp(dg);
    }
    float dl = 0.f;
    for (int j = n - 1; j >= 0; --j) {
        if (!mask_bit(cols, j)) continue;
        const float dj = read_lane(acc * rdiag, j);
        dl = (lane == j) ? dj : dl;
        if (lane < j) acc = fmaf(-U[lane * (kLcpUStride - 1) + boff + j], dj, acc);
    }
    return dl;
}

// ---- the active-set method's linear solve on the matrix cores ------------------
// S d = rhs over the free rows (freeM; a held or dead row is an identity row and
// column, rhs 0, d 0), S = the Delassus registers a[] (lane c: a[r] = A[r][c]),
// symmetric positive definite on the free rows (DART's CFM).  Block LDL^T with
// 2x2 pivot blocks and no pivot search (SPD), right-looking: every block step
// is ONE v_mfma_f32_32x32x2_f32 per 32x32 tile -- the rank-2 update
// S -= P D^-1 P^T of the trailing matrix, P = the two pivot columns, with
// fp32 operands and fp32 accumulation (exact f32 FMAs on gfx950) -- instead of
// two elimination steps of lcp_ge_solve (an LDS round trip and ~32 FMAs
// each).  The tiles live in the MFMA accumulator layout: lane l holds column
// l % 32, rows 8 (i / 4) + 4 (l / 32) + i % 4 in accumulator i, so row j of a
// tile -- by symmetry its column j, the pivot panel -- is accumulator
// 4 (j / 8) + j % 4 of one lane half, and one v_permlane32_swap turns it into
// the MFMA's A operand (lane l: P[l % 32][l / 32]).  R <= 32: tile T00;
// R <= 64: the upper tiles T00, T01, T11 (T10 = T01^T is not kept).  Block
// steps whose two rows are both held are skipped (stage 1 holds every
// friction row).  The forward substitution rides along (rhs in lane = row),
// the L columns go to LDS (Lw, column-major, stride 65: the back substitution's
// lane c reads row j of column c conflict-free), D^-1 is applied per 2x2
// block, then the back substitution by lane reads of d.
constexpr int kLcpLStride = 65;
constexpr int kLcpMfmaWorkFloats = 64 * kLcpLStride;

// x's lanes 32..63 <-> y's lanes 0..31 (v_permlane32_swap_b32)
__device__ __forceinline__ void lane_swap32(float& x, float& y) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(y), false, false);
    x = __uint_as_float(r[0]);
    y = __uint_as_float(r[1]);
}
// the value of lane l ^ 32
__device__ __forceinline__ float lane_xor32(float v) {
    float lo = v, hi = v;
    lane_swap32(lo, hi);  // lo = [v_lo, v_lo], hi = [v_hi, v_hi]
    return (lane_id() >= 32) ? lo : hi;
}

// The pivot block of rows / columns J, J + 1 of tile T, eliminated by two 1x1
// pivots (d0 = s00, l = s01 / s00, d1 = s11 - l s01: the elimination's own
// arithmetic -- an explicit 2x2 inverse through ac - b^2 cancels on the
// redundant contact rows, cond(A) ~1e7, and is not backward stable); uniform.
template <int J>
__device__ __forceinline__ void mfma_pivot(const v16f& T, float& i0, float& l, float& i1) {
    constexpr int i = 4 * (J / 8) + (J % 4), hl = 32 * ((J / 4) % 2);
    const float s00 = read_lane(T[i], J + hl), s01 = read_lane(T[i], J + 1 + hl);
    const float s11 = read_lane(T[i + 1], J + 1 + hl);
    // a zero pivot (two identical joint rows: DART's joint CFM, 1e-9, is below
    // fp32's resolution) takes the elimination's guard (lcp_ge_solve): its
    // column is exactly zero, the row's unknown grows large and the active-set
    // step's blocking bound resolves the degenerate pair
    i0 = rcp((fabsf(s00) < 1e-30f) ? 1e-30f : s00);
    l = s01 * i0;
    const float d1 = fmaf(-l, s01, s11);
    i1 = rcp((fabsf(d1) < 1e-30f) ? 1e-30f : d1);
}
// this lane's panel entry P[lane % 32][J + lane / 32] of tile T
template <int J>
__device__ __forceinline__ float mfma_panel(const v16f& T) {
    constexpr int i = 4 * (J / 8) + (J % 4);
    float x = T[i], y = T[i + 1];
    lane_swap32(x, y);
    return ((J / 4) % 2) ? y : x;
}

// LS: the column stride of the L record in Lw (column-major, L[row][col] at
// Lw[col * LS + row]; only rows < LROWS are stored).
template <int RC, int LS = kLcpLStride, int LROWS = 64>
struct MfmaLdl {
    v16f T00, T01, T11;
    float r, y;
    uint64_t freeM;
    float* Lw;

    __device__ __forceinline__ void put_l(int row, int col, float v) const {
        if (LROWS >= 64 || row < LROWS) Lw[col * LS + row] = v;
    }

    // block step of rows / columns J, J + 1: the two eliminated columns
    // Q = [p0, p1 - l p0] (the second one reduced by the first), one MFMA
    // per tile for S -= Q diag(1/d0, 1/d1) Q^T, and the forward substitution
    template <int J>
    __device__ __forceinline__ void step() {
        if (((freeM >> J) & 3ull) == 0ull) return;  // two held rows: identity, nothing to do
        const int lane = lane_id();
        const int c = lane & 31;
        const bool hi = lane >= 32;
        constexpr int JT = J % 32;
        float i0, l, i1, mine, mineb = 0.f, othb = 0.f;
        if constexpr (J < 32) {
            mfma_pivot<JT>(T00, i0, l, i1);
            mine = mfma_panel<JT>(T00);
            if constexpr (RC == 64) {
                mineb = mfma_panel<JT>(T01);
                othb = lane_xor32(mineb);
            }
        } else {
            mfma_pivot<JT>(T11, i0, l, i1);
            mine = mfma_panel<JT>(T11);
        }
        const float oth = lane_xor32(mine);
        // Q[c][h] of this lane (top panel: rows c; J >= 32: rows 32 + c)
        const float p0 = hi ? oth : mine, p1 = hi ? mine : oth;
        const float q = hi ? fmaf(-l, p0, p1) : p0;
        const float ih = hi ? i1 : i0;
        const float Lm = q * ih;  // L[c][J + h]
        const int col = J + (hi ? 1 : 0);
        float r0 = p0, r1 = fmaf(-l, p0, p1);  // this lane's ROW of Q (lane = row)
        if constexpr (J < 32) {
            T00 = __builtin_amdgcn_mfma_f32_32x32x2f32(-q, Lm, T00, 0, 0, 0);
            put_l(c, col, Lm);
            if constexpr (RC == 64) {
                const float b0 = hi ? othb : mineb, b1 = hi ? mineb : othb;
                const float qb = hi ? fmaf(-l, b0, b1) : b0;
                const float Lb = qb * ih;
                T01 = __builtin_amdgcn_mfma_f32_32x32x2f32(-q, Lb, T01, 0, 0, 0);
                T11 = __builtin_amdgcn_mfma_f32_32x32x2f32(-qb, Lb, T11, 0, 0, 0);
                put_l(32 + c, col, Lb);
                if (hi) {  // rows 32 + c come from the bottom panel
                    r0 = b0;
                    r1 = fmaf(-l, b0, b1);
                }
            }
        } else {
            T11 = __builtin_amdgcn_mfma_f32_32x32x2f32(-q, Lm, T11, 0, 0, 0);
            put_l(32 + c, col, Lm);
        }
        // forward substitution, lane = row, one column after the other
        // (selects, not branches: a divergent branch here made the compiler
        // copy whole accumulator tiles out of the AGPRs at every step)
        const float z0 = read_lane(r, J);
        const float ra = fmaf(-(r0 * i0), z0, r);
        r = (lane > J) ? ra : r;  // row J + 1 takes l z0
        const float z1 = read_lane(r, J + 1);
        const float rb = fmaf(-(r1 * i1), z1, r);
        r = (lane > J + 1) ? rb : r;
        y = (lane == J) ? z0 * i0 : y;
        y = (lane == J + 1) ? z1 * i1 : y;
    }
    template <int J>
    __device__ __forceinline__ void forward() {
        step<J>();
        if constexpr (J + 2 < RC) forward<J + 2>();
    }
};

// back substitution L^T d = y (lane = row, y in and d out) over the pairs of
// freeM, from the last: row J + 1, then row J; lane c reads column c of L
// (L[J][c] at Lw[c * LS + J])
template <int J, int LS = kLcpLStride>
__device__ __forceinline__ void ldl_backward(float& y, uint64_t freeM, const float* __restrict__ Lw) {
    if (((freeM >> J) & 3ull) != 0ull) {
        const int lane = lane_id();
        const float* col = Lw + lane * LS;
        const float dj1 = read_lane(y, J + 1);
        const float ya = fmaf(-col[J + 1], dj1, y);
        y = (lane <= J) ? ya : y;  // lane J: the pair's own l
        const float dj = read_lane(y, J);
        const float yb = fmaf(-col[J], dj, y);
        y = (lane < J) ? yb : y;
    }
    if constexpr (J >= 2) ldl_backward<J - 2, LS>(y, freeM, Lw);
}

template <int RC>
__device__ __forceinline__ float lcp_mfma_solve(const float (&a)[kWaveMaxRows], float rhs, uint64_t freeM,
                                                float* __restrict__ Lw) {
    static_assert(RC == 32 || RC == 64, "one or two tile rows");
    const int lane = lane_id();
    const int c = lane & 31;
    const bool hi = lane >= 32;
    MfmaLdl<RC> M;
    M.freeM = freeM;
    M.Lw = Lw;
    M.T01 = v16f{};
    M.T11 = v16f{};
    // ---- the masked tiles: free x free entries of A, identity elsewhere
    const bool cf0 = mask_bit(freeM, c), cf1 = mask_bit(freeM, 32 + c);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int r0 = 8 * (i / 4) + (i % 4), r1 = r0 + 4;
        const int rr = hi ? r1 : r0;  // this lane's row of accumulator i
        const bool rf = hi ? mask_bit(freeM, r1) : mask_bit(freeM, r0);
        float x = a[r0], y = a[r1];
        lane_swap32(x, y);  // x: A[rr][c] (T00), y: A[rr][32 + c] (T01)
        M.T00[i] = (rf && cf0) ? x : ((rr == c) ? 1.f : 0.f);
        if constexpr (RC == 64) {
            M.T01[i] = (rf && cf1) ? y : 0.f;
            const bool rf1 = hi ? mask_bit(freeM, 32 + r1) : mask_bit(freeM, 32 + r0);
            float u = a[32 + r0], v = a[32 + r1];
            lane_swap32(u, v);  // v: A[32 + rr][32 + c]
            M.T11[i] = (rf1 && cf1) ? v : ((rr == c) ? 1.f : 0.f);
        }
    }
    // rhs of a held / dead row is 0 (its d is 0)
    M.r = mask_bit(freeM, lane) ? rhs : 0.f;
    M.y = 0.f;
    M.template forward<0>();
    wave_lds_sync();
    ldl_backward<RC - 2>(M.y, freeM, Lw);
    return mask_bit(freeM, lane) ? M.y : 0.f;
}

// One strictly convex box QP  min 1/2 x'Ax - b'x,  L <= x <= U  (bounds fixed,
// per lane; a dead or pinned row has L = U) by the primal active-set method
// from x (inside the box): the working set starts as ws0 (1 held at L, 2 held
// at U, 0 free; -1: the start point's own -- at a bound or not), the held rows
// sit on their bound, every linear solve minimises over the free rows (A_FF is
// symmetric positive definite: no pivot search, the held rows' steps skipped)
// and takes the longest step that stays in the box; the first bound met joins
// the working set (every bound met, when the step has zero length); at the
// working set's minimiser every held row whose
// multiplier is wrongly signed beyond its own tolerance (the scale the
// residual test uses) leaves it -- several at once: contacts that barely
// touch (approach velocities of 1e-7 m/s in a settling stack) would each
// cost a solve one at a time (scripts/proto_dantzig.py MULTI).  If none is and the residual
// still misses the tolerance, what remains is the fp32 solve's own error: one
// more solve on the same working set from the compensated residual refines it
// (iterative refinement), until a refinement moves nothing (kLcpStall: the
// fp32 floor; converged if within kLcpFloorAccept of the tolerance).  solves
// counts the linear solves against `budget`.  Termination: a step of nonzero
// length lowers the objective; zero-length steps only add rows to the working
// set; a release that cannot move its rows freezes them (below), and after a
// blocked multi-release rows leave singly until the next full step.
// Returns true when every row's residual is within tolerance.
template <int RC, bool LongRows = false, int MFMA = kLcpMfma32>
__device__ __forceinline__ bool wave_boxqp(const float (&a)[kWaveMaxRows], bool live, float b, float L, float U,
                                           float arr, int n, int budget, float* __restrict__ Uw, float& xl, int ws0,
                                           int& solves, int& iters, long long& ge_cycles) {
    const int lane = lane_id();
    const bool pinned = !live || U - L <= 0.f;
    int ws;
    {
        const float t0 = 2e-6f * (1.f + wave_fmax(live ? fabsf(xl) : 0.f));
        const int own = (xl <= L + t0) ? 1 : ((xl >= U - t0) ? 2 : 0);
        ws = pinned ? 1 : ((ws0 < 0) ? own : ws0);
        xl = (ws == 1) ? L : ((ws == 2) ? U : xl);
        xl = live ? xl : 0.f;
    }
    // the last step reached the working set's minimiser (a working set with
    // no free row is its own minimiser: no solve)
    bool at_min = __ballot(!pinned && ws == 0) == 0ull;
    bool stalled = false; // ... by a refinement solve that moved nothing
    bool fresh = false;   // w / g / mag / xmax / rel belong to the current x
    bool single = false;  // release one row at a time (after a blocked multi-release, until the next full step)
    uint64_t released = 0ull;  // the rows of the last release
    // rows whose release could not move them: the solve on the grown free set
    // moved nothing, or turned the one released row straight back out of its
    // box.  In exact arithmetic a released row with a wrongly signed
    // multiplier always moves inward (d_r = -(A_FF^-1)_rr g_r); here its
    // multiplier is below the fp32 solve's resolution.  Frozen rows stay on
    // their bound for the rest of this call (their residual still counts):
    // without this a pair of such rows cycled release / block until the
    // budget (scene dumps, scripts/lcp_dump_check.py).
    uint64_t frozen = 0ull;
    float w = 0.f, g = 0.f, mag = 0.f, xmax = 0.f, rel = 0.f;
    float rel_refine = 3.4e38f;  // the residual when the last refinement solve started
    for (int it = 0; it < 4 * budget + 8 + n; ++it, ++iters) {
        if (!fresh) {
            w = lcp_matvec<RC>(a, xl, n, mag);
            g = w - b;
            xmax = wave_fmax(live ? fabsf(xl) : 0.f);
            float e_abs;
            rel = wave_fmax(lcp_row_residual(live, b, xl, w, mag, arr, L, U, 2e-6f * (1.f + xmax), e_abs));
            if (rel <= 1.f) return true;
            fresh = true;
        }
        if (at_min) {
            at_min = false;
            float v = (ws == 1) ? -g : ((ws == 2) ? g : 0.f);
            v = (pinned || mask_bit(frozen, lane)) ? 0.f : v * rcp(kLcpRelTol * (fabsf(b) + mag) + kLcpAbsTol);
            // every held row whose multiplier is wrongly signed beyond its
            // tolerance leaves at once (one solve for several micro-contacts).
            // Each step stays in the box and does not raise the objective, but
            // with several rows released a released row can block the next
            // step at zero length and rejoin; once that happens the rows leave
            // one at a time, the most violated first (the textbook primal
            // active-set rule, finite for a strictly convex QP).
            const float vmax = wave_fmax(v);
            if (vmax > 1.f) {
                bool rel_me = v > 1.f;
                if (single) rel_me = lane == __builtin_ctzll(static_cast<unsigned long long>(__ballot(v == vmax)));
                if (rel_me) ws = 0;
                released = __ballot(rel_me);
                stalled = false;
                continue;
            }
            // every multiplier is signed right and the last solve on this
            // working set was a refinement that moved nothing, or did not
            // halve the residual (the elimination's own error at the
            // system's conditioning): the fp32 floor
            if (stalled || rel > 0.5f * rel_refine) return rel <= kLcpFloorAccept;
            rel_refine = rel;
        } else {
            rel_refine = 3.4e38f;
        }
        if (solves >= budget) return false;
        // ---- one linear solve over the free rows
        const bool fr = !pinned && ws == 0;
        const uint64_t freeM = __ballot(fr);
#ifdef MW_WAVE_PROF
        const long long tg0 = clock64();
#endif
        // block LDL^T on the matrix cores (R <= 32: one tile, else three) for
        // the widths the kernel's MFMA policy selects
        float d;
        constexpr int bit = (RC <= 16) ? 1 : ((RC <= 32) ? 2 : 4);
        if constexpr ((MFMA & bit) == 0) {
            float k[RC];
#pragma unroll
            for (int c = 0; c < RC; ++c) k[c] = (fr && mask_bit(freeM, c)) ? a[c] : ((!fr && c == lane) ? 1.f : 0.f);
            d = lcp_ge_solve<RC, LongRows>(k, fr ? -g : 0.f, n, Uw, false, freeM);
        } else {
            d = lcp_mfma_solve<(RC <= 32) ? 32 : 64>(a, fr ? -g : 0.f, freeM, Uw);
        }
#ifdef MW_WAVE_PROF
        ge_cycles += clock64() - tg0;
#else
        (void)ge_cycles;
#endif
        ++solves;
        // the longest feasible step along d (at most 1)
        // ... moves nothing: no impulse by more than kLcpStall (relative to
        // 1 + max |x|) and no row's own residual (d_r A_rr) by more than its
        // tolerance.  The second test keeps steps that are tiny in x but not
        // for their row: a joint-limit row (A_rr ~ 136 on the humanoid, b ~
        // 1e-5) needed x = -9e-8 and counted unconverged at the floor (the 8
        // unconverged world-steps of the humanoid leg, scripts/lcp_dump_check.py)
        const float dmax = wave_fmax(fr ? fabsf(d) : 0.f);
        const float dres = wave_fmax(fr ? fabsf(d) * arr * rcp(kLcpRelTol * (fabsf(b) + mag) + kLcpAbsTol) : 0.f);
        if (dmax <= kLcpStall * (1.f + xmax) && dres <= 1.f) {
            if (released) {  // the release moved nothing: back to the bounds, frozen
                if (mask_bit(released, lane)) ws = (xl <= L) ? 1 : 2;
                frozen |= released;
                released = 0ull;
            }
            at_min = true;
            stalled = true;
            continue;
        }
        stalled = false;
        fresh = false;
        float al = 1.f;
        int side = 0;
        if (fr && d < 0.f && xl + d < L) { al = (L - xl) * rcp(d); side = 1; }
        else if (fr && d > 0.f && xl + d > U) { al = (U - xl) * rcp(d); side = 2; }
        al = fmaxf(al, 0.f);
        const float amin = wave_fmin(al);
        if (amin < 1.f) {
            const int block = wave_argmax(-al);
            const int bside = __builtin_amdgcn_readlane(side, block);
            // a row of a multi-row release blocks at once: release singly
            // until the next full step; a single released row that blocks at
            // once is frozen, and the working set is the one before the
            // release, at its minimiser
            bool back = false;
            if (amin <= 0.f && mask_bit(released, block)) {
                if (__builtin_popcountll(released) > 1) {
                    single = true;
                } else {
                    frozen |= released;
                    back = true;
                }
            }
            released = 0ull;
            xl = fr ? xl + amin * d : xl;
            if (lane == block) {
                xl = (bside == 1) ? L : U;
                ws = bside;
            }
            // a zero-length step: every row it blocks joins its bound now
            // (x does not move, so each would block the next solve at zero
            // length, one solve per row: warm starts whose friction boxes
            // shrank)
            if (amin <= 0.f && fr && side != 0 && al <= 0.f) {
                xl = (side == 1) ? L : U;
                ws = side;
            }
            at_min = back;
        } else {
            xl = fr ? xl + d : xl;
            at_min = true;
            released = 0ull;
            single = false;
        }
    }
    return false;
}

// Projected Gauss-Seidel sweeps on a box problem with fixed per-row bounds
// (the starting point of a stage's exact solve): row constants {b, 1/A_rr,
// L, U} through the LDS array rc (lane r writes row r; rows >= n inert),
// impulses uniform in registers, the residual w_c = (A x)_c distributed over
// the lanes and updated by one column per row (wave_step's PGS without the
// friction coupling).  Ends once a sweep moves no constraint velocity by more
// than tol.  x: lane r's impulse, in and out.
template <int RC>
__device__ __forceinline__ void wave_pgs_box(const float (&a)[kWaveMaxRows], F4* __restrict__ rc, bool live, float b,
                                             float arr, float L, float U, int n, int sweeps, float tol, float& xl) {
    const int lane = lane_id();
    const int npad = (n + 7) & ~7;
    if (lane < npad) rc[lane] = live ? F4{b, rcp(arr), L, U} : F4{0.f, 0.f, 0.f, 0.f};
    wave_lds_sync();
    float xu[RC];
#pragma unroll
    for (int r = 0; r < RC; ++r) xu[r] = read_lane(xl, r);
    for (int it = 0; it < sweeps; ++it) {
        float w = 0.f;
#pragma unroll
        for (int rb = 0; rb < RC; rb += 8) {
            if (rb >= npad) break;
#pragma unroll
            for (int k = 0; k < 8; ++k) w += a[rb + k] * xu[rb + k];
        }
        const float w_start = w;
#pragma unroll
        for (int rb = 0; rb < RC; rb += 8) {
            if (rb >= npad) break;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int r = rb + k;
                const F4 c = rc[r];
                const float xb = fmaf(c.x, c.y, xu[r]);
                const float wpre = fmaf(-a[r], xu[r], w);
                const float v = clamp_ordered(fmaf(-read_lane(w, r), c.y, xb), c.z, c.w);
                w = fmaf(a[r], v, wpre);
                xu[r] = v;
            }
        }
        if (wave_fmax(fabsf(w - w_start)) <= tol) break;
    }
    float xo = xl;
#pragma unroll
    for (int r = 0; r < RC; ++r) xo = (lane == r) ? xu[r] : xo;
    xl = live ? xo : 0.f;
}

// The exact solve, DART's two stages (header).  x1: lane r's stage-1 impulse
// of the previous step, returned as this step's stage-1 solution; xl: the
// previous step's final impulse, returned solved.  Each stage starts from the
// previous step's impulse of the stage (projected onto this step's boxes),
// runs up to min(sweeps, kLcpStageSweeps) PGS sweeps on the stage's box
// problem (tolerance exit pgs_tol; rc: the LDS row-constant array they use),
// then the active-set method from the previous step's working set: a row that
// sat on a bound of its stage's box last step starts held there; a row with a
// zero impulse last step (no record: a new contact, or a friction row of a
// contact without normal force) takes the class of the PGS point.  At a
// steady contact state that is one linear solve per stage.  a: the Delassus
// registers (a[c] = A[lane][c], CFM included).  Returns true when both stages
// converged within max_solves linear solves in total; n_solves / n_rounds /
// n_solves2: linear solves, iterations, linear solves of stage 2.
// (prototype, standing humanoid / drops: 12 -> 4 sweeps costs +0.09 linear
// solves per world-step and saves two thirds of the sweeps)
#ifndef MW_LCP_STAGE_SWEEPS
#define MW_LCP_STAGE_SWEEPS 4
#endif
constexpr int kLcpStageSweeps = MW_LCP_STAGE_SWEEPS;

// STAGE_SWEEPS: the cap on the sweeps per stage (the scene kernel's
// three-cube stacks converge more often with 6: 3253 -> 2575 unconverged
// world-steps, 1.757 -> 1.708 ms, profiles/r04z ab_sweeps)
template <int RC, bool LongRows = false, int STAGE_SWEEPS = kLcpStageSweeps, int MFMA = kLcpMfma32>
__device__ __forceinline__ bool wave_lcp_exact(const float (&a)[kWaveMaxRows], const LcpRow& R, float mu, int n,
                                               int max_solves, int sweeps, float pgs_tol, F4* __restrict__ rc,
                                               float* __restrict__ Uw, float& x1, float& xl, int& n_solves,
                                               int& n_rounds, int& n_solves2, long long (&cyc)[3]) {
    // cyc (MW_WAVE_PROF builds): [0] cycles in the linear solves, [1] in the
    // PGS sweeps, [2] in stage 1
    long long& ge_cycles = cyc[0];
#ifdef MW_WAVE_PROF
    const long long tc0 = clock64();
#endif
    const int lane = lane_id();
    float arr = 1.f;  // A_rr (a dynamic register index would go to scratch)
#pragma unroll
    for (int c = 0; c < RC; ++c) arr = (lane == c && R.live) ? a[c] : arr;
    sweeps = sweeps < STAGE_SWEEPS ? sweeps : STAGE_SWEEPS;
    int solves = 0, iters = 0;
    const bool fric = R.kind == 1;
    const float x1p = R.live ? x1 : 0.f, xlp = R.live ? xl : 0.f;  // the previous step's
    // stage 1: normal and joint rows; friction impulses pinned at 0
    const float L1 = (fric || !R.live) ? 0.f : R.lo;
    const float U1 = (fric || !R.live) ? 0.f : R.hi;
    int ws;
    {
        const float t = 2e-6f * (1.f + wave_fmax(fabsf(x1p)));
        ws = (x1p == 0.f) ? -1 : ((x1p <= L1 + t) ? 1 : ((x1p >= U1 - t) ? 2 : 0));
    }
    float x = fminf(fmaxf(x1p, L1), U1);
#ifdef MW_WAVE_PROF
    long long tp = clock64();
#endif
    if (sweeps > 0) wave_pgs_box<RC>(a, rc, R.live, R.b, arr, L1, U1, n, sweeps, pgs_tol, x);
#ifdef MW_WAVE_PROF
    cyc[1] += clock64() - tp;
#endif
    const bool ok1 = wave_boxqp<RC, LongRows, MFMA>(a, R.live, R.b, L1, U1, arr, n, max_solves, Uw, x, ws, solves, iters, ge_cycles);
    x1 = R.live ? x : 0.f;
#ifdef MW_WAVE_PROF
    cyc[2] += clock64() - tc0;
#endif
    const int s1 = solves;
    // stage 2: each friction row boxed by mu x_n of its contact's stage-1
    // normal; the previous step's boxes from its own stage-1 normals
    const float xn1 = gather_normal<RC>(x, R, n);
    const float xn1p = gather_normal<RC>(x1p, R, n);
    float L = L1, U = U1, Lp = L1, Up = U1;
    if (fric && R.live) {
        U = mu * fmaxf(xn1, 0.f);
        L = -U;
        Up = mu * fmaxf(xn1p, 0.f);
        Lp = -Up;
    }
    {
        const float t = 2e-6f * (1.f + wave_fmax(fabsf(xlp)));
        ws = (xlp == 0.f || Up - Lp <= 0.f) ? -1 : ((xlp <= Lp + t) ? 1 : ((xlp >= Up - t) ? 2 : 0));
    }
    x = fminf(fmaxf(xlp, L), U);
#ifdef MW_WAVE_PROF
    tp = clock64();
#endif
    if (sweeps > 0) wave_pgs_box<RC>(a, rc, R.live, R.b, arr, L, U, n, sweeps, pgs_tol, x);
#ifdef MW_WAVE_PROF
    cyc[1] += clock64() - tp;
#endif
    const bool ok2 = wave_boxqp<RC, LongRows, MFMA>(a, R.live, R.b, L, U, arr, n, max_solves, Uw, x, ws, solves, iters, ge_cycles);
    xl = R.live ? x : 0.f;
    n_solves = solves;
    n_rounds = iters;
    n_solves2 = solves - s1;
    return ok1 && ok2;
}

}  // namespace dev
}  // namespace mw
