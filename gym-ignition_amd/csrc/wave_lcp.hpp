// wave_lcp.hpp -- exact solve of the world-per-wavefront kernel's boxed LCP
// (contact normal rows x_n >= 0, friction rows |x_t| <= mu x_n, joint rows in
// [lo, hi]), the problem DART's primary boxed-LCP solver (Dantzig pivoting,
// BoxedLcpConstraintSolver [EXT], reached from ForwardStep at
// /root/reference/cpp/scenario/plugins/Physics/Physics.cpp:1824-1835) solves
// exactly.  Specification: oracle.c lcp_refine / boxqp_solve (the fixed point
// of the friction boxes with the box QP of every round solved exactly).
//
// Lane r owns row r: its Delassus row a[c] = A[r][c] (the PGS registers of
// wave_step), its impulse x_r and its row data.  After the PGS sweeps:
//
//   1. semismooth Newton rounds on the coupled conditions: a row is held at
//      a bound when its gradient g = A x - b pushes it outward, a friction row
//      held at +-mu x_n moves with its normal (d_t = +-mu d_n), every other
//      row is free; the Newton system (free rows, coupled columns folded into
//      their normal's column) is solved by Gaussian elimination with partial
//      pivoting over the lanes; the step is accepted only when it lowers the
//      largest complementarity residual (halved up to 3 times);
//   2. if a round fails, the oracle's own method: friction boxes frozen at the
//      current normals, the box QP solved by the primal active-set method
//      (one bound joins or leaves the working set per step), the boxes
//      updated, until they stop moving;
//
// within a budget of linear solves per step.  Converged = every row's
// complementarity residual (oracle lcp_residual, velocity units) within fp32
// round-off of its own terms.  A world that runs out of budget keeps its
// current impulses projected onto the boxes of its current normals (feasible:
// x_n >= 0, |x_t| <= mu x_n, box rows in [lo, hi]) and is counted.
#pragma once

namespace mw {
namespace dev {

constexpr float kLcpRelTol = 4e-6f;   // residual <= kLcpRelTol (|b| + sum |A_rc x_c|) + kLcpAbsTol
constexpr float kLcpAbsTol = 1e-7f;   // m/s or rad/s
constexpr int kLcpLineSearch = 3;     // step halvings of a Newton round
// A residual within kLcpLoose x the tolerance is accepted after one more
// linear solve (the polish round) whatever that round reaches: the last
// decade costs the redundant-corner standing LCPs (conditioned ~1e7 by the
// CFM) many active-set rounds, while the joint velocities follow the
// residual / sqrt(CFM) and want the tight tolerance after impacts
constexpr float kLcpLoose = 10.f;

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

// w_r = sum_c A[r][c] x_c and mag = sum_c |A[r][c] x_c| (round-off scale)
template <int RC>
__device__ __forceinline__ float lcp_matvec(const float (&a)[kWaveMaxRows], float xl, int n, float& mag) {
    float w = 0.f, m = 0.f;
#pragma unroll
    for (int c = 0; c < RC; ++c) {
        if ((c & 7) == 0 && c >= n) break;
        const float t = a[c] * read_lane(xl, c);
        w += t;
        m += fabsf(t);
    }
    mag = m;
    return w;
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

// box of row r at the lane-distributed impulses xl (friction: [-mu x_n, mu x_n])
template <int RC>
__device__ __forceinline__ void lcp_bounds(const LcpRow& R, float xl, float mu, int n, float& L, float& U) {
    const float xn = gather_normal<RC>(xl, R, n);
    const float u = mu * fmaxf(xn, 0.f);
    L = (R.kind == 1) ? -u : R.lo;
    U = (R.kind == 1) ? u : R.hi;
}

// complementarity residual of row r (oracle lcp_residual, velocity units),
// relative to its round-off scale: <= 1 is converged
__device__ __forceinline__ float lcp_row_residual(const LcpRow& R, float xl, float w, float mag, float arr, float L,
                                                  float U, float tolx, float& e_abs) {
    if (!R.live) {
        e_abs = 0.f;
        return 0.f;
    }
    const float s = R.b - w;
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
    return e * rcp(kLcpRelTol * (fabsf(R.b) + mag) + kLcpAbsTol);
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
// kLcpUStride * 64 floats.
constexpr int kLcpUStride = 68;
constexpr int kLcpRhs = 64;
constexpr int kLcpWorkFloats = 64 * kLcpUStride;  // the workspace the caller provides

// pivot = false: the system is symmetric positive definite (the staggered
// rounds' principal submatrices A_FF, identity rows elsewhere), eliminated in
// lane order without the pivot search -- the argmax's DPP chain is most of an
// elimination step's dependent latency
template <int RC>
__device__ __forceinline__ float lcp_ge_solve(float (&k)[RC], float rhs, int n, float* __restrict__ U, bool pivot) {
    static_assert(RC % 8 == 0, "row blocks of 8");
    const int lane = lane_id();
    bool used = lane >= n;
    for (int j = 0; j < n; ++j) {
        const int p = pivot ? wave_argmax(used ? -1.f : fabsf(k[0])) : j;
        const int left = n - j;  // live columns
        float* row = U + j * kLcpUStride;
        if (lane == p) {
            float4* u = reinterpret_cast<float4*>(row);
#pragma unroll
            for (int c = 0; c < RC; c += 4) {
                if ((c & 7) == 0 && c >= left) break;
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
            if ((c & 7) == 0 && c >= left) break;
            const float4 nxt = (c + 4 < RC) ? ur[c / 4 + 1] : make_float4(0.f, 0.f, 0.f, 0.f);
            k[c] = fmaf(-f, cur.y, k[c + 1]);
            k[c + 1] = fmaf(-f, cur.z, k[c + 2]);
            k[c + 2] = fmaf(-f, cur.w, k[c + 3]);
            if (c + 4 < RC) k[c + 3] = fmaf(-f, nxt.x, k[c + 4]);
            cur = nxt;
        }
        rhs = fmaf(-f, prhs, rhs);
        used = used || lane == p;
    }
    // back substitution, right-looking: lane l holds row l (pivot of step l)
    wave_lds_sync();
    float acc = 0.f, rdiag = 1.f;
    if (lane < n) {
        acc = U[lane * kLcpUStride + kLcpRhs];
        float dg = U[lane * kLcpUStride];
        dg = (fabsf(dg) < 1e-30f) ? 1e-30f : dg;
        rdiag = rcp(dg);
    }
    float dl = 0.f;
    for (int j = n - 1; j >= 0; --j) {
        const float dj = read_lane(acc * rdiag, j);
        dl = (lane == j) ? dj : dl;
        if (lane < j) acc = fmaf(-U[lane * (kLcpUStride - 1) + j], dj, acc);
    }
    return dl;
}

// The exact solve.  xl: lane r's impulse from the PGS (feasible), returned
// solved.  a: the Delassus registers (a[c] = A[lane][c], CFM included).
// Returns true when converged within max_solves linear solves.
template <int RC>
__device__ __forceinline__ bool wave_lcp_exact(const float (&a)[kWaveMaxRows], const LcpRow& R, float mu, int n,
                                               int max_solves, float* __restrict__ Uw, float& xl, int& n_solves,
                                               int& n_rounds, int& n_solves_staggered, long long& ge_cycles) {
    const int lane = lane_id();
    float arr = 1.f;  // A_rr (a dynamic register index would go to scratch)
#pragma unroll
    for (int c = 0; c < RC; ++c) arr = (lane == c && R.live) ? a[c] : arr;
    int solves = 0, solves1 = 0;
    bool converged = false;
    int phase = 0;          // 0 semismooth Newton, 1 staggered active set (oracle lcp_refine)
    int ws = 0;             // phase 1 working set: 0 free, 1 held at L, 2 held at U
    float Lf = 0.f, Uf = 0.f, prev = 0.f;  // phase 1: the round's frozen box, the round's start
    bool at_min = false, new_round = true;
    bool polish = false;  // inside the loose band: one more solve, then accept
    int polish_at = 0;
    int iter = 0;
    for (; iter < 4 * max_solves + 8; ++iter) {
        float mag;
        const float w = lcp_matvec<RC>(a, xl, n, mag);
        const float g = w - R.b;
        float L, U;
        lcp_bounds<RC>(R, xl, mu, n, L, U);
        const float xmax = wave_fmax(R.live ? fabsf(xl) : 0.f);
        const float tolx = 2e-6f * (1.f + xmax);
        float e_abs;
        const float rel = wave_fmax(lcp_row_residual(R, xl, w, mag, arr, L, U, tolx, e_abs));
        if (rel <= 1.f || (polish && rel <= kLcpLoose && solves > polish_at)) {
            converged = true;
            break;
        }
        if (rel > kLcpLoose) {
            polish = false;
        } else if (!polish) {
            polish = true;  // the next linear solve is the polish round
            polish_at = solves;
        }
        if (solves >= max_solves) break;
        if (phase == 1 && new_round) {
            // a round of lcp_refine: boxes frozen at the current normals
            new_round = false;
            Lf = L;
            Uf = U;
            prev = xl;
            if (xl <= Lf) { xl = Lf; ws = 1; }
            else if (xl >= Uf) { xl = Uf; ws = 2; }
            else ws = 0;
            if (Lf == Uf || !R.live) ws = 1;
            at_min = false;
            continue;  // re-evaluate at the clamped start
        }
        if (phase == 1 && at_min) {
            // boxqp_solve: minimiser on the working set -> release the worst multiplier
            at_min = false;
            float v = (ws == 1) ? -g : ((ws == 2) ? g : 0.f);
            v = (Lf == Uf || !R.live) ? 0.f : v;
            const float gm = wave_fmax(R.live ? fabsf(g) : 0.f);
            const int worst = wave_argmax(v);
            if (read_lane(v, worst) <= kLcpRelTol * (1.f + gm)) {
                // the round's QP is solved: the next round on the updated boxes
                if (wave_fmax(fabsf(xl - prev)) <= tolx) break;  // fixed point at the round-off floor
                new_round = true;
            } else if (lane == worst) {
                ws = 0;
            }
            continue;
        }
        // ---- one linear solve: the Newton system of this round ----
        float k[RC];
        bool fr;
        bool pivot = false;  // only a folded friction column makes the system unsymmetric
        float coup = 0.f;  // phase 0: d_t = coup d_n of a friction row held at +-mu x_n
        const float emax = wave_fmax(e_abs);
        if (phase == 0) {
            // a row is held when its gradient pushes it out of its box; a
            // friction row on its box edge moves with its normal
            bool fixed = !R.live;
            if (R.kind == 0) fixed = fixed || (xl <= 0.f && g >= 0.f);
            if (R.kind == 2) fixed = fixed || (xl <= R.lo && g >= 0.f) || (xl >= R.hi && g <= 0.f);
            const bool nfixed = mask_bit(static_cast<uint64_t>(__ballot(fixed)), R.nrow);
            bool cpos = false, cneg = false;
            if (R.kind == 1 && R.live && !fixed) {
                if (nfixed) {
                    fixed = true;
                } else if (U <= 0.f) {
                    // a contact opening from x_n = 0: its friction rows start on the
                    // pyramid edge they push towards (sliding); a zero gradient stays
                    if (g < 0.f) cpos = true;
                    else if (g > 0.f) cneg = true;
                    else fixed = true;
                } else if (xl >= U && g <= 0.f) {
                    cpos = true;
                } else if (xl <= L && g >= 0.f) {
                    cneg = true;
                }
            }
            fr = R.live && !fixed && !cpos && !cneg;
            coup = cpos ? mu : (cneg ? -mu : 0.f);
            const uint64_t freeM = __ballot(fr), cpM = __ballot(cpos), cnM = __ballot(cneg);
#pragma unroll
            for (int c = 0; c < RC; ++c) k[c] = (fr && mask_bit(freeM, c)) ? a[c] : ((!fr && c == lane) ? 1.f : 0.f);
            // x_t = +-mu x_n: the held friction column folds into its normal's
            pivot = (cpM | cnM) != 0ull;
            if (pivot) {
#pragma unroll
                for (int c = 0; c + 2 < RC; c += 3) {
                    const float s1 = (mask_bit(cpM, c + 1) ? 1.f : 0.f) - (mask_bit(cnM, c + 1) ? 1.f : 0.f);
                    const float s2 = (mask_bit(cpM, c + 2) ? 1.f : 0.f) - (mask_bit(cnM, c + 2) ? 1.f : 0.f);
                    if (fr) k[c] += mu * (s1 * a[c + 1] + s2 * a[c + 2]);
                }
            }
        } else {
            fr = R.live && ws == 0;
            const uint64_t freeM = __ballot(fr);
#pragma unroll
            for (int c = 0; c < RC; ++c) k[c] = (fr && mask_bit(freeM, c)) ? a[c] : ((!fr && c == lane) ? 1.f : 0.f);
        }
#ifdef MW_WAVE_PROF
        const long long tg0 = clock64();
#endif
        float d = lcp_ge_solve<RC>(k, fr ? -g : 0.f, n, Uw, pivot);
#ifdef MW_WAVE_PROF
        ge_cycles += clock64() - tg0;
#endif
        ++solves;
        solves1 += phase;
        if (phase == 0) {
            const float dn = gather_normal<RC>(d, R, n);
            d = fr ? d : coup * dn;
            // monotone line search on the largest residual
            bool accepted = false;
            float step = 1.f;
            for (int ls = 0; ls <= kLcpLineSearch; ++ls, step *= 0.5f) {
                float xt = xl + step * d;
                if (R.kind == 0) xt = fmaxf(xt, 0.f);
                if (R.kind == 2) xt = fminf(fmaxf(xt, R.lo), R.hi);
                float Lt, Ut;
                lcp_bounds<RC>(R, xt, mu, n, Lt, Ut);  // the friction boxes of the projected normals
                if (R.kind == 1) xt = fminf(fmaxf(xt, Lt), Ut);
                xt = R.live ? xt : 0.f;
                float mt;
                const float wt = lcp_matvec<RC>(a, xt, n, mt);
                const float xmt = wave_fmax(R.live ? fabsf(xt) : 0.f);
                float et;
                (void)lcp_row_residual(R, xt, wt, mt, arr, Lt, Ut, 2e-6f * (1.f + xmt), et);
                if (wave_fmax(et) < emax) {
                    xl = xt;
                    accepted = true;
                    break;
                }
            }
            if (!accepted) {
                phase = 1;
                new_round = true;
            }
            continue;
        }
        // boxqp_solve step: the longest feasible step along d (at most 1)
        const float dmax = wave_fmax(fabsf(d));
        if (dmax <= 1e-7f * (1.f + xmax)) {
            at_min = true;
            continue;
        }
        float al = 1.f;
        int side = 0;
        if (fr && d < 0.f && xl + d < Lf) { al = (Lf - xl) * rcp(d); side = 1; }
        else if (fr && d > 0.f && xl + d > Uf) { al = (Uf - xl) * rcp(d); side = 2; }
        al = fmaxf(al, 0.f);
        const float amin = wave_fmin(al);
        if (amin < 1.f) {
            const int block = wave_argmax(-al);
            const int bside = __builtin_amdgcn_readlane(side, block);
            xl = fr ? xl + amin * d : xl;
            if (lane == block) {
                xl = (bside == 1) ? Lf : Uf;
                ws = bside;
            }
        } else {
            xl = fr ? xl + d : xl;
            at_min = true;
        }
    }
    if (!converged) {
        // out of budget: inside a staggered round the friction rows keep to the
        // round's boxes, frozen at its starting normals, while the normals may
        // have shrunk since -- project onto the boxes of the current impulses
        // (normals >= 0, box rows in [lo, hi], |x_t| <= mu x_n) so the impulses
        // handed back are feasible
        float xp = xl;
        if (R.kind == 0) xp = fmaxf(xp, 0.f);
        if (R.kind == 2) xp = fminf(fmaxf(xp, R.lo), R.hi);
        float Lp, Up;
        lcp_bounds<RC>(R, xp, mu, n, Lp, Up);
        if (R.kind == 1) xp = fminf(fmaxf(xp, Lp), Up);
        xl = R.live ? xp : 0.f;
    }
    n_solves = solves;
    n_rounds = iter;
    n_solves_staggered = solves1;
    return converged;
}

}  // namespace dev
}  // namespace mw
