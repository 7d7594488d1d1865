/* mwstep_testhooks.h -- test-only entry points of libmwstep.so.
 *
 * Not part of the ScenarI/O surface (include/mwstep.h) and not meant for a
 * running simulator: each hook allocates its own device buffers and its own
 * stream, and synchronises only that stream.  tests/ binds them through
 * mwstep.native.TEST_SIGNATURES. */
#ifndef MWSTEP_TESTHOOKS_H
#define MWSTEP_TESTHOOKS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One linear solve of the exact LCP's active-set method on a single wavefront
 * (csrc/wave_lcp.hpp): S d = rhs restricted to the rows of free_mask (held
 * rows: d = 0), S = the row-major n x n matrix A (n <= 64, symmetric positive
 * definite on the free rows), host buffers.  method 0: block LDL^T on the
 * matrix cores (lcp_mfma_solve, the kernels' default), 1: Gaussian
 * elimination over the lanes (lcp_ge_solve).  Returns 0 on success. */
int mw_debug_lcp_solve(const float* A, const float* rhs, uint64_t free_mask, int32_t n, int32_t method, float* d);

/* The convex hull the scene kernel's mesh narrow phase builds for n <= 16
 * support points (csrc/hull.hpp build_hull, fp64, host only): counts = {faces,
 * edges} (0, 0 for a flat set); planes [32][4] = outward normal, offset (inside
 * n . x <= d); faces [32][17] = vertex count, then the polygon's vertex
 * indices counter-clockwise seen from outside; edges [48][4] = the two
 * vertices, then the two faces meeting there.  Returns 0 (MW_OK). */
int mw_debug_hull(const double* pts, int32_t n, double* planes, int32_t* faces, int32_t* edges, int32_t* counts);

/* The large-contact workspace of world w of a scene after its last run
 * (csrc/scene_kernel.hip ScBigWs: contacts [cmax][20], then the row fields
 * [11][rows]; the world's last step took the large-contact path when its
 * contact count exceeds 32 or its rows 64): the first min(cap, 20 cmax + 11
 * rows) floats into out.  cmax = rows = 0: the scene has no workspace.
 * Synchronises the scene's stream.  Returns 0 on success. */
typedef struct mw_scene mw_scene;
int mw_debug_scene_big_ws(mw_scene* s, int32_t w, float* out, int64_t cap, int32_t* cmax, int32_t* rows);

#ifdef __cplusplus
}
#endif
#endif /* MWSTEP_TESTHOOKS_H */
