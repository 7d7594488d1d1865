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

#ifdef __cplusplus
}
#endif
#endif /* MWSTEP_TESTHOOKS_H */
