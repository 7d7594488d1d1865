/* Test-only: runs the fp64 oracle (oracle/oracle.c) under AddressSanitizer +
 * UndefinedBehaviorSanitizer (tests/test_sanitizers.py).
 *
 *   oracle_san <case file> <out file>
 *
 * A case file is what tests/test_sanitizers.py wrote from pyoracle's own
 * ctypes structures (little endian):
 *   int32 kind, int32 steps, int32 pgs_iters, int32 warm, double dt
 *   kind 0 (or_step, fixed-base chain / tree):
 *       or_model, double q[n], double qd[n], int32 mode[n], double cmd[n]
 *   kind 1 (or_float_step_warm, floating base with ground contacts):
 *       or_float_model, or_float_state, int32 mode[n], double cmd[n]
 * The out file receives the final q, qd (kind 0) or the final or_float_state
 * followed by the last step's contact count and forces (kind 1). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static int read_all(FILE* f, void* dst, size_t n)
{
    return fread(dst, 1, n, f) == n;
}

int main(int argc, char** argv)
{
    if (argc != 3) {
        fprintf(stderr, "usage: %s <case> <out>\n", argv[0]);
        return 2;
    }
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    int32_t hdr[4];
    double dt;
    if (!read_all(f, hdr, sizeof hdr) || !read_all(f, &dt, sizeof dt)) return 3;
    const int kind = hdr[0], steps = hdr[1], pgs = hdr[2], use_warm = hdr[3];
    FILE* o = fopen(argv[2], "wb");
    if (!o) return 2;
    int32_t mode[OR_MAXB];
    double cmd[OR_MAXB];
    if (kind == 0) {
        or_model* m = malloc(sizeof *m);
        double q[OR_MAXB], qd[OR_MAXB], qdd[OR_MAXB], force[OR_MAXB];
        if (!m || !read_all(f, m, sizeof *m) || m->n < 0 || m->n > OR_MAXB) return 3;
        const int n = m->n;
        if (!read_all(f, q, sizeof(double) * n) || !read_all(f, qd, sizeof(double) * n) ||
            !read_all(f, mode, sizeof(int32_t) * n) || !read_all(f, cmd, sizeof(double) * n))
            return 3;
        for (int s = 0; s < steps; ++s) or_step(m, dt, q, qd, mode, cmd, pgs, qdd, force);
        fwrite(q, sizeof(double), n, o);
        fwrite(qd, sizeof(double), n, o);
        free(m);
    } else if (kind == 1) {
        or_float_model* m = malloc(sizeof *m);
        or_float_state st;
        double* warm = calloc(OR_WARM_WORDS, sizeof(double));
        double* cp = calloc(3 * OR_MAXFC, sizeof(double));
        double* cf = calloc(3 * OR_MAXFC, sizeof(double));
        double* cd = calloc(OR_MAXFC, sizeof(double));
        int32_t* cb = calloc(OR_MAXFC, sizeof(int32_t));
        if (!m || !warm || !cp || !cf || !cd || !cb) return 4;
        if (!read_all(f, m, sizeof *m) || !read_all(f, &st, sizeof st) || m->tree.n < 0 || m->tree.n > OR_MAXB)
            return 3;
        const int n = m->tree.n;
        if (!read_all(f, mode, sizeof(int32_t) * n) || !read_all(f, cmd, sizeof(double) * n)) return 3;
        int32_t nc = 0;
        for (int s = 0; s < steps; ++s)
            nc = or_float_step_warm(m, dt, &st, mode, cmd, pgs, 0.0, use_warm ? warm : NULL, cp, cf, cd, cb);
        fwrite(&st, sizeof st, 1, o);
        fwrite(&nc, sizeof nc, 1, o);
        fwrite(cf, sizeof(double), 3 * (size_t)nc, o);
        free(m); free(warm); free(cp); free(cf); free(cd); free(cb);
    } else {
        return 3;
    }
    fclose(f);
    fclose(o);
    return 0;
}
