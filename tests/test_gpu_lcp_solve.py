"""The exact LCP's linear solve (csrc/wave_lcp.hpp) in isolation, through the
test hook mw_debug_lcp_solve: one wavefront solves S d = rhs over the free
rows of a random symmetric positive definite system (held rows: identity,
d = 0), by the block LDL^T on the matrix cores (lcp_mfma_solve, the kernels'
default) and by the lane elimination it replaced (lcp_ge_solve).  Reference:
numpy fp64 on the same fp32 inputs.  The systems are shaped like the kernels'
Delassus matrices: a Gram matrix J M^-1 J^T of random rows with DART's CFM on
the diagonal (contact rows 1e-5, joint rows 1e-3 relative), including
redundant rows (cond ~1e6), at every size 1..64 and with random held sets
(stage 1 of DART's two-stage LCP holds every friction row)."""

import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _system(rng, n, redundant):
    k = max(1, n // 2) if redundant else n + 6
    J = rng.normal(size=(n, k))
    if redundant and n > 2:
        J[1::3] = J[0::3][: len(J[1::3])] + 1e-3 * rng.normal(size=J[1::3].shape)
    A = J @ J.T
    A[np.diag_indices(n)] *= 1.0 + 1e-5
    return A.astype(np.float32)


def _solve(A, rhs, free, method):
    from mwstep import native as N
    n = A.shape[0]
    mask = 0
    for i in np.flatnonzero(free):
        mask |= 1 << int(i)
    d = np.zeros(n, np.float32)
    fp = ctypes.POINTER(ctypes.c_float)
    A = np.ascontiguousarray(A, np.float32)
    rhs = np.ascontiguousarray(rhs, np.float32)
    rc = N.lib().mw_debug_lcp_solve(A.ctypes.data_as(fp), rhs.ctypes.data_as(fp), ctypes.c_uint64(mask), n, method,
                                   d.ctypes.data_as(fp))
    assert rc == 0
    return d


def _reference(A, rhs, free):
    A64 = A.astype(np.float64)
    d = np.zeros(A.shape[0])
    f = np.flatnonzero(free)
    if len(f):
        d[f] = np.linalg.solve(A64[np.ix_(f, f)], rhs.astype(np.float64)[f])
    return d


@pytest.mark.parametrize("method", [0, 1])
def test_linear_solve_matches_numpy(require_gpu, method):
    rng = np.random.default_rng(5)
    worst = 0.0
    for n in list(range(1, 65)) + [12, 24, 31, 32, 33, 48, 63, 64]:
        for trial in range(3):
            redundant = trial == 2
            A = _system(rng, n, redundant)
            rhs = rng.normal(size=n).astype(np.float32)
            free = rng.random(n) < (1.0 if trial == 0 else 0.6)
            if trial == 1:
                free[0::3] = True   # stage 1: normals free, friction rows mostly held
            ref = _reference(A, rhs, free)
            d = _solve(A, rhs, free, method)
            assert np.all(d[~free] == 0.0)
            # backward error: the residual of the fp32 solve relative to the
            # system's scale (what the active-set method's refinement sees)
            f = np.flatnonzero(free)
            if len(f):
                A64 = A.astype(np.float64)[np.ix_(f, f)]
                res = np.abs(A64 @ d[f] - rhs[f]).max() / (np.abs(A64).max() * np.abs(d[f]).max() + np.abs(rhs[f]).max())
                worst = max(worst, res)
                assert res < 2e-5, (n, trial, res)
                if not redundant:
                    assert np.abs(d - ref).max() <= 2e-3 * (1.0 + np.abs(ref).max()), (n, trial)
    print(f"linear solve method {method}: worst relative residual {worst:.2e}")


def test_methods_agree_on_well_conditioned(require_gpu):
    rng = np.random.default_rng(9)
    for n in (3, 12, 17, 32, 40, 64):
        A = _system(rng, n, False)
        rhs = rng.normal(size=n).astype(np.float32)
        free = np.ones(n, bool)
        free[rng.random(n) < 0.3] = False
        d0, d1 = _solve(A, rhs, free, 0), _solve(A, rhs, free, 1)
        assert np.abs(d0 - d1).max() <= 1e-3 * (1.0 + np.abs(d1).max())
