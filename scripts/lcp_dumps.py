"""Reading the kernels' exact-LCP dumps (debug builds with -DMW_WAVE_PROF;
-DMW_DUMP_FAIL dumps the unconverged world-steps): scripts/wave_prof.py and
scripts/leg_probe.py (LEG_DUMP=1) save them, scripts/lcp_dump_check.py
re-solves them in fp64."""
import ctypes
import os

import numpy as np


def save_dumps(fd, nvec, name, slots=8):
    """The kernels' LCP dumps (up to `slots`; debug builds, see wave_tree.hpp
    g_wave_dump): every slot as n, A (n x n), the row vectors, solve counts."""
    per = 8 + 64 * 64 + nvec * 64
    dump = np.zeros(slots * per, dtype=np.float32)
    fd.argtypes = [ctypes.c_void_p, ctypes.c_int]
    if fd(dump.ctypes.data, dump.size) != 0:
        return
    D = dump.reshape(slots, per)
    used = [k for k in range(slots) if D[k, 0] > 0]
    if not used:
        print("no LCP dumped")
        return
    out = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", name)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    # row r of the dump = lane r's registers a[c] = A[r][c] written at [c][r]: transpose
    A = np.stack([D[k, 8:8 + 64 * 64].reshape(64, 64).T for k in used])
    V = np.stack([D[k, 8 + 64 * 64:].reshape(nvec, 64) for k in used])
    H = np.stack([D[k, :8] for k in used])
    np.savez(out, A=A, V=V, head=H, layout=("scene" if nvec == 8 else "wave"))
    for k in range(len(used)):
        print(f"dumped LCP {k}: {int(H[k, 0])} rows, {int(H[k, 1])} solves ({int(H[k, 2])} in stage 2), ok {int(H[k, 4])}")
