"""Constant-folded ("baked") kernels for the shipped models: the generated
header is up to date, and the library picks a baked kernel only for a
bit-identical parameter block (CPU; the GPU equivalence test is in
test_gpu_vecenv_parity.py)."""

import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT


def test_header_up_to_date():
    rc = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "bake_models.py"), "--check"]).returncode
    assert rc == 0, "gym-ignition_amd/csrc/baked_models.hpp is stale: run scripts/bake_models.py"


def _baked(path, pose=(0, 0, 0, 1, 0, 0, 0), gravity=None, param=None):
    from mwstep import native as N
    cfg = N.MwConfig(1e-3, 1.0, 1, 1, 0, 0)
    h = ctypes.c_void_p()
    N.check(N.lib().mw_create(ctypes.byref(cfg), ctypes.byref(h)))
    try:
        p = np.array(pose, dtype=np.float64)
        N.check(N.lib().mw_load_model(h, path.encode(), N.dptr(p), b""))
        if gravity is not None:
            g = np.array(gravity, dtype=np.float64)
            N.check(N.lib().mw_set_gravity(h, N.dptr(g)))
        if param is not None:
            N.check(N.lib().mw_set_joint_param(h, *param))
        v = ctypes.c_int32()
        N.check(N.lib().mw_baked_model(h, ctypes.byref(v)))
        return v.value
    finally:
        N.lib().mw_destroy(h)


def test_baked_selection(cartpole_file, pendulum_file, monkeypatch):
    from mwstep import native as N
    assert _baked(cartpole_file) == 1
    assert _baked(pendulum_file) == 2
    assert _baked(cartpole_file, pose=(0, 0, 0, 0.7071068, 0.7071068, 0, 0)) == 0  # gravity in base frame
    assert _baked(cartpole_file, gravity=(0, 0, -9.81)) == 0
    assert _baked(pendulum_file, param=(0, N.PARAM_VISCOUS_FRICTION, 0.1)) == 0
    assert _baked(cartpole_file, pose=(1, 2, 3, 1, 0, 0, 0)) == 1  # translation does not enter the block
    monkeypatch.setenv("MWSTEP_DISABLE_BAKED", "1")
    assert _baked(cartpole_file) == 0
