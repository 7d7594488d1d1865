"""The fp64 oracle reproduces the committed golden fixtures (tests/golden/,
made by tests/golden/make_golden.py): any change of the oracle's arithmetic
shows up here before it can move the GPU parity tests' reference."""

import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import make_golden  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("name", sorted(make_golden.FIXTURES))
def test_oracle_reproduces_fixture(name):
    ref = np.load(os.path.join(GOLDEN, name + ".npz"))
    new = make_golden.FIXTURES[name]()
    assert set(ref.files) == set(new)
    for k in ref.files:
        if ref[k].dtype.kind in "fc":
            np.testing.assert_allclose(new[k], ref[k], rtol=0, atol=1e-12, err_msg=f"{name}:{k}")
        else:
            assert np.array_equal(new[k], ref[k]), f"{name}:{k}"


def test_fixtures_are_meaningful():
    c = np.load(os.path.join(GOLDEN, "cartpole_discrete.npz"))
    assert c["done"].any() and not c["done"].all()            # episodes end inside the horizon
    h = np.load(os.path.join(GOLDEN, "icub_stand.npz"))
    assert len(h["contact_fz"]) == 8                           # four corners per foot
    assert h["contact_fz"].sum() == pytest.approx(30.7 * 9.8, abs=3.0)   # still swaying by ~1%
    assert len(h["joint_names"]) == 32 and "l_knee" in h["joint_names"]
