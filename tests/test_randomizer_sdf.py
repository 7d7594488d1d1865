"""CPU tests of the model-description randomizer mirror
(gym_ignition.randomizers.model.sdf; reference
python/gym_ignition/randomizers/model/sdf.py:166-374), as used by the
CartPole randomizer (randomizers/cartpole.py:100-135)."""

import numpy as np
import pytest

from mwstep import get_model_file
from gym_ignition.randomizers.model.sdf import (Distribution, GaussianParams, Method, SDFRandomizer,
                                                UniformParams)
from gym_ignition.utils import misc

SDF = """<sdf version="1.7"><model name="m">
<link name="a"><inertial><mass>2.0</mass></inertial></link>
<link name="b"><inertial><mass>0.0</mass></inertial></link>
<link name="c"><inertial><mass>3.0</mass></inertial></link>
</model></sdf>"""


def _masses_urdf(text):
    from xml.etree import ElementTree as etree
    return [float(m.attrib["value"]) for m in etree.fromstring(text).findall("link/inertial/mass")]


def test_cartpole_urdf_additive_force_positive():
    """The CartPole randomization: every link mass + max(U(-0.2, 0.2), 0),
    from the reference's SDF XPath on this backend's URDF."""
    r = SDFRandomizer(get_model_file("cartpole"))
    r.seed(7)
    r.new_randomization().at_xpath("*/link/inertial/mass").method(Method.Additive) \
        .sampled_from(Distribution.Uniform, UniformParams(low=-0.2, high=0.2)).force_positive().add()
    r.process_data()
    nominal = _masses_urdf(open(get_model_file("cartpole")).read())
    assert len(r.get_active_randomizations()) == len(nominal) == 3
    rng = np.random.default_rng(7)
    seen_clip = seen_shift = False
    for _ in range(20):
        got = _masses_urdf(r.sample())
        expect = [m + max(rng.uniform(-0.2, 0.2), 0.0) for m in nominal]
        assert got == pytest.approx(expect, abs=1e-12)
        seen_clip |= any(g == m for g, m in zip(got, nominal))
        seen_shift |= any(g > m for g, m in zip(got, nominal))
    assert seen_clip and seen_shift


def test_methods_distributions_and_ignore_zeros():
    path = misc.string_to_file(SDF)
    r = SDFRandomizer(path)
    r.seed(3)
    r.new_randomization().at_xpath("model/link/inertial/mass").method(Method.Coefficient) \
        .sampled_from(Distribution.Gaussian, GaussianParams(variance=0.1, mean=1.0)).ignore_zeros(True).add()
    r.process_data()
    assert len(r.get_active_randomizations()) == 2          # the zero mass is skipped
    rng = np.random.default_rng(3)
    from xml.etree import ElementTree as etree
    for _ in range(5):
        m = [float(e.text) for e in etree.fromstring(r.sample()).findall("model/link/inertial/mass")]
        # Gaussian: the reference passes `variance` as the scale
        assert m == pytest.approx([2.0 * rng.normal(1.0, 0.1), 0.0, 3.0 * rng.normal(1.0, 0.1)], abs=1e-12)
    r.clean()
    r.new_randomization().at_xpath("model/link/inertial/mass").method(Method.Absolute) \
        .sampled_from(Distribution.Uniform, UniformParams(low=5.0, high=6.0)).add()
    r.process_data()
    m = [float(e.text) for e in etree.fromstring(r.sample()).findall("model/link/inertial/mass")]
    assert all(5.0 <= v <= 6.0 for v in m)


def test_errors():
    r = SDFRandomizer(misc.string_to_file(SDF))
    with pytest.raises(RuntimeError):
        r.new_randomization().at_xpath("model/joint/axis").method(Method.Absolute) \
            .sampled_from(Distribution.Uniform, UniformParams(0.0, 1.0)).add()
    with pytest.raises(ValueError):
        r.new_randomization().sampled_from(Distribution.Gaussian, UniformParams(0.0, 1.0))
    with pytest.raises(ValueError):
        SDFRandomizer("/nonexistent/model.sdf")
