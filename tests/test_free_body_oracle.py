"""Pin the fp64 free-body oracle (or_free_step) before trusting it (CPU).

  * free fall: DART's semi-implicit Euler (velocity first, then position) in
    closed form;
  * torque-free spin about a principal axis: the FreeJoint position update
    T <- T exp(dt V) composes exactly to exp(t V);
  * the reference contact KAT (tests/test_scenario/test_contacts.py:57-122):
    a 5 kg, 0.2 m cube released 5 cm above the ground plane is in contact
    after 150 ms, every normal is +z, the vertical contact forces sum to its
    weight within 0.1 N, and Link::contactWrench (Link.cpp:436-482) is
    [0, 0, m g, 0, 0, 0]; also for the double-collision cube of :22-54;
  * Coulomb friction: a cube sliding at 1 m/s decelerates at mu g;
  * a sphere resting on the plane carries its weight on one point.
"""

import math

import numpy as np
import pytest

G = 9.8


def cube_urdf(double=False, mass=5.0, edge=0.2):
    i = 1 / 12 * mass * (edge ** 2 + edge ** 2)
    if double:
        col = "".join(f'<collision><geometry><box size="{edge} {edge / 2} {edge}"/></geometry>'
                      f'<origin rpy="0 0 0" xyz="0 {s * edge / 4} 0"/></collision>' for s in (-1, 1))
    else:
        col = f'<collision><geometry><box size="{edge} {edge} {edge}"/></geometry></collision>'
    return (f'<robot name="cube_robot"><link name="cube"><inertial><origin rpy="0 0 0" xyz="0 0 0"/>'
            f'<mass value="{mass}"/><inertia ixx="{i}" ixy="0" ixz="0" iyy="{i}" iyz="0" izz="{i}"/>'
            f'</inertial>{col}</link></robot>')


def sphere_urdf(mass=2.0, r=0.1):
    i = 0.4 * mass * r * r
    return (f'<robot name="ball"><link name="ball"><inertial><mass value="{mass}"/>'
            f'<inertia ixx="{i}" iyy="{i}" izz="{i}" ixy="0" ixz="0" iyz="0"/></inertial>'
            f'<collision><geometry><sphere radius="{r}"/></geometry></collision></link></robot>')


def contact_wrench(world):
    """Link::contactWrench: sum of forces, sum of (p - o_L) x f, world frame."""
    f = np.zeros(3)
    t = np.zeros(3)
    for p, n, force, d in world.contacts:
        f += force
        t += np.cross(p - world.p, force)
    return np.concatenate([f, t])


def test_free_fall(oracle):
    cm = oracle.load_urdf(cube_urdf(), pose_xyz=(0, 0, 10.0))
    w = oracle.FreeWorld(cm, ground=False)
    dt, z, v = 1e-3, 10.0, 0.0
    for _ in range(1000):
        w.step()
        v -= G * dt
        z += v * dt
    assert abs(w.p[2] - z) < 1e-10 and abs(w.twist[1][2] - v) < 1e-10
    assert len(w.contacts) == 0


def test_torque_free_spin(oracle):
    cm = oracle.load_urdf(cube_urdf(), pose_xyz=(0, 0, 10.0))
    cm.free.gravity[2] = 0.0
    w = oracle.FreeWorld(cm, ground=False)
    w.set_twist([0.0, 0.0, 2.0], [0.5, 0.0, 0.0])
    for _ in range(1000):
        w.step()
    # isotropic inertia, COM at the origin: the angular velocity is constant, so
    # the rotation composes exactly to Rz(2 rad); the origin's WORLD velocity is
    # constant (the body-frame v turns against w: v' = v x w), up to the
    # semi-implicit discretisation
    th = 2.0
    Rz = np.array([[math.cos(th), -math.sin(th), 0], [math.sin(th), math.cos(th), 0], [0, 0, 1]])
    np.testing.assert_allclose(w.R, Rz, atol=1e-12)
    np.testing.assert_allclose(w.p, [0.5, 0.0, 10.0], atol=2e-3)
    np.testing.assert_allclose(w.R @ w.twist[1], [0.5, 0.0, 0.0], atol=2e-3)


@pytest.mark.parametrize("double", [False, True])
def test_cube_contact_kat(oracle, double):
    cm = oracle.load_urdf(cube_urdf(double), pose_xyz=(0, 0, 0.15))
    w = oracle.FreeWorld(cm)
    w.step()
    assert len(w.contacts) == 0               # 5 cm gap: no contact yet
    for _ in range(149):
        w.step()
    assert len(w.contacts) == (8 if double else 4)
    for p, n, f, d in w.contacts:
        np.testing.assert_allclose(n, [0, 0, 1])
        assert f[2] > 0 and d > 0
    fz = sum(c[2][2] for c in w.contacts)
    assert fz == pytest.approx(5 * G, abs=0.1)
    np.testing.assert_allclose(contact_wrench(w), [0, 0, fz, 0, 0, 0], atol=1e-6)


def test_coulomb_sliding(oracle):
    cm = oracle.load_urdf(cube_urdf(), pose_xyz=(0, 0, 0.1))
    w = oracle.FreeWorld(cm, mu=0.5)
    for _ in range(50):                        # settle
        w.step()
    w.set_twist([0, 0, 0], [1.0, 0, 0])
    for _ in range(100):
        w.step()
    vx = (w.R @ w.twist[1])[0]
    assert vx == pytest.approx(1.0 - 0.5 * G * 0.1, abs=0.02)
    for _ in range(200):
        w.step()
    assert abs((w.R @ w.twist[1])[0]) < 1e-3   # stopped (sticks)


def test_resting_sphere(oracle):
    cm = oracle.load_urdf(sphere_urdf(), pose_xyz=(0, 0, 0.1))
    w = oracle.FreeWorld(cm)
    for _ in range(500):
        w.step()
    assert len(w.contacts) == 1
    p, n, f, d = w.contacts[0]
    assert f[2] == pytest.approx(2.0 * G, abs=0.05) and abs(p[2]) < 1e-3
