"""Models of the scene tests: the reference's contact-test cubes
(tests/common/utils.py:148-176 get_cube_urdf_string, and the double-collision
variant of tests/test_scenario/test_contacts.py:22-53), written here from
their stated parameters (5 kg, 0.2 m edge)."""


def cube_urdf(double_collision: bool = False, mass: float = 5.0, edge: float = 0.2) -> str:
    i = 1 / 12 * mass * (edge ** 2 + edge ** 2)
    if double_collision:
        col = "".join(f'<collision><origin xyz="0 {y} 0" rpy="0 0 0"/><geometry><box size="{edge} {edge / 2} {edge}"/>'
                      f'</geometry></collision>' for y in (-edge / 4, edge / 4))
    else:
        col = f'<collision><origin xyz="0 0 0" rpy="0 0 0"/><geometry><box size="{edge} {edge} {edge}"/></geometry></collision>'
    return (f'<robot name="cube_robot"><link name="cube"><inertial><origin rpy="0 0 0" xyz="0 0 0"/>'
            f'<mass value="{mass}"/><inertia ixx="{i}" ixy="0" ixz="0" iyy="{i}" iyz="0" izz="{i}"/></inertial>'
            f'{col}</link></robot>')


def sphere_urdf(mass: float = 1.0, radius: float = 0.1) -> str:
    i = 0.4 * mass * radius ** 2
    return (f'<robot name="ball"><link name="ball"><inertial><mass value="{mass}"/>'
            f'<inertia ixx="{i}" iyy="{i}" izz="{i}" ixy="0" ixz="0" iyz="0"/></inertial>'
            f'<collision><geometry><sphere radius="{radius}"/></geometry></collision></link></robot>')


def plank_urdf(k: int = 5, mass: float = 5.0, edge: float = 0.2) -> str:
    """k cubes of `edge` fused along x into one rigid link (k box collisions)."""
    L = k * edge
    ixx = 1 / 12 * mass * (2 * edge ** 2)
    iyy = 1 / 12 * mass * (L ** 2 + edge ** 2)
    col = "".join(f'<collision><origin xyz="{(i - (k - 1) / 2) * edge} 0 0" rpy="0 0 0"/><geometry>'
                  f'<box size="{edge} {edge} {edge}"/></geometry></collision>' for i in range(k))
    return (f'<robot name="plank"><link name="plank"><inertial><origin rpy="0 0 0" xyz="0 0 0"/>'
            f'<mass value="{mass}"/><inertia ixx="{ixx}" ixy="0" ixz="0" iyy="{iyy}" iyz="0" izz="{iyy}"/>'
            f'</inertial>{col}</link></robot>')
