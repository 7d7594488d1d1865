"""Mesh collision fixtures written at test time (the reference ships no mesh
files; its Physics.cpp:897-931 loads whatever a <mesh> URI names): a cube as
binary / ASCII STL and OBJ, an irregular 12-vertex "rock" (a stretched,
perturbed icosahedron) as OBJ and STL, and URDF / SDF models around them."""

import struct

import numpy as np

CUBE_TRIS = [(0, 2, 1), (1, 2, 3), (4, 5, 6), (5, 7, 6), (0, 1, 4), (1, 5, 4),
             (2, 6, 3), (3, 6, 7), (0, 4, 2), (2, 4, 6), (1, 3, 5), (3, 7, 5)]


def cube_vertices(half=(0.1, 0.1, 0.1)):
    """8 corners in the box corner order (bit 2: x, bit 1: y, bit 0: z)."""
    return np.array([[(1 if c & 4 else -1) * half[0], (1 if c & 2 else -1) * half[1], (1 if c & 1 else -1) * half[2]]
                     for c in range(8)], dtype=float)


def icosahedron():
    t = (1 + 5 ** 0.5) / 2
    v = np.array([(-1, t, 0), (1, t, 0), (-1, -t, 0), (1, -t, 0), (0, -1, t), (0, 1, t), (0, -1, -t), (0, 1, -t),
                  (t, 0, -1), (t, 0, 1), (-t, 0, -1), (-t, 0, 1)], dtype=float)
    f = [(0, 11, 5), (0, 5, 1), (0, 1, 7), (0, 7, 10), (0, 10, 11), (1, 5, 9), (5, 11, 4), (11, 10, 2), (10, 7, 6),
         (7, 1, 8), (3, 9, 4), (3, 4, 2), (3, 2, 6), (3, 6, 8), (3, 8, 9), (4, 9, 5), (2, 4, 11), (6, 2, 10),
         (8, 6, 7), (9, 8, 1)]
    return v / np.linalg.norm(v[0]), f


def rock_vertices(seed=0, size=(0.12, 0.08, 0.06)):
    v, f = icosahedron()
    rng = np.random.default_rng(seed)
    v = v * np.asarray(size) * rng.uniform(0.85, 1.15, (len(v), 1))
    return v.astype(np.float32).astype(float), f   # exact in binary STL


def write_stl_binary(path, v, tris):
    with open(path, "wb") as fh:
        fh.write(b"mesh fixture".ljust(80, b" "))
        fh.write(struct.pack("<I", len(tris)))
        for t in tris:
            fh.write(struct.pack("<3f", 0.0, 0.0, 0.0))
            for i in t:
                fh.write(struct.pack("<3f", *v[i]))
            fh.write(struct.pack("<H", 0))


def write_stl_ascii(path, v, tris):
    with open(path, "w") as fh:
        fh.write("solid fixture\n")
        for t in tris:
            fh.write("  facet normal 0 0 0\n    outer loop\n")
            for i in t:
                fh.write(f"      vertex {float(v[i][0])!r} {float(v[i][1])!r} {float(v[i][2])!r}\n")
            fh.write("    endloop\n  endfacet\n")
        fh.write("endsolid fixture\n")


def write_obj(path, v, tris):
    with open(path, "w") as fh:
        fh.write("# mesh fixture\n")
        for p in v:
            fh.write(f"v {float(p[0])!r} {float(p[1])!r} {float(p[2])!r}\n")
        for t in tris:
            fh.write("f " + " ".join(str(i + 1) for i in t) + "\n")


def mesh_body_urdf(uri, mass=2.0, half=(0.1, 0.1, 0.1), scale=(1, 1, 1), xyz=(0, 0, 0), rpy=(0, 0, 0),
                   name="rock"):
    """a floating body whose only collision is the mesh (box inertia of `half`)"""
    a, b, c = (2 * h for h in half)
    ixx, iyy, izz = mass * (b * b + c * c) / 12, mass * (a * a + c * c) / 12, mass * (a * a + b * b) / 12
    return (f'<robot name="{name}"><link name="body"><inertial><mass value="{mass}"/>'
            f'<inertia ixx="{ixx}" iyy="{iyy}" izz="{izz}" ixy="0" ixz="0" iyz="0"/></inertial>'
            f'<collision><origin xyz="{xyz[0]} {xyz[1]} {xyz[2]}" rpy="{rpy[0]} {rpy[1]} {rpy[2]}"/>'
            f'<geometry><mesh filename="{uri}" scale="{scale[0]} {scale[1]} {scale[2]}"/></geometry>'
            f'</collision></link></robot>')


def mesh_body_sdf(uri, mass=2.0, half=(0.1, 0.1, 0.1), scale=(1, 1, 1), pose="0 0 0 0 0 0", name="rock"):
    a, b, c = (2 * h for h in half)
    ixx, iyy, izz = mass * (b * b + c * c) / 12, mass * (a * a + c * c) / 12, mass * (a * a + b * b) / 12
    return (f'<?xml version="1.0"?><sdf version="1.7"><model name="{name}"><link name="body">'
            f'<inertial><mass>{mass}</mass><inertia><ixx>{ixx}</ixx><iyy>{iyy}</iyy><izz>{izz}</izz>'
            f'<ixy>0</ixy><ixz>0</ixz><iyz>0</iyz></inertia></inertial>'
            f'<collision name="c"><pose>{pose}</pose><geometry><mesh><uri>{uri}</uri>'
            f'<scale>{scale[0]} {scale[1]} {scale[2]}</scale></mesh></geometry></collision>'
            f'</link></model></sdf>')


def write_dae(path, geoms, nodes, unit=1.0, extra_geom=None):
    """COLLADA fixture: geoms = {id: [V, 3] positions}; nodes = list of
    (transform elements xml, [geometry ids], [child nodes]) instantiated by the
    visual scene; extra_geom = an id of geoms left un-instantiated"""
    def node_xml(n):
        tr, gids, kids = n
        return ("<node>" + tr + "".join(f'<instance_geometry url="#{g}"/>' for g in gids) +
                "".join(node_xml(k) for k in kids) + "</node>")
    lib = ""
    for gid, v in geoms.items():
        arr = " ".join(repr(float(x)) for x in np.asarray(v).reshape(-1))
        lib += (f'<geometry id="{gid}"><mesh><source id="{gid}-pos"><float_array id="{gid}-arr" count="{v.size}">'
                f'{arr}</float_array><technique_common><accessor source="#{gid}-arr" count="{len(v)}" stride="3">'
                f'<param name="X" type="float"/><param name="Y" type="float"/><param name="Z" type="float"/>'
                f'</accessor></technique_common></source><vertices id="{gid}-vtx"><input semantic="POSITION" '
                f'source="#{gid}-pos"/></vertices></mesh></geometry>')
    text = ('<?xml version="1.0" encoding="utf-8"?>\n<COLLADA xmlns="http://www.collada.org/2005/11/COLLADASchema" '
            f'version="1.4.1"><asset><unit name="u" meter="{unit!r}"/><up_axis>Z_UP</up_axis></asset>'
            f'<library_geometries>{lib}</library_geometries><library_visual_scenes><visual_scene id="scene">'
            + "".join(node_xml(n) for n in nodes) +
            '</visual_scene></library_visual_scenes><scene><instance_visual_scene url="#scene"/></scene></COLLADA>')
    with open(path, "w") as fh:
        fh.write(text)
