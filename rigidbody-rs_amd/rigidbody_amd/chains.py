"""Synthetic serial chains and the input distributions of the benchmark configs.

SURVEY.md §8(d): the 30-DOF stress chain cycles FR3-like link constants with every
joint axis along z; inputs are q ~ U(lower, upper), qd ~ U(+-velocity),
qdd ~ U(+-10 rad/s^2), tau ~ U(+-effort) per joint.

The chain is emitted as URDF with the same top-level structure the reference's
loader relies on (multibody.rs:65-77 pairs joints and links BY INDEX): a fixed
world->base joint first, then joint k (base-side parent -> link k) at index k, so
index pairing and child pairing agree.
"""
from __future__ import annotations

import os
import xml.etree.ElementTree as ET

_HERE = os.path.dirname(os.path.abspath(__file__))
FR3_COMPACT = os.path.join(os.path.dirname(_HERE), "assets", "fr3_compact.urdf")

SEED = 20250224


def fr3_urdf_text() -> str:
    with open(FR3_COMPACT) as f:
        return f.read()


def _fr3_chain_rows():
    """(joint origin xyz/rpy text, link inertial attrs) for the 7 FR3 revolute joints."""
    root = ET.fromstring(fr3_urdf_text())
    links = {el.get("name"): el for el in root if el.tag == "link"}
    rows = []
    for el in root:
        if el.tag == "joint" and el.get("type") == "revolute":
            o = el.find("origin")
            link = links[el.find("child").get("link")]
            inr = link.find("inertial")
            rows.append({
                "xyz": o.get("xyz", "0 0 0"),
                "rpy": o.get("rpy", "0 0 0"),
                "com": inr.find("origin").get("xyz"),
                "mass": inr.find("mass").get("value"),
                "inertia": {k: inr.find("inertia").get(k) for k in ("ixx", "ixy", "ixz", "iyy", "iyz", "izz")},
            })
    return rows


def synthetic_chain_urdf(n: int, lower=-3.141592653589793, upper=3.141592653589793,
                         velocity=2.0, effort=50.0) -> str:
    """n-DOF z-axis serial chain cycling the FR3 joint origins and link inertials."""
    rows = _fr3_chain_rows()
    out = ['<?xml version="1.0"?>', f'<robot name="chain{n}">',
           '  <link name="base"/>']
    for k in range(1, n + 1):
        r = rows[(k - 1) % len(rows)]
        i = r["inertia"]
        out += [f'  <link name="link{k}">',
                "    <inertial>",
                f'      <origin rpy="0 0 0" xyz="{r["com"]}"/>',
                f'      <mass value="{r["mass"]}"/>',
                f'      <inertia ixx="{i["ixx"]}" ixy="{i["ixy"]}" ixz="{i["ixz"]}" iyy="{i["iyy"]}" iyz="{i["iyz"]}" izz="{i["izz"]}"/>',
                "    </inertial>",
                "  </link>"]
    out.append('  <link name="world"/>')
    out += ['  <joint name="world_joint" type="fixed">',
            '    <origin rpy="0 0 0" xyz="0 0 0"/>',
            '    <parent link="world"/>', '    <child link="base"/>', "  </joint>"]
    for k in range(1, n + 1):
        r = rows[(k - 1) % len(rows)]
        parent = "base" if k == 1 else f"link{k - 1}"
        out += [f'  <joint name="joint{k}" type="revolute">',
                f'    <origin rpy="{r["rpy"]}" xyz="{r["xyz"]}"/>',
                f'    <parent link="{parent}"/>', f'    <child link="link{k}"/>',
                '    <axis xyz="0 0 1"/>',
                f'    <limit effort="{effort}" lower="{lower}" upper="{upper}" velocity="{velocity}"/>',
                "  </joint>"]
    out.append("</robot>")
    return "\n".join(out) + "\n"


def general_chain_urdf(n: int, seed: int = 7) -> str:
    """Test model beyond the reference's reading, for
    RB_MODEL_URDF_TREE | RB_MODEL_GENERAL_AXES: n revolute/continuous joints with random
    unit axes (every 4th +z, one -z), random origins, inertial-origin rpy, a massive
    fixed-joint link after every 3rd body, a fixed-only side branch on body 2, and a
    fixed world->base joint.  Document order is deliberately NOT the chain order."""
    import numpy as np
    rng = np.random.default_rng(seed)

    def inertial(mass):
        a, b = rng.uniform(0.01, 0.05, 2)
        c = rng.uniform(abs(a - b) + 0.005, a + b - 0.001)  # triangle inequality
        com = rng.uniform(-0.1, 0.1, 3)
        rpy = rng.uniform(-np.pi, np.pi, 3)
        return ("    <inertial>\n"
                f'      <origin rpy="{float(rpy[0])!r} {float(rpy[1])!r} {float(rpy[2])!r}" xyz="{float(com[0])!r} {float(com[1])!r} {float(com[2])!r}"/>\n'
                f'      <mass value="{float(mass)!r}"/>\n'
                f'      <inertia ixx="{float(a)!r}" ixy="0" ixz="0" iyy="{float(b)!r}" iyz="0" izz="{float(c)!r}"/>\n'
                "    </inertial>")

    def origin():
        xyz = rng.uniform(-0.15, 0.15, 3)
        rpy = rng.uniform(-np.pi, np.pi, 3)
        return f'    <origin rpy="{float(rpy[0])!r} {float(rpy[1])!r} {float(rpy[2])!r}" xyz="{float(xyz[0])!r} {float(xyz[1])!r} {float(xyz[2])!r}"/>'

    links, joints = ['  <link name="world"/>', '  <link name="base"/>'], [
        '  <joint name="world_joint" type="fixed">\n    <origin rpy="0 0 0" xyz="0 0 0.1"/>\n'
        '    <parent link="world"/>\n    <child link="base"/>\n  </joint>']
    parent = "base"
    for k in range(1, n + 1):
        if k % 4 == 1:
            axis = np.array([0.0, 0.0, 1.0])
        elif k == 3:
            axis = np.array([0.0, 0.0, -1.0])
        else:
            axis = rng.normal(size=3)
            axis /= np.linalg.norm(axis) / rng.uniform(0.5, 2.0)  # not unit: the reader normalises
        name = f"body{k}"
        links.append(f'  <link name="{name}">\n{inertial(float(rng.uniform(0.5, 3.0)))}\n  </link>')
        kind = "continuous" if k == 2 else "revolute"
        lim = ('    <limit effort="40" velocity="2.5"/>' if kind == "continuous" else
               '    <limit effort="40" lower="-2.8" upper="2.8" velocity="2.5"/>')
        joints.append(f'  <joint name="j{k}" type="{kind}">\n{origin()}\n    <parent link="{parent}"/>\n'
                      f'    <child link="{name}"/>\n    <axis xyz="{float(axis[0])!r} {float(axis[1])!r} {float(axis[2])!r}"/>\n'
                      f"{lim}\n  </joint>")
        parent = name
        if k % 3 == 0:  # a massive fixed link between bodies: merged into body k
            fx = f"flange{k}"
            links.append(f'  <link name="{fx}">\n{inertial(float(rng.uniform(0.2, 1.0)))}\n  </link>')
            joints.append(f'  <joint name="fix{k}" type="fixed">\n{origin()}\n    <parent link="{parent}"/>\n'
                          f'    <child link="{fx}"/>\n  </joint>')
            parent = fx
        if k == 2:  # fixed-only side branch (a sensor): merged, not a chain branch
            links.append(f'  <link name="sensor">\n{inertial(0.3)}\n  </link>')
            joints.append(f'  <joint name="sensor_mount" type="fixed">\n{origin()}\n    <parent link="{name}"/>\n'
                          '    <child link="sensor"/>\n  </joint>')
    order = rng.permutation(len(joints))
    return ('<?xml version="1.0"?>\n<robot name="general{n}">\n' + "\n".join(links) + "\n"
            + "\n".join(joints[i] for i in order) + "\n</robot>\n").replace("{n}", str(n))


def tree_urdf(seed: int = 11, floating: bool = False) -> str:
    """Branching test model (RB_MODEL_URDF_TREE | RB_MODEL_GENERAL_AXES):
    a prismatic lift base -> torso, then three branches off the torso body -- a 3-joint arm
    (revolute, revolute, continuous), a 3-joint arm ending in a prismatic slide, and a
    2-joint head mounted on a massive fixed plate (a movable child of a merged fixed link).
    Random origins / axes / inertials, shuffled document order; 9 DOF.  floating=True: the
    torso itself is the root link (no world / base / lift) for RB_MODEL_FLOATING_BASE, 8 DOF
    + 6 virtual ones (a massless base below a prismatic lift would make H singular).
    The same seed gives the same torso and branches in both forms."""
    import numpy as np
    rng = np.random.default_rng(seed)

    def f(x):
        return " ".join(repr(float(v)) for v in x)

    def inertial(mass):
        a, b = rng.uniform(0.01, 0.05, 2)
        c = rng.uniform(abs(a - b) + 0.005, a + b - 0.001)
        return ("    <inertial>\n"
                f'      <origin rpy="{f(rng.uniform(-np.pi, np.pi, 3))}" xyz="{f(rng.uniform(-0.1, 0.1, 3))}"/>\n'
                f'      <mass value="{float(mass)!r}"/>\n'
                f'      <inertia ixx="{float(a)!r}" ixy="0" ixz="0" iyy="{float(b)!r}" iyz="0" izz="{float(c)!r}"/>\n'
                "    </inertial>")

    def axis():
        a = rng.normal(size=3)
        return a / np.linalg.norm(a)

    links, joints = [], []
    if not floating:
        links += ['  <link name="world"/>', '  <link name="base"/>']
        joints += ['  <joint name="world_joint" type="fixed">\n    <origin rpy="0 0 0" xyz="0 0 0.05"/>\n'
                   '    <parent link="world"/>\n    <child link="base"/>\n  </joint>']

    def joint(name, kind, parent, child, ax, lim):
        joints.append(f'  <joint name="{name}" type="{kind}">\n'
                      f'    <origin rpy="{f(rng.uniform(-np.pi, np.pi, 3))}" xyz="{f(rng.uniform(-0.2, 0.2, 3))}"/>\n'
                      f'    <parent link="{parent}"/>\n    <child link="{child}"/>\n    <axis xyz="{f(ax)}"/>\n'
                      f"{lim}\n  </joint>")

    def body(name, mass):
        links.append(f'  <link name="{name}">\n{inertial(mass)}\n  </link>')

    rev = '    <limit effort="40" lower="-2.5" upper="2.5" velocity="2.0"/>'
    cont = '    <limit effort="20" velocity="2.0"/>'
    slide = '    <limit effort="100" lower="-0.2" upper="0.2" velocity="0.5"/>'
    body("torso", 8.0)
    if not floating:
        joint("lift", "prismatic", "base", "torso", (0.0, 0.0, 1.0), slide)
    else:
        rng.uniform(-np.pi, np.pi, 3), rng.uniform(-0.2, 0.2, 3)  # keep the random stream aligned
    body("plate", 1.5)
    joints.append('  <joint name="plate_mount" type="fixed">\n'
                  f'    <origin rpy="{f(rng.uniform(-np.pi, np.pi, 3))}" xyz="0 0 0.3"/>\n'
                  '    <parent link="torso"/>\n    <child link="plate"/>\n  </joint>')
    parent = "torso"
    for k, kind in enumerate(("revolute", "revolute", "continuous")):
        body(f"la{k + 1}", rng.uniform(0.5, 2.0))
        joint(f"la_j{k + 1}", kind, parent, f"la{k + 1}", axis(), cont if kind == "continuous" else rev)
        parent = f"la{k + 1}"
    parent = "torso"
    for k, kind in enumerate(("revolute", "revolute", "prismatic")):
        body(f"ra{k + 1}", rng.uniform(0.5, 2.0))
        joint(f"ra_j{k + 1}", kind, parent, f"ra{k + 1}", axis(), slide if kind == "prismatic" else rev)
        parent = f"ra{k + 1}"
    parent = "plate"
    for k in range(2):
        body(f"head{k + 1}", rng.uniform(0.3, 1.0))
        joint(f"head_j{k + 1}", "revolute", parent, f"head{k + 1}", (0.0, 0.0, 1.0) if k == 0 else axis(), rev)
        parent = f"head{k + 1}"
    order = rng.permutation(len(joints))
    return ('<?xml version="1.0"?>\n<robot name="tree9">\n' + "\n".join(links) + "\n"
            + "\n".join(joints[i] for i in order) + "\n</robot>\n")


def input_ranges(limits, kind: str):
    """Per-joint (lo, hi) for kind in {'q','qd','qdd','tau'} from URDF limits (a joint
    without position limits -- continuous -- samples q in [-pi, pi])."""
    import math
    lower, upper, vel, eff = limits
    n = len(lower)
    if kind == "q":
        return ([-math.pi if math.isnan(x) else x for x in lower],
                [math.pi if math.isnan(x) else x for x in upper])
    if kind == "qd":
        return [-v for v in vel], list(vel)
    if kind == "qdd":
        return [-10.0] * n, [10.0] * n
    if kind == "tau":
        return [-e for e in eff], list(eff)
    raise ValueError(kind)


# splitmix64 counter generator, identical to the device fill (kinematics.hip)
_M64 = (1 << 64) - 1


def _splitmix64(z):
    import numpy as np
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def host_uniform(rows: int, batch: int, lo, hi, seed: int, dtype="float64", start: int = 0):
    """Host reproduction of rb_fill_uniform_* for configurations [start, start+batch)."""
    import numpy as np
    b = np.arange(start, start + batch, dtype=np.uint64)
    out = np.empty((rows, batch), dtype=dtype)
    with np.errstate(over="ignore"):
        base = np.uint64((seed * 0x9E3779B97F4A7C15) & _M64)
        for j in range(rows):
            idx = (np.uint64(j) << np.uint64(40)) | b
            u = _splitmix64(base + idx + np.uint64(1))
            if np.dtype(dtype) == np.float64:
                r = (u >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
            else:
                r = (u >> np.uint64(40)).astype(np.float64) * 2.0 ** -24
            out[j] = (lo[j] + (hi[j] - lo[j]) * r).astype(dtype)
    return out
