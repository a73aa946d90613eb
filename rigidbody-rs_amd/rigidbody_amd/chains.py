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


def input_ranges(limits, kind: str):
    """Per-joint (lo, hi) for kind in {'q','qd','qdd','tau'} from URDF limits."""
    lower, upper, vel, eff = limits
    n = len(lower)
    if kind == "q":
        return list(lower), list(upper)
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
