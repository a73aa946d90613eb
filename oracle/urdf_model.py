"""TEST INFRASTRUCTURE ONLY -- oracle-side URDF model extraction.

Restates how the reference turns a URDF into its `Multibody`:

* xurdf 0.2.5 (Cargo.lock:618-629; third-party, absent here) `parse_urdf_from_file`
  returns `Robot {links, joints}` holding the *top-level* `<link>` / `<joint>`
  children of `<robot>` in document order.  Nested `<joint>` tags inside
  `<transmission>` / `<gazebo>` are not robot joints.  Missing `<origin>` attributes
  default to zeros, a missing `<axis>` to (1, 0, 0), a missing `<inertial>` to zeros.
* `Multibody::from_urdf` (multibody.rs:65-77) zips `robot.joints` with `robot.links`
  BY INDEX and keeps every pair whose joint type does not contain "fixed".
* `RevoluteJoint::from_xurdf_joint` (joint.rs:53-68) takes the joint origin xyz/rpy,
  the axis, and the paired link's inertial mass, inertial-origin xyz (rpy ignored)
  and inertia tensor.

Returns raw arrays; the nalgebra conversions happen in oracle.c
(`oracle_model_from_raw`).  Independent of the product's C++ loader
(rigidbody-rs_amd/csrc/urdf.cpp), which tests compare against this.
"""
from __future__ import annotations

import xml.etree.ElementTree as ET

import numpy as np


def _vec(text, n=3, default=0.0):
    if text is None:
        return [default] * n
    vals = [float(t) for t in text.split()]
    if len(vals) != n:
        raise ValueError(f"expected {n} numbers, got {text!r}")
    return vals


def parse_robot(xml_text: str):
    """Top-level links and joints in document order (xurdf semantics)."""
    root = ET.fromstring(xml_text)
    if root.tag != "robot":
        raise ValueError("root element is not <robot>")
    links, joints = [], []
    for el in root:
        if el.tag == "link":
            inertial = el.find("inertial")
            if inertial is not None:
                org = inertial.find("origin")
                mass_el = inertial.find("mass")
                ine = inertial.find("inertia")
                com = _vec(org.get("xyz") if org is not None else None)
                com_rpy = _vec(org.get("rpy") if org is not None else None)
                mass = float(mass_el.get("value")) if mass_el is not None else 0.0
                if ine is not None:
                    i6 = [float(ine.get(k, "0")) for k in ("ixx", "ixy", "ixz", "iyy", "iyz", "izz")]
                else:
                    i6 = [0.0] * 6
            else:
                com, com_rpy, mass, i6 = [0.0] * 3, [0.0] * 3, 0.0, [0.0] * 6
            links.append({"name": el.get("name"), "mass": mass, "com": com, "com_rpy": com_rpy, "inertia6": i6})
        elif el.tag == "joint":
            org = el.find("origin")
            ax = el.find("axis")
            par = el.find("parent")
            chi = el.find("child")
            lim = el.find("limit")
            joints.append({
                "name": el.get("name"),
                "type": el.get("type", ""),
                "xyz": _vec(org.get("xyz") if org is not None else None),
                "rpy": _vec(org.get("rpy") if org is not None else None),
                "axis": _vec(ax.get("xyz") if ax is not None else None) if ax is not None else [1.0, 0.0, 0.0],
                "parent": par.get("link") if par is not None else None,
                "child": chi.get("link") if chi is not None else None,
                "mimic": el.find("mimic") is not None,
                "limit": None if lim is None else {k: float(lim.get(k)) for k in ("lower", "upper", "effort", "velocity") if lim.get(k) is not None},
            })
    return links, joints


def model_raw_from_urdf(xml_text: str):
    """multibody.rs:65-77 restated: index zip, skip joint types containing 'fixed'."""
    links, joints = parse_robot(xml_text)
    sel = []
    for joint, link in zip(joints, links):
        if "fixed" not in joint["type"]:
            sel.append((joint, link))
    n = len(sel)
    raw = {
        "n": n,
        "xyz": np.array([j["xyz"] for j, _ in sel], dtype=np.float64).reshape(n, 3),
        "rpy": np.array([j["rpy"] for j, _ in sel], dtype=np.float64).reshape(n, 3),
        "axis": np.array([j["axis"] for j, _ in sel], dtype=np.float64).reshape(n, 3),
        "mass": np.array([l["mass"] for _, l in sel], dtype=np.float64).reshape(n),
        "com": np.array([l["com"] for _, l in sel], dtype=np.float64).reshape(n, 3),
        "inertia6": np.array([l["inertia6"] for _, l in sel], dtype=np.float64).reshape(n, 6),
        "joint_names": [j["name"] for j, _ in sel],
        "link_names": [l["name"] for _, l in sel],
        "child_names": [j["child"] for j, _ in sel],
        "limits": [j["limit"] for j, _ in sel],
    }
    return raw


def index_pairing_matches_child(raw) -> bool:
    """the reference pairs by index; physically the body is the joint's child."""
    return list(raw["link_names"]) == list(raw["child_names"])


# ----------------------------------------------------------------------------------
# Physical-tree reading (RB_MODEL_URDF_TREE) -- beyond the
# reference, which pairs by index and drops fixed joints with their bodies.  Restated
# independently of rigidbody-rs_amd/csrc/model.cpp (chain_from_tree): plain 3x3
# matrices, inertia merged about the COM with the parallel-axis theorem.

def _rpy(r, p, y):
    cr, sr, cp, sp, cy, sy = np.cos(r), np.sin(r), np.cos(p), np.sin(p), np.cos(y), np.sin(y)
    return (np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]]) @ np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
            @ np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]]))


def _skew(v):
    return np.array([[0.0, -v[2], v[1]], [v[2], 0.0, -v[0]], [-v[1], v[0], 0.0]])


# Floating base (RB_MODEL_FLOATING_BASE): six massless virtual joints from the world to the
# root body -- prismatic x, y, z (world axes), then revolute z, y, x (yaw, pitch, roll: the
# root orientation is Rz Ry Rx, singular at pitch = +-pi/2).  Their "limits" only shape
# test / benchmark inputs (pitch kept within +-1.2 rad).
FLOAT_AXES = ((1.0, 0.0, 0.0), (0.0, 1.0, 0.0), (0.0, 0.0, 1.0), (0.0, 0.0, 1.0), (0.0, 1.0, 0.0), (1.0, 0.0, 0.0))
FLOAT_PRISMATIC = (1, 1, 1, 0, 0, 0)
FLOAT_LIMITS = tuple({"lower": lo, "upper": hi, "velocity": v, "effort": 1000.0}
                     for lo, hi, v in ((-1.0, 1.0, 1.0),) * 3 + ((-np.pi, np.pi, 2.0), (-1.2, 1.2, 2.0), (-np.pi, np.pi, 2.0)))
MOVABLE = ("revolute", "continuous", "prismatic")


def model_frames_from_urdf_tree(xml_text: str, floating: bool = False):
    """Kinematic tree by joint parent/child names from the root link; fixed joints merged.
    Links are numbered in depth-first preorder (a body's movable child joints in the order
    a stack walk of its fixed subtree meets them, each link's joints in document order), so
    parent[i] < i.  Returns dict(Rp [n,3,3], p [n,3], axis [n,3] (unit), mass [n],
    com [n,3], icom [n,3,3], parent [n], prismatic [n], limits [n]) -- body i is joint i's
    child link plus its fixed-joint subtree.  floating=True prepends the six virtual
    joints above and gives the root body to the last of them."""
    links, joints = parse_robot(xml_text)
    by_name = {l["name"]: l for l in links}
    children = [j["child"] for j in joints]
    roots = [l["name"] for l in links if l["name"] not in children]
    if len(roots) != 1:
        raise ValueError(f"expected one root link, got {roots}")

    def body(root_link):
        parts, movable = [], []  # (link, R, t) of the body's fixed subtree; its movable joints
        stack = [(root_link, np.eye(3), np.zeros(3))]
        while stack:
            ln, R, t = stack.pop()
            parts.append((by_name[ln], R, t))
            for j in joints:
                if j["parent"] != ln:
                    continue
                if j["mimic"]:
                    raise ValueError("mimic joint")
                Rj, tj = R @ _rpy(*j["rpy"]), t + R @ np.asarray(j["xyz"], float)
                if j["type"] == "fixed":
                    stack.append((j["child"], Rj, tj))
                elif j["type"] in MOVABLE:
                    movable.append((j, Rj, tj))
                else:
                    raise ValueError(f"joint type {j['type']}")
        m = sum(l["mass"] for l, _, _ in parts)
        c = sum(l["mass"] * (R @ np.asarray(l["com"], float) + t) for l, R, t in parts)
        c = c / m if m > 0 else np.zeros(3)
        Ic = np.zeros((3, 3))
        for l, R, t in parts:
            i6 = l["inertia6"]
            Il = np.array([[i6[0], i6[1], i6[2]], [i6[1], i6[3], i6[4]], [i6[2], i6[4], i6[5]]])
            Rin = R @ _rpy(*l["com_rpy"])
            d = R @ np.asarray(l["com"], float) + t - c
            Ic += Rin @ Il @ Rin.T + l["mass"] * (d @ d * np.eye(3) - np.outer(d, d))
        return (m, c, Ic), movable

    out = {k: [] for k in ("Rp", "p", "axis", "parent", "prismatic", "limits")}
    bodies = {}

    def add_link(R, t, axis, prismatic, parent, limits):
        a = np.asarray(axis, float)
        out["Rp"].append(R)
        out["p"].append(t)
        out["axis"].append(a / np.linalg.norm(a))
        out["parent"].append(parent)
        out["prismatic"].append(int(prismatic))
        out["limits"].append(limits)
        return len(out["Rp"]) - 1

    def visit(j, Rj, tj, parent):
        i = add_link(Rj, tj, j["axis"], j["type"] == "prismatic", parent, j["limit"])
        bodies[i], movable = body(j["child"])
        for jc, Rc, tc in movable:
            visit(jc, Rc, tc, i)

    root_body, movable = body(roots[0])
    base = -1
    if floating:
        for k in range(6):
            add_link(np.eye(3), np.zeros(3), FLOAT_AXES[k], FLOAT_PRISMATIC[k], k - 1, dict(FLOAT_LIMITS[k]))
            bodies[k] = (0.0, np.zeros(3), np.zeros((3, 3)))
        bodies[5] = root_body
        base = 5
    for j, Rj, tj in movable:
        visit(j, Rj, tj, base)
    n = len(out["Rp"])
    res = {k: np.array(out[k], dtype=np.float64) for k in ("Rp", "p", "axis")}
    res["parent"] = np.array(out["parent"], dtype=np.int32)
    res["prismatic"] = np.array(out["prismatic"], dtype=np.int32)
    res["mass"] = np.array([bodies[i][0] for i in range(n)], dtype=np.float64)
    res["com"] = np.array([bodies[i][1] for i in range(n)], dtype=np.float64).reshape(n, 3)
    res["icom"] = np.array([bodies[i][2] for i in range(n)], dtype=np.float64).reshape(n, 3, 3)
    res["limits"] = out["limits"]
    res["n"] = n
    return res
