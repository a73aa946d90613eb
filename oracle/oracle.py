"""TEST INFRASTRUCTURE ONLY -- ctypes front-end of the fp64 CPU restatement (oracle.c).

Used by tests/ (as the parity checker), __graft_entry__.smoke() (as the checker) and
bench.py's cpu_baseline leg (as the timed "port" baseline).  The product library never
imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# ORACLE_LIB: an alternative build of the same source (the ASan/UBSan one, `make sanitize`)
_LIB_PATH = os.environ.get("ORACLE_LIB") or os.path.join(_HERE, "liboracle.so")
_lib = None

_dp = ctypes.POINTER(ctypes.c_double)


def build(force: bool = False) -> str:
    if os.environ.get("ORACLE_LIB"):
        return _LIB_PATH
    if force or not os.path.exists(_LIB_PATH) or (
        os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "oracle.c"))
    ):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_model_size.restype = ctypes.c_int
        L.oracle_model_from_raw.restype = ctypes.c_int
        L.oracle_model_from_raw.argtypes = [ctypes.c_void_p, ctypes.c_int] + [_dp] * 6
        for name in ("oracle_rnea",):
            getattr(L, name).argtypes = [ctypes.c_void_p, _dp, _dp, _dp, _dp]
        L.oracle_crba.argtypes = [ctypes.c_void_p, _dp, _dp]
        L.oracle_fwd_kin.argtypes = [ctypes.c_void_p, _dp, _dp]
        L.oracle_jac.argtypes = [ctypes.c_void_p, _dp, _dp]
        L.oracle_fd.argtypes = [ctypes.c_void_p, _dp, _dp, _dp, _dp]
        L.oracle_fd.restype = ctypes.c_int
        L.oracle_rnea_batch.argtypes = [ctypes.c_void_p, _dp, _dp, _dp, _dp, ctypes.c_long, ctypes.c_long, ctypes.c_int]
        L.oracle_fd_batch.argtypes = [ctypes.c_void_p, _dp, _dp, _dp, _dp, ctypes.c_long, ctypes.c_long, ctypes.c_int]
        L.oracle_crba_batch.argtypes = [ctypes.c_void_p, _dp, _dp, ctypes.c_long, ctypes.c_long, ctypes.c_int]
        L.oracle_rollout_batch.argtypes = [ctypes.c_void_p, _dp, _dp, _dp, ctypes.c_double, ctypes.c_int, _dp,
                                           ctypes.c_long, ctypes.c_long, ctypes.c_int]
        L.oracle_model_from_frames.restype = ctypes.c_int
        L.oracle_model_from_frames.argtypes = [ctypes.c_void_p, ctypes.c_int] + [_dp] * 6
        L.oracle_model_set_general_axes.argtypes = [ctypes.c_void_p, ctypes.c_int]
        _ip = ctypes.POINTER(ctypes.c_int)
        L.oracle_model_set_topology.restype = ctypes.c_int
        L.oracle_model_set_topology.argtypes = [ctypes.c_void_p, _ip, _ip]
        L.oracle_quat_from_scaled_axis.argtypes = [_dp, _dp]
        L.oracle_quat_from_axis_angle.argtypes = [_dp, ctypes.c_double, _dp]
        L.oracle_quat_to_matrix.argtypes = [_dp, _dp]
        L.oracle_rotation_from_euler.argtypes = [ctypes.c_double] * 3 + [_dp]
        L.oracle_rotation_scaled_axis.argtypes = [_dp, _dp]
        L.oracle_motion_transform.argtypes = [_dp] * 5
        L.oracle_force_transform.argtypes = [_dp] * 5
        L.oracle_iso_inverse.argtypes = [_dp, _dp]
        L.oracle_quat_rotate.argtypes = [_dp, _dp, _dp]
        L.oracle_parent_to_child.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_double, _dp]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"], (a.dtype, a.flags)
    return a.ctypes.data_as(_dp)


def _c(a):
    return np.ascontiguousarray(a, dtype=np.float64)


class Model:
    """fp64 oracle model built from raw URDF values (oracle/urdf_model.py).

    general=True: motion subspace along each joint's own axis (oracle.h general_axes);
    frames=...: the tree-mode reading (urdf_model.model_frames_from_urdf_tree), whose
    optional "parent" / "prismatic" entries give a kinematic tree and joint types."""

    def __init__(self, raw=None, general=False, frames=None):
        L = lib()
        self._buf = ctypes.create_string_buffer(L.oracle_model_size())
        if frames is not None:
            self.n = int(frames["n"])
            arrs = [_c(frames[k]) for k in ("Rp", "p", "axis", "mass", "com", "icom")]
            self._keep = arrs
            rc = L.oracle_model_from_frames(self._buf, self.n, *[_p(a) for a in arrs])
        else:
            self.n = int(raw["n"])
            arrs = [_c(raw[k]) for k in ("xyz", "rpy", "axis", "mass", "com", "inertia6")]
            self._keep = arrs
            rc = L.oracle_model_from_raw(self._buf, self.n, *[_p(a) for a in arrs])
        if rc != 0:
            raise ValueError(f"oracle model construction failed: {rc}")
        L.oracle_model_set_general_axes(self._buf, int(bool(general)))
        if frames is not None and ("parent" in frames or "prismatic" in frames):
            par = np.ascontiguousarray(frames.get("parent", np.arange(self.n) - 1), dtype=np.int32)
            pri = np.ascontiguousarray(frames.get("prismatic", np.zeros(self.n)), dtype=np.int32)
            self._keep += [par, pri]
            _ip = ctypes.POINTER(ctypes.c_int)
            if L.oracle_model_set_topology(self._buf, par.ctypes.data_as(_ip), pri.ctypes.data_as(_ip)) != 0:
                raise ValueError("bad tree topology")
        self.parent = (np.asarray(frames["parent"], int) if frames is not None and "parent" in frames
                       else np.arange(self.n) - 1)

    @property
    def ptr(self):
        return ctypes.cast(self._buf, ctypes.c_void_p)

    # ---- single configuration -------------------------------------------------
    def rnea(self, q, qd, qdd):
        out = np.zeros(self.n)
        lib().oracle_rnea(self.ptr, _p(_c(q)), _p(_c(qd)), _p(_c(qdd)), _p(out))
        return out

    def crba(self, q):
        H = np.zeros(self.n * self.n)
        lib().oracle_crba(self.ptr, _p(_c(q)), _p(H))
        return H.reshape(self.n, self.n).T.copy()  # column-major buffer -> matrix

    def crba_raw(self, q):
        H = np.zeros(self.n * self.n)
        lib().oracle_crba(self.ptr, _p(_c(q)), _p(H))
        return H

    def fwd_kin(self, q):
        out = np.zeros(3)
        lib().oracle_fwd_kin(self.ptr, _p(_c(q)), _p(out))
        return out

    def jac_raw(self, q):
        J = np.zeros(6 * self.n)
        lib().oracle_jac(self.ptr, _p(_c(q)), _p(J))
        return J

    def jac(self, q):
        return self.jac_raw(q).reshape(self.n, 6).T.copy()

    def fd(self, q, qd, tau):
        out = np.zeros(self.n)
        rc = lib().oracle_fd(self.ptr, _p(_c(q)), _p(_c(qd)), _p(_c(tau)), _p(out))
        if rc != 0:
            raise ValueError("mass matrix not SPD")
        return out

    def parent_to_child(self, i, qi):
        out = np.zeros(7)
        lib().oracle_parent_to_child(self.ptr, int(i), float(qi), _p(out))
        return out

    # ---- batched SoA [n, B] ---------------------------------------------------
    def rnea_batch(self, q, qd, qdd, nthreads=0):
        q, qd, qdd = _c(q), _c(qd), _c(qdd)
        B = q.shape[1]
        tau = np.empty_like(q)
        lib().oracle_rnea_batch(self.ptr, _p(q), _p(qd), _p(qdd), _p(tau), B, B, int(nthreads))
        return tau

    def fd_batch(self, q, qd, tau, nthreads=0):
        q, qd, tau = _c(q), _c(qd), _c(tau)
        B = q.shape[1]
        qdd = np.empty_like(q)
        lib().oracle_fd_batch(self.ptr, _p(q), _p(qd), _p(tau), _p(qdd), B, B, int(nthreads))
        return qdd

    def rollout_batch(self, q, qd, tau_seq, dt, want_traj=False, nthreads=0):
        """K semi-implicit Euler steps; q, qd [n, B]; tau_seq [K, n, B].  Returns
        (q_K, qd_K, traj [K, n, B] or None)."""
        q, qd, tau_seq = _c(q).copy(), _c(qd).copy(), _c(tau_seq)
        K, n, B = tau_seq.shape
        traj = np.empty((K, n, B)) if want_traj else None
        lib().oracle_rollout_batch(self.ptr, _p(q), _p(qd), _p(tau_seq), float(dt), int(K),
                                   _p(traj) if traj is not None else None, B, B, int(nthreads))
        return q, qd, traj

    def crba_batch(self, q, nthreads=0):
        q = _c(q)
        B = q.shape[1]
        H = np.empty((self.n * self.n, B))
        lib().oracle_crba_batch(self.ptr, _p(q), _p(H), B, B, int(nthreads))
        return H


# ---- op counts of the reference formulation (oracle/flops.cpp) ---------------
_flops = None


def flops_lib():
    """The op-counting build of oracle.c: same symbols, same binary layout (FlopD = one double)."""
    global _flops
    if _flops is None:
        path = os.path.join(_HERE, "liboracle_flops.so")
        if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(os.path.join(_HERE, "oracle.c")):
            subprocess.run(["make", "-s", "-C", _HERE, "liboracle_flops.so"], check=True)
        L = ctypes.CDLL(path)
        L.oracle_rnea.argtypes = [ctypes.c_void_p, _dp, _dp, _dp, _dp]
        L.oracle_crba.argtypes = [ctypes.c_void_p, _dp, _dp]
        L.oracle_fd.argtypes = [ctypes.c_void_p, _dp, _dp, _dp, _dp]
        L.oracle_fd.restype = ctypes.c_int
        L.oracle_flops_get.argtypes = [ctypes.POINTER(ctypes.c_long)]
        _flops = L
    return _flops


def op_counts(model: "Model", kind: str, q, qd=None, x=None) -> dict:
    """Operations the reference's formulation executes for ONE evaluation (oracle.c under the
    counting type): kind 'rnea' (x = qdd), 'crba', 'fd' (x = tau; the CRBA + RNEA(q, qd, 0) +
    Cholesky definition).  flops = add + mul + div (+ sqrt); trig separate."""
    L = flops_lib()
    n = model.n
    q = _c(q)
    qd = _c(np.zeros(n) if qd is None else qd)
    x = _c(np.zeros(n) if x is None else x)
    out = np.zeros(n * n)
    L.oracle_flops_reset()
    if kind == "rnea":
        L.oracle_rnea(model.ptr, _p(q), _p(qd), _p(x), _p(out))
    elif kind == "crba":
        L.oracle_crba(model.ptr, _p(q), _p(out))
    elif kind == "fd":
        L.oracle_fd(model.ptr, _p(q), _p(qd), _p(x), _p(out))
    else:
        raise ValueError(kind)
    c = (ctypes.c_long * 5)()
    L.oracle_flops_get(c)
    add, mul, div, sq, trig = (int(v) for v in c)
    return {"add": add, "mul": mul, "div": div, "sqrt": sq, "trig": trig, "flops": add + mul + div + sq,
            "result": out[:n * n if kind == "crba" else n].copy()}


# ---- primitives for the restated reference unit tests -----------------------
def quat_from_scaled_axis(v):
    out = np.zeros(4)
    lib().oracle_quat_from_scaled_axis(_p(_c(v)), _p(out))
    return out


def quat_from_axis_angle(axis, angle):
    out = np.zeros(4)
    lib().oracle_quat_from_axis_angle(_p(_c(axis)), float(angle), _p(out))
    return out


def quat_to_matrix(q):
    out = np.zeros(9)
    lib().oracle_quat_to_matrix(_p(_c(q)), _p(out))
    return out.reshape(3, 3)


def rotation_from_euler(r, p, y):
    out = np.zeros(9)
    lib().oracle_rotation_from_euler(float(r), float(p), float(y), _p(out))
    return out.reshape(3, 3)


def rotation_scaled_axis(R):
    out = np.zeros(3)
    lib().oracle_rotation_scaled_axis(_p(_c(np.asarray(R).reshape(9))), _p(out))
    return out


def iso(q, t):
    return _c(np.concatenate([np.asarray(q, float), np.asarray(t, float)]))


def motion_transform(iso7, lin, rot):
    ol, orr = np.zeros(3), np.zeros(3)
    lib().oracle_motion_transform(_p(_c(iso7)), _p(_c(lin)), _p(_c(rot)), _p(ol), _p(orr))
    return ol, orr


def force_transform(iso7, lin, rot):
    ol, orr = np.zeros(3), np.zeros(3)
    lib().oracle_force_transform(_p(_c(iso7)), _p(_c(lin)), _p(_c(rot)), _p(ol), _p(orr))
    return ol, orr


def iso_inverse(iso7):
    out = np.zeros(7)
    lib().oracle_iso_inverse(_p(_c(iso7)), _p(out))
    return out


def quat_rotate(q, v):
    out = np.zeros(3)
    lib().oracle_quat_rotate(_p(_c(q)), _p(_c(v)), _p(out))
    return out
