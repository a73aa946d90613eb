"""TEST INFRASTRUCTURE ONLY -- independent 6x6 cross-check of the C restatement.

A second, structurally different formulation of the same dynamics, used to validate
oracle.c (which follows the reference's quaternion/isometry code path):

* rotations as 3x3 matrices built directly (Rz(y)Ry(p)Rx(r) and Rodrigues for the
  joint), never through quaternions or the axis-angle round trip of joint.rs:57-64;
* Featherstone 6x6 Pluecker matrices in the reference's [rot; lin] ordering
  (spatial.rs:137-149): motion transform B_X_A = [[E, 0], [-E r^, E]]
  (spatial.rs:32-47 form, E = parent->child rotation, r = child origin in parent),
  force transforms as its transpose, spatial inertia in the `to_matrix6` form
  (inertia.rs:53-70), motion/force cross-product matrices (Featherstone 2.31/2.32);
* RNEA and CRBA as Featherstone Tables 5.1 / 6.2, and the Articulated-Body
  Algorithm (Table 7.1) as an independent forward-dynamics check of the oracle's
  CRBA-solve definition.

Like the reference it injects joint motion about local z (multibody.rs:130-138)
and applies gravity as a +9.81 z base acceleration (multibody.rs:117-120).  With
general=True the motion subspace is the joint's own axis, S_i = [axis_i; 0] -- the
general-axis extension the reference does not have; this module
is then its only independent check.  Likewise for kinematic trees (frames["parent"]) and
prismatic joints (frames["prismatic"], S_i = [0; axis_i]): Featherstone's tree forms of
Tables 5.1 / 6.2 / 7.1 with the parent array lambda(i) < i.
"""
from __future__ import annotations

import numpy as np

G = 9.81


def skew(v):
    return np.array([[0.0, -v[2], v[1]], [v[2], 0.0, -v[0]], [-v[1], v[0], 0.0]])


def rpy_matrix(r, p, y):
    cr, sr, cp, sp, cy, sy = np.cos(r), np.sin(r), np.cos(p), np.sin(p), np.cos(y), np.sin(y)
    Rx = np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
    Ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
    Rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


def axis_angle_matrix(a, q):
    a = np.asarray(a, float) / np.linalg.norm(a)
    K = skew(a)
    return np.eye(3) + np.sin(q) * K + (1 - np.cos(q)) * (K @ K)


def xmotion(E, r):
    """B_X_A (spatial.rs:32-47 form) for E = rotation A->B coords, r = B origin in A."""
    X = np.zeros((6, 6))
    X[:3, :3] = E
    X[3:, 3:] = E
    X[3:, :3] = -E @ skew(r)
    return X


def inertia6(mass, com, icom):
    """Inertia::from_com (inertia.rs:21-35) then to_matrix6 (inertia.rs:53-70)."""
    C = skew(com)
    Io = icom + mass * C @ C.T
    M = np.zeros((6, 6))
    M[:3, :3] = Io
    M[:3, 3:] = mass * C
    M[3:, :3] = mass * C.T
    M[3:, 3:] = mass * np.eye(3)
    return M


def crm(v):
    M = np.zeros((6, 6))
    M[:3, :3] = skew(v[:3])
    M[3:, 3:] = skew(v[:3])
    M[3:, :3] = skew(v[3:])
    return M


def crf(v):
    return -crm(v).T


class Model6:
    def __init__(self, raw=None, general=False, frames=None):
        """raw: urdf_model.model_raw_from_urdf output; or frames = dict(Rp [n,3,3], p [n,3],
        axis [n,3], mass [n], com [n,3], icom [n,3,3]) (tree-mode reading)."""
        if frames is not None:
            self.n = len(frames["mass"])
            self.Rp = [np.asarray(frames["Rp"][i], float) for i in range(self.n)]
            self.p = [np.asarray(frames["p"][i], float) for i in range(self.n)]
            self.axis = [np.asarray(frames["axis"][i], float) for i in range(self.n)]
            self.I = [inertia6(frames["mass"][i], np.asarray(frames["com"][i], float),
                               np.asarray(frames["icom"][i], float)) for i in range(self.n)]
            self.parent = [int(x) for x in frames.get("parent", np.arange(self.n) - 1)]
            self.prismatic = [bool(x) for x in frames.get("prismatic", np.zeros(self.n))]
        else:
            self.n = int(raw["n"])
            self.Rp = [rpy_matrix(*raw["rpy"][i]) for i in range(self.n)]
            self.p = [np.asarray(raw["xyz"][i], float) for i in range(self.n)]
            self.axis = [np.asarray(raw["axis"][i], float) for i in range(self.n)]
            self.I = []
            for i in range(self.n):
                j = raw["inertia6"][i]
                ic = np.array([[j[0], j[1], j[2]], [j[1], j[3], j[4]], [j[2], j[4], j[5]]])
                self.I.append(inertia6(raw["mass"][i], np.asarray(raw["com"][i], float), ic))
            self.parent = list(range(-1, self.n - 1))
            self.prismatic = [False] * self.n
        self.S = []
        for i in range(self.n):
            a = self.axis[i] / np.linalg.norm(self.axis[i]) if general else np.array([0.0, 0.0, 1.0])
            self.S.append(np.concatenate([np.zeros(3), a] if self.prismatic[i] else [a, np.zeros(3)]))

    def poses(self, q):
        out = []
        for i in range(self.n):
            if self.prismatic[i]:
                a = self.axis[i] / np.linalg.norm(self.axis[i])
                out.append((self.Rp[i], self.p[i] + self.Rp[i] @ (a * q[i])))
            else:
                out.append((self.Rp[i] @ axis_angle_matrix(self.axis[i], q[i]), self.p[i]))
        return out

    def ancestors(self, i):
        """i, parent(i), ..., root."""
        out = []
        while i >= 0:
            out.append(i)
            i = self.parent[i]
        return out

    def xforms(self, q):
        return [xmotion(R.T, p) for R, p in self.poses(q)]

    def rnea(self, q, qd, qdd):
        X = self.xforms(q)
        v0, a0 = np.zeros(6), np.array([0, 0, 0, 0, 0, G], float)
        v, a, f = [None] * self.n, [None] * self.n, []
        for i in range(self.n):
            p = self.parent[i]
            vJ = self.S[i] * qd[i]
            v[i] = X[i] @ (v0 if p < 0 else v[p]) + vJ
            a[i] = X[i] @ (a0 if p < 0 else a[p]) + self.S[i] * qdd[i] + crm(v[i]) @ vJ
            f.append(self.I[i] @ a[i] + crf(v[i]) @ self.I[i] @ v[i])
        tau = np.zeros(self.n)
        for i in range(self.n - 1, -1, -1):
            tau[i] = self.S[i] @ f[i]
            if self.parent[i] >= 0:
                f[self.parent[i]] = f[self.parent[i]] + X[i].T @ f[i]
        return tau

    def crba(self, q):
        X = self.xforms(q)
        Ic = [M.copy() for M in self.I]
        for i in range(self.n - 1, -1, -1):
            if self.parent[i] >= 0:
                Ic[self.parent[i]] = Ic[self.parent[i]] + X[i].T @ Ic[i] @ X[i]
        H = np.zeros((self.n, self.n))
        for i in range(self.n):
            F = Ic[i] @ self.S[i]
            H[i, i] = self.S[i] @ F
            j = i
            while self.parent[j] >= 0:
                F = X[j].T @ F
                j = self.parent[j]
                H[i, j] = H[j, i] = self.S[j] @ F
        return H

    def aba(self, q, qd, tau):
        n = self.n
        X = self.xforms(q)
        v, c, IA, pA = [None] * n, [None] * n, [None] * n, [None] * n
        for i in range(n):
            vJ = self.S[i] * qd[i]
            v[i] = X[i] @ (np.zeros(6) if self.parent[i] < 0 else v[self.parent[i]]) + vJ
            c[i] = crm(v[i]) @ vJ
            IA[i] = self.I[i].copy()
            pA[i] = crf(v[i]) @ self.I[i] @ v[i]
        U, D, u = [None] * n, np.zeros(n), np.zeros(n)
        for i in range(n - 1, -1, -1):
            U[i] = IA[i] @ self.S[i]
            D[i] = self.S[i] @ U[i]
            u[i] = tau[i] - self.S[i] @ pA[i]
            p = self.parent[i]
            if p >= 0:
                Ia = IA[i] - np.outer(U[i], U[i]) / D[i]
                pa = pA[i] + Ia @ c[i] + U[i] * u[i] / D[i]
                IA[p] = IA[p] + X[i].T @ Ia @ X[i]
                pA[p] = pA[p] + X[i].T @ pa
        qdd = np.zeros(n)
        a = [None] * n
        for i in range(n):
            p = self.parent[i]
            a[i] = X[i] @ (np.array([0, 0, 0, 0, 0, G], float) if p < 0 else a[p]) + c[i]
            qdd[i] = (u[i] - U[i] @ a[i]) / D[i]
            a[i] = a[i] + self.S[i] * qdd[i]
        return qdd

    def fwd_kin(self, q):
        R, p = np.eye(3), np.zeros(3)
        poses = self.poses(q)
        for i in reversed(self.ancestors(self.n - 1)):  # root -> last link
            Ri, pi = poses[i]
            p = p + R @ pi
            R = R @ Ri
        return p

    def jac(self, q):
        """Body Jacobian of the last link, rows [lin; rot] (multibody.rs:95-108); columns of
        joints off its path to the root are zero."""
        poses = self.poses(q)
        n = self.n
        J = np.zeros((6, n))
        R, p = np.eye(3), np.zeros(3)  # pose of the last frame in frame i (built backwards)
        for i in self.ancestors(n - 1):
            # joint-i axis z in frame i, expressed at/in the last frame: X(R^T, p) applied to S
            X = xmotion(R.T, p)
            sv = X @ self.S[i]
            J[:3, i] = sv[3:]
            J[3:, i] = sv[:3]
            Ri, pi = poses[i]
            p = pi + Ri @ p
            R = Ri @ R
        return J
