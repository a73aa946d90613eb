"""ctypes binding of librigidbody_bindings.so (include/rigidbody.h + rigidbody_batch.h).

Host-side mirror of the reference's interface for the hot path:

* `Multibody.new()` / `.from_urdf(path)` / `.from_urdf_string(xml)` <- `multibody_new`,
  `Multibody::from_urdf` (rigidbody_bindings/src/lib.rs:8-12, multibody.rs:65-77)
* `.rnea(q, dq, ddq)`, `.crba(q)`, `.fwd_kin(q)`, `.jac(q)` <- the single-config C ABI
  (lib.rs:15-70), same argument meaning and result layout; computed on the calling thread
  with the GPU lane bodies compiled for the host (`.single_config_path()`), or on the GPU
* `.rnea_batch`, `.fd_batch`, `.crba_batch`, `.fwd_kin_batch`, `.jac_batch` <- batched
  device-pointer entry points on torch CUDA tensors laid out [n, B] (SoA)

Errors: the reference panics (aborting across FFI) on a bad URDF, a wrong DOF or a
NULL handle; here every failure raises RigidBodyError with the library's message.

torch is imported before the library is loaded on purpose: torch ships its own
libamdhip64.so.7 and the dynamic loader then binds this library to that same
runtime (same SONAME), so torch tensors, streams and these kernels share one HIP
runtime.  There is no CPU fallback: if the library is missing this import fails.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch  # noqa: F401  -- must precede the CDLL load (shared HIP runtime)

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("RIGIDBODY_AMD_LIB", os.path.join(_PKG, "librigidbody_bindings.so"))

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"{LIB_PATH} not found: build the HIP library first (python -c 'import __graft_entry__ as g; g.build()' "
        "or make -C rigidbody-rs_amd)")

_lib = ctypes.CDLL(LIB_PATH)

_dp = ctypes.POINTER(ctypes.c_double)
_vp = ctypes.c_void_p
_i64 = ctypes.c_int64

# exported symbols declared in include/*.h (tests check the list against the headers)
REFERENCE_SYMBOLS = ["multibody_new", "multibody_fwd_kin", "multibody_jac", "multibody_rnea",
                     "multibody_crba", "multibody_free"]


def _sig(name, restype, argtypes):
    f = getattr(_lib, name)
    f.restype = restype
    f.argtypes = argtypes
    return f


_sig("multibody_new", _vp, [])
_sig("multibody_free", None, [_vp])
for _n in ("multibody_fwd_kin", "multibody_jac", "multibody_crba"):
    _sig(_n, _dp, [_vp, _dp])
_sig("multibody_rnea", _dp, [_vp, _dp, _dp, _dp])
_sig("multibody_new_from_urdf", _vp, [ctypes.c_char_p])
_sig("multibody_new_from_urdf_string", _vp, [ctypes.c_char_p, ctypes.c_size_t])
_sig("multibody_new_from_urdf_ex", _vp, [ctypes.c_char_p, ctypes.c_uint])
_sig("multibody_new_from_urdf_string_ex", _vp, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint])
_sig("multibody_flags", ctypes.c_uint, [_vp])
_sig("multibody_blob_size", _i64, [_vp])
_sig("multibody_export_blob", ctypes.c_int, [_vp, _dp, _i64])
_sig("multibody_new_from_blob", _vp, [_dp, _i64])
_sig("multibody_dof", ctypes.c_int, [_vp])
_sig("multibody_total_mass", ctypes.c_double, [_vp])
_sig("multibody_limits", ctypes.c_int, [_vp, _dp, _dp, _dp, _dp])
_sig("multibody_supported_dofs", ctypes.c_int, [ctypes.POINTER(ctypes.c_int), ctypes.c_int])
_sig("multibody_upload", ctypes.c_int, [_vp])
_sig("multibody_result_free", None, [_dp])
_sig("rb_last_error", ctypes.c_char_p, [])
_sig("rb_version", ctypes.c_char_p, [])
for _t in ("f32", "f64"):
    _sig(f"multibody_rnea_batch_{_t}", ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _vp])
    _sig(f"multibody_fd_batch_{_t}", ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _vp])
    _sig(f"multibody_crba_batch_{_t}", ctypes.c_int, [_vp, _vp, _vp, _i64, _i64, _vp])
    _sig(f"rb_fill_uniform_{_t}", ctypes.c_int, [_vp, ctypes.c_int, _i64, _i64, _dp, _dp, ctypes.c_uint64, _vp])
    _sig(f"multibody_rnea_fd_batch_{_t}", ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _vp])
    _sig(f"multibody_rnea_fd_batch_tiled_{_t}", ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp])
_sig("multibody_fwd_kin_batch_f64", ctypes.c_int, [_vp, _vp, _vp, _i64, _i64, _vp])
_sig("multibody_fwd_kin_batch_f32", ctypes.c_int, [_vp, _vp, _vp, _i64, _i64, _vp])
_sig("multibody_jac_batch_f32", ctypes.c_int, [_vp, _vp, _vp, _i64, _i64, _vp])
_sig("multibody_jac_batch_f64", ctypes.c_int, [_vp, _vp, _vp, _i64, _i64, _vp])
_sig("multibody_rnea_batch_host_f64", ctypes.c_int, [_vp, _dp, _dp, _dp, _dp, _i64])
_fp = ctypes.POINTER(ctypes.c_float)
_sig("multibody_rnea_batch_host_f32", ctypes.c_int, [_vp, _fp, _fp, _fp, _fp, _i64])
_sig("multibody_fd_batch_host_f32", ctypes.c_int, [_vp, _fp, _fp, _fp, _fp, _i64])
_sig("multibody_rnea_kernel_path", ctypes.c_int, [_vp, ctypes.c_int])
_sig("multibody_single_config_path", ctypes.c_int, [_vp])
_sig("multibody_kernel_path", ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int])
_sig("multibody_kernel_path_ex", ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _i64, ctypes.c_int])
_sig("multibody_kernel_form_ex", ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _i64, ctypes.c_int])
_sig("multibody_jit_source", ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_char_p, _i64])
_sig("multibody_jit_compile", _i64, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_char_p])
_sig("multibody_jit_source_ex", ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _i64, ctypes.c_int, ctypes.c_char_p, _i64])
_sig("multibody_jit_compile_ex", _i64, [_vp, ctypes.c_int, ctypes.c_int, _i64, ctypes.c_int, ctypes.c_char_p])
KINDS = {"rnea": 0, "fd": 1, "crba": 2, "rollout": 3, "fwd_kin": 4, "jac": 5, "rnea_fd": 6}
GENERAL_AXES, URDF_TREE, FLOATING_BASE = 1, 2, 4  # rigidbody_batch.h RB_MODEL_*
_ip = ctypes.POINTER(ctypes.c_int)
_sig("multibody_topology", ctypes.c_int, [_vp, _ip, _ip])
for _t in ("f32", "f64"):
    _sig(f"multibody_rollout_batch_{_t}", ctypes.c_int,
         [_vp, _vp, _vp, _vp, ctypes.c_double, ctypes.c_int, _vp, _i64, _i64, _vp])
_sig("rb_set_tuning", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int])
_sig("multibody_fd_batch_host_f64", ctypes.c_int, [_vp, _dp, _dp, _dp, _dp, _i64])
_sig("multibody_rnea_fd_batch_host_f64", ctypes.c_int, [_vp, _dp, _dp, _dp, _dp, _dp, _dp, _i64])
_sig("multibody_rnea_fd_batch_host_f32", ctypes.c_int, [_vp, _fp, _fp, _fp, _fp, _fp, _fp, _i64])
for _t in ("f32", "f64"):
    _sig(f"multibody_rnea_batch_tiled_{_t}", ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _i64, _vp])
    _sig(f"multibody_fd_batch_tiled_{_t}", ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _i64, _vp])
    _sig(f"rb_to_tiled_{_t}", ctypes.c_int, [_vp, _i64, _vp, ctypes.c_int, _i64, _vp])
    for _k in ("crba", "fwd_kin", "jac"):
        _sig(f"multibody_{_k}_batch_tiled_{_t}", ctypes.c_int, [_vp, _vp, _vp, _i64, _vp])
    _sig(f"rb_from_tiled_{_t}", ctypes.c_int, [_vp, _vp, _i64, ctypes.c_int, _i64, _vp])
TILE = 256  # configurations per tile of the tiled layout (rigidbody_batch.h)


class RigidBodyError(RuntimeError):
    pass


def last_error() -> str:
    return (_lib.rb_last_error() or b"").decode()


def version() -> str:
    return _lib.rb_version().decode()


def lib():
    return _lib


def supported_dofs():
    buf = (ctypes.c_int * 64)()
    n = _lib.multibody_supported_dofs(buf, 64)
    return [buf[i] for i in range(n)]


def set_tuning(key: str, value: int):
    """rb_set_tuning: process-wide knobs -- production "jit", "pack", "rnea_stream",
    "single_gpu"; the A/B selectors only with RB_EXPERIMENTAL=1 (csrc/tuning.hpp)."""
    _check(_lib.rb_set_tuning(key.encode(), int(value)), f"set_tuning({key})")


def _check(rc, what):
    if rc != 0:
        raise RigidBodyError(f"{what} failed (status {rc}): {last_error()}")


def _dvec(x, n):
    a = np.ascontiguousarray(x, dtype=np.float64)
    if a.shape != (n,):
        raise ValueError(f"expected {n} values, got shape {a.shape}")
    return a


def _take(ptr, count):
    if not ptr:
        raise RigidBodyError(last_error())
    out = np.ctypeslib.as_array(ptr, shape=(count,)).copy()
    _lib.multibody_result_free(ptr)
    return out


_TORCH_SUFFIX = {torch.float32: "f32", torch.float64: "f64"}


def _stream_ptr(stream, device=None):
    """The HIP stream a call is enqueued on: `stream`, else the current stream of `device`."""
    if stream is None:
        stream = torch.cuda.current_stream(device)
    elif device is not None and stream.device != device:
        raise ValueError(f"stream is on {stream.device}, the arrays on {device}")
    return ctypes.c_void_p(stream.cuda_stream)


def _one_device(ts):
    """All arrays of one call must live on one device: the library uploads the model and
    launches on the CURRENT device (hipGetDevice), so the caller makes it theirs
    (`with torch.cuda.device(dev)` around the call)."""
    devs = {t.device for t in ts}
    if len(devs) != 1:
        raise ValueError(f"all arrays of one call must be on one device, got {sorted(map(str, devs))}")
    return devs.pop()


def _host_soa(arrs, n, dtype):
    """[n, B] host arrays of one batched host call: same shape, n rows, converted to `dtype`
    (float64, the reference's Real, or float32 for the *_host_f32 entry points)."""
    dt = np.dtype(dtype)
    if dt not in (np.dtype(np.float64), np.dtype(np.float32)):
        raise TypeError(f"dtype must be float64 or float32, got {dt}")
    out = [np.ascontiguousarray(x, dtype=dt) for x in arrs]
    for a in out:
        if a.ndim != 2 or a.shape[0] != n or a.shape != out[0].shape:
            raise ValueError(f"host batch arrays must all be [{n}, B], got {[x.shape for x in out]}")
    return out


def _soa(t, n, name, dtype=None, B=None):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TypeError(f"{name} must be a CUDA (HIP) torch tensor of shape [n, B]")
    if t.dim() != 2 or t.shape[0] != n:
        raise ValueError(f"{name} must have shape [{n}, B], got {tuple(t.shape)}")
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"{name} has dtype {t.dtype}, expected {dtype}")
    if B is not None and t.shape[1] != B:
        raise ValueError(f"{name} has batch {t.shape[1]}, expected {B}")
    if t.shape[1] > 1 and t.stride(1) != 1:
        raise ValueError(f"{name} must be contiguous along the batch axis")
    return t


def _ld(t):
    """Leading dimension (row stride in elements) of an [n, B] tensor."""
    if t.shape[1] == 0:
        return 1
    ld = t.stride(0) if t.shape[0] > 1 else t.shape[1]
    if ld < t.shape[1]:
        raise ValueError("rows of an [n, B] array must not overlap (row stride < B)")
    return ld


def _same_ld(ts):
    lds = {_ld(t) for t in ts}
    if len(lds) != 1:
        raise ValueError("all [n, B] arrays of one call must share the leading dimension")
    return lds.pop()


def _kin_out(out, rows, q):
    """Output of fwd_kin / jac batches: [rows, B] of q's dtype with the input's leading dimension."""
    B = q.shape[1]
    if not isinstance(out, torch.Tensor) or out.dtype != q.dtype or tuple(out.shape) != (rows, B) or \
            (B > 1 and (out.stride(1) != 1 or out.stride(0) != _ld(q))):
        raise ValueError(f"out must be a {q.dtype} [{rows}, {B}] tensor with the input's leading dimension")


class Multibody:
    """Handle to a loaded serial chain (reference: `Multibody`, multibody.rs:32)."""

    def __init__(self, handle):
        if not handle:
            raise RigidBodyError(last_error())
        self._h = ctypes.c_void_p(handle)
        self.n = _lib.multibody_dof(self._h)

    # ------------------------------------------------------------------ construction
    @classmethod
    def new(cls):
        """multibody_new(): $RIGIDBODY_URDF, else the embedded FR3 model."""
        return cls(_lib.multibody_new())

    @classmethod
    def from_urdf(cls, path, flags: int = 0):
        """flags: GENERAL_AXES | URDF_TREE | FLOATING_BASE (rigidbody_batch.h RB_MODEL_*); 0 = the
        reference's reading."""
        if flags:
            return cls(_lib.multibody_new_from_urdf_ex(os.fsencode(path), flags))
        return cls(_lib.multibody_new_from_urdf(os.fsencode(path)))

    @classmethod
    def from_urdf_string(cls, xml: str, flags: int = 0):
        b = xml.encode()
        if flags:
            return cls(_lib.multibody_new_from_urdf_string_ex(b, len(b), flags))
        return cls(_lib.multibody_new_from_urdf_string(b, len(b)))

    @property
    def flags(self) -> int:
        return int(_lib.multibody_flags(self._h))

    @classmethod
    def from_blob(cls, blob):
        a = np.ascontiguousarray(blob, dtype=np.float64)
        return cls(_lib.multibody_new_from_blob(a.ctypes.data_as(_dp), a.size))

    def blob(self) -> np.ndarray:
        size = _lib.multibody_blob_size(self._h)
        out = np.zeros(size, dtype=np.float64)
        _check(_lib.multibody_export_blob(self._h, out.ctypes.data_as(_dp), size), "export_blob")
        return out

    def close(self):
        if getattr(self, "_h", None):
            _lib.multibody_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    @property
    def total_mass(self) -> float:
        return _lib.multibody_total_mass(self._h)

    def limits(self):
        arrs = [np.zeros(self.n) for _ in range(4)]
        _check(_lib.multibody_limits(self._h, *[a.ctypes.data_as(_dp) for a in arrs]), "limits")
        return tuple(arrs)  # lower, upper, velocity, effort

    def topology(self):
        """(parent [n] (-1 = base), joint_type [n] (0 revolute, 1 prismatic))."""
        par, typ = np.zeros(self.n, dtype=np.int32), np.zeros(self.n, dtype=np.int32)
        _check(_lib.multibody_topology(self._h, par.ctypes.data_as(_ip), typ.ctypes.data_as(_ip)), "topology")
        return par, typ

    def upload(self):
        _check(_lib.multibody_upload(self._h), "upload")

    def kernel_path(self, kind="rnea", f64=False, batch=1 << 20, tiled=False) -> str:
        """'jit' if the model-specialised hipRTC kernel of `kind` runs on this device for a
        launch of `batch` configurations (tiled: the *_tiled entry points)."""
        r = _lib.multibody_kernel_path_ex(self._h, KINDS[kind], int(bool(f64)), int(batch), int(bool(tiled)))
        if r < 0:
            raise RigidBodyError(last_error())
        return "jit" if r == 1 else "generic"

    def kernel_form(self, kind="rnea", f64=False, batch=1 << 20, tiled=False) -> int:
        """Configurations-per-lane form of the kernel such a launch takes (rigidbody_batch.h
        multibody_kernel_form_ex): 0 generic, 1 one per lane, 2 packed pair, 3 sequential pair,
        4 / 5 the packed / one-per-lane wave split."""
        r = _lib.multibody_kernel_form_ex(self._h, KINDS[kind], int(bool(f64)), int(batch), int(bool(tiled)))
        if r < 0:
            raise RigidBodyError(last_error())
        return r

    def single_config_path(self) -> str:
        """'host' when the single-configuration queries (rnea, crba, fwd_kin, jac) run on the
        calling thread (host_eval.cpp), 'gpu' when each is a GPU launch."""
        r = _lib.multibody_single_config_path(self._h)
        if r < 0:
            raise RigidBodyError(last_error())
        return "host" if r == 0 else "gpu"

    def rnea_kernel_path(self, f64=False) -> str:
        return self.kernel_path("rnea", f64)

    def jit_source(self, f64=False, kind="rnea", batch=1 << 20, tiled=False) -> str:
        """hipRTC source of the kernel a launch of `batch` configurations takes (tiled: the
        *_tiled entry points) -- multibody_jit_source_ex."""
        k, f, b, t = KINDS[kind], int(bool(f64)), int(batch), int(bool(tiled))
        n = _lib.multibody_jit_source_ex(self._h, k, f, b, t, None, 0)
        if n < 0:
            raise RigidBodyError(last_error())
        buf = ctypes.create_string_buffer(n + 1)
        _lib.multibody_jit_source_ex(self._h, k, f, b, t, buf, n + 1)
        return buf.value.decode()

    def jit_compile(self, f64=False, arch="gfx950", kind="rnea", batch=1 << 20, tiled=False) -> int:
        r = _lib.multibody_jit_compile_ex(self._h, KINDS[kind], int(bool(f64)), int(batch), int(bool(tiled)),
                                          arch.encode())
        if r < 0:
            raise RigidBodyError(last_error())
        return r

    # ------------------------------------------------- single configuration (ABI)
    def rnea(self, q, dq, ddq) -> np.ndarray:
        q, dq, ddq = (_dvec(x, self.n) for x in (q, dq, ddq))
        return _take(_lib.multibody_rnea(self._h, q.ctypes.data_as(_dp), dq.ctypes.data_as(_dp),
                                         ddq.ctypes.data_as(_dp)), self.n)

    def crba_raw(self, q) -> np.ndarray:
        """n*n column-major buffer exactly as multibody_crba returns it."""
        q = _dvec(q, self.n)
        return _take(_lib.multibody_crba(self._h, q.ctypes.data_as(_dp)), self.n * self.n)

    def crba(self, q) -> np.ndarray:
        return self.crba_raw(q).reshape(self.n, self.n).T.copy()

    def fwd_kin(self, q) -> np.ndarray:
        q = _dvec(q, self.n)
        return _take(_lib.multibody_fwd_kin(self._h, q.ctypes.data_as(_dp)), 3)

    def jac_raw(self, q) -> np.ndarray:
        q = _dvec(q, self.n)
        return _take(_lib.multibody_jac(self._h, q.ctypes.data_as(_dp)), 6 * self.n)

    def jac(self, q) -> np.ndarray:
        return self.jac_raw(q).reshape(self.n, 6).T.copy()

    # ------------------------------------------------------- batched, device [n, B]
    def rnea_batch(self, q, qd, qdd, out=None, stream=None):
        q = _soa(q, self.n, "q")
        B = q.shape[1]
        qd = _soa(qd, self.n, "qd", q.dtype, B)
        qdd = _soa(qdd, self.n, "qdd", q.dtype, B)
        if out is None:
            out = torch.empty_strided(q.shape, q.stride(), dtype=q.dtype, device=q.device)
        _soa(out, self.n, "tau", q.dtype, B)
        ld = _same_ld((q, qd, qdd, out))
        dev = _one_device((q, qd, qdd, out))
        fn = getattr(_lib, f"multibody_rnea_batch_{_TORCH_SUFFIX[q.dtype]}")
        with torch.cuda.device(dev):
            _check(fn(self._h, q.data_ptr(), qd.data_ptr(), qdd.data_ptr(), out.data_ptr(), B, ld,
                      _stream_ptr(stream, dev)), "rnea_batch")
        return out

    def fd_batch(self, q, qd, tau, out=None, stream=None):
        q = _soa(q, self.n, "q")
        B = q.shape[1]
        qd = _soa(qd, self.n, "qd", q.dtype, B)
        tau = _soa(tau, self.n, "tau", q.dtype, B)
        if out is None:
            out = torch.empty_strided(q.shape, q.stride(), dtype=q.dtype, device=q.device)
        _soa(out, self.n, "qdd", q.dtype, B)
        ld = _same_ld((q, qd, tau, out))
        dev = _one_device((q, qd, tau, out))
        fn = getattr(_lib, f"multibody_fd_batch_{_TORCH_SUFFIX[q.dtype]}")
        with torch.cuda.device(dev):
            _check(fn(self._h, q.data_ptr(), qd.data_ptr(), tau.data_ptr(), out.data_ptr(), B, ld,
                      _stream_ptr(stream, dev)), "fd_batch")
        return out

    def rnea_fd_batch(self, q, qd, qdd, tau_in, tau=None, qdd_out=None, stream=None):
        """multibody_rnea_fd_batch_*: (tau = rnea(q, qd, qdd), qdd_out = fd(q, qd, tau_in)) in one
        launch for mass-matrix models (two kernels otherwise); [n, B] CUDA tensors."""
        q = _soa(q, self.n, "q")
        B = q.shape[1]
        ins = [q] + [_soa(x, self.n, k, q.dtype, B) for x, k in ((qd, "qd"), (qdd, "qdd"), (tau_in, "tau_in"))]
        outs = []
        for o, k in ((tau, "tau"), (qdd_out, "qdd_out")):
            o = torch.empty_strided(q.shape, q.stride(), dtype=q.dtype, device=q.device) if o is None else o
            outs.append(_soa(o, self.n, k, q.dtype, B))
        ld = _same_ld(ins + outs)
        dev = _one_device(ins + outs)
        fn = getattr(_lib, f"multibody_rnea_fd_batch_{_TORCH_SUFFIX[q.dtype]}")
        with torch.cuda.device(dev):
            _check(fn(self._h, *[t.data_ptr() for t in ins + outs], B, ld, _stream_ptr(stream, dev)), "rnea_fd_batch")
        return outs[0], outs[1]

    def rnea_fd_batch_tiled(self, q, qd, qdd, tau_in, B, tau=None, qdd_out=None, stream=None):
        """The same on tiled [ceil(B/256), n, 256] tensors (multibody_rnea_fd_batch_tiled_*)."""
        q = self._tiled(q, "q", B)
        ins = [q] + [self._tiled(x, k, B, q.dtype) for x, k in ((qd, "qd"), (qdd, "qdd"), (tau_in, "tau_in"))]
        outs = [torch.empty_like(q) if o is None else self._tiled(o, k, B, q.dtype)
                for o, k in ((tau, "tau"), (qdd_out, "qdd_out"))]
        dev = _one_device(ins + outs)
        fn = getattr(_lib, f"multibody_rnea_fd_batch_tiled_{_TORCH_SUFFIX[q.dtype]}")
        with torch.cuda.device(dev):
            _check(fn(self._h, *[t.data_ptr() for t in ins + outs], B, _stream_ptr(stream, dev)),
                   "rnea_fd_batch_tiled")
        return outs[0], outs[1]

    # ---- tiled layout [ceil(B/256), n, 256] (rigidbody_batch.h) ----------------------
    def _tiled(self, t, name, B, dtype=None):
        T = (B + TILE - 1) // TILE
        if not isinstance(t, torch.Tensor) or not t.is_cuda:
            raise TypeError(f"{name} must be a CUDA (HIP) torch tensor of shape [tiles, n, 256]")
        if tuple(t.shape) != (T, self.n, TILE) or not t.is_contiguous():
            raise ValueError(f"{name} must be a contiguous [{T}, {self.n}, {TILE}] tensor for batch {B}")
        if dtype is not None and t.dtype != dtype:
            raise TypeError(f"{name} has dtype {t.dtype}, expected {dtype}")
        return t

    def _tiled_call(self, kind, a, b, c, B, out, stream):
        a = self._tiled(a, "arg0", B)
        b, c = self._tiled(b, "arg1", B, a.dtype), self._tiled(c, "arg2", B, a.dtype)
        out = torch.empty_like(a) if out is None else self._tiled(out, "out", B, a.dtype)
        dev = _one_device((a, b, c, out))
        fn = getattr(_lib, f"multibody_{kind}_batch_tiled_{_TORCH_SUFFIX[a.dtype]}")
        with torch.cuda.device(dev):
            _check(fn(self._h, a.data_ptr(), b.data_ptr(), c.data_ptr(), out.data_ptr(), B,
                      _stream_ptr(stream, dev)), f"{kind}_batch_tiled")
        return out

    def rnea_batch_tiled(self, q, qd, qdd, B, out=None, stream=None):
        """RNEA on tiled [ceil(B/256), n, 256] tensors (see to_tiled)."""
        return self._tiled_call("rnea", q, qd, qdd, B, out, stream)

    def fd_batch_tiled(self, q, qd, tau, B, out=None, stream=None):
        return self._tiled_call("fd", q, qd, tau, B, out, stream)

    def _q_tiled(self, kind, rows, q, B, out, stream):
        q = self._tiled(q, "q", B)
        if q.dtype not in (torch.float32, torch.float64):
            raise TypeError(f"q has dtype {q.dtype}, expected float32 or float64")
        shape = ((B + TILE - 1) // TILE, rows, TILE)
        if out is None:
            out = torch.empty(shape, dtype=q.dtype, device=q.device)
        elif tuple(out.shape) != shape or out.dtype != q.dtype or not out.is_contiguous():
            raise ValueError(f"out must be a contiguous {list(shape)} tensor of q's dtype")
        dev = _one_device((q, out))
        fn = getattr(_lib, f"multibody_{kind}_batch_tiled_{_TORCH_SUFFIX[q.dtype]}")
        with torch.cuda.device(dev):
            _check(fn(self._h, q.data_ptr(), out.data_ptr(), B, _stream_ptr(stream, dev)), f"{kind}_batch_tiled")
        return out

    def crba_batch_tiled(self, q, B, out=None, stream=None):
        """Mass matrices on the tiled layout: q [ceil(B/256), n, 256] -> [ceil(B/256), n*n, 256]."""
        return self._q_tiled("crba", self.n * self.n, q, B, out, stream)

    def fwd_kin_batch_tiled(self, q, B, out=None, stream=None):
        return self._q_tiled("fwd_kin", 3, q, B, out, stream)

    def jac_batch_tiled(self, q, B, out=None, stream=None):
        return self._q_tiled("jac", 6 * self.n, q, B, out, stream)

    def rollout_batch(self, q, qd, tau_seq, dt, traj=False, stream=None):
        """K fused forward-dynamics + semi-implicit Euler steps, in place on q and qd
        ([n, B] CUDA tensors); tau_seq [K, n, B].  Returns the trajectory [K, n, B] of q
        when traj=True (else None)."""
        q = _soa(q, self.n, "q")
        B = q.shape[1]
        qd = _soa(qd, self.n, "qd", q.dtype, B)
        if not isinstance(tau_seq, torch.Tensor) or tau_seq.dim() != 3 or tau_seq.shape[1:] != (self.n, B):
            raise ValueError(f"tau_seq must be [K, {self.n}, {B}]")
        if tau_seq.dtype != q.dtype or not tau_seq.is_contiguous():
            raise ValueError("tau_seq must be contiguous with the state's dtype")
        ld = _same_ld((q, qd))
        if B > 1 and ld != B:
            raise ValueError("rollout needs contiguous [n, B] state (ld == B), like tau_seq")
        K = tau_seq.shape[0]
        tr = torch.empty_like(tau_seq) if traj else None
        dev = _one_device((q, qd, tau_seq))
        fn = getattr(_lib, f"multibody_rollout_batch_{_TORCH_SUFFIX[q.dtype]}")
        with torch.cuda.device(dev):
            _check(fn(self._h, q.data_ptr(), qd.data_ptr(), tau_seq.data_ptr(), float(dt), int(K),
                      tr.data_ptr() if tr is not None else None, B, max(ld, B, 1), _stream_ptr(stream, dev)),
                   "rollout_batch")
        return tr

    def crba_batch(self, q, out=None, stream=None):
        q = _soa(q, self.n, "q")
        B = q.shape[1]
        if out is None:
            out = torch.empty((self.n * self.n, _ld(q)), dtype=q.dtype, device=q.device)[:, :B]
        fn = getattr(_lib, f"multibody_crba_batch_{_TORCH_SUFFIX[q.dtype]}")
        if out.shape != (self.n * self.n, B) or (B > 1 and out.stride(0) != _ld(q)):
            raise ValueError("out must be [n*n, B] with the inputs' leading dimension")
        dev = _one_device((q, out))
        with torch.cuda.device(dev):
            _check(fn(self._h, q.data_ptr(), out.data_ptr(), B, _ld(q), _stream_ptr(stream, dev)), "crba_batch")
        return out

    def fwd_kin_batch(self, q, out=None, stream=None):
        q = _soa(q, self.n, "q")
        if q.dtype not in (torch.float32, torch.float64):
            raise TypeError(f"q has dtype {q.dtype}, expected float32 or float64")
        B = q.shape[1]
        if out is None:
            out = torch.empty((3, _ld(q)), dtype=q.dtype, device=q.device)[:, :B]
        _kin_out(out, 3, q)
        dev = _one_device((q, out))
        with torch.cuda.device(dev):
            fn = _lib.multibody_fwd_kin_batch_f64 if q.dtype == torch.float64 else _lib.multibody_fwd_kin_batch_f32
            _check(fn(self._h, q.data_ptr(), out.data_ptr(), B, _ld(q), _stream_ptr(stream, dev)), "fwd_kin_batch")
        return out

    def jac_batch(self, q, out=None, stream=None):
        q = _soa(q, self.n, "q")
        if q.dtype not in (torch.float32, torch.float64):
            raise TypeError(f"q has dtype {q.dtype}, expected float32 or float64")
        B = q.shape[1]
        if out is None:
            out = torch.empty((6 * self.n, _ld(q)), dtype=q.dtype, device=q.device)[:, :B]
        _kin_out(out, 6 * self.n, q)
        dev = _one_device((q, out))
        with torch.cuda.device(dev):
            fn = _lib.multibody_jac_batch_f64 if q.dtype == torch.float64 else _lib.multibody_jac_batch_f32
            _check(fn(self._h, q.data_ptr(), out.data_ptr(), B, _ld(q), _stream_ptr(stream, dev)), "jac_batch")
        return out

    # -------------------------------------------------------- batched, host [n, B]
    def rnea_batch_host(self, q, qd, qdd, dtype=np.float64):
        """Blocking host form: multibody_rnea_batch_host_f64 (default: fp64, the reference's Real,
        whatever the inputs' dtype) or _f32 with dtype=np.float32."""
        return self._host_call("rnea", (q, qd, qdd), dtype)

    def fd_batch_host(self, q, qd, tau, dtype=np.float64):
        """Blocking host form: multibody_fd_batch_host_f64 (default) or _f32 (dtype=np.float32)."""
        return self._host_call("fd", (q, qd, tau), dtype)

    def rnea_fd_batch_host(self, q, qd, qdd, tau_in, dtype=np.float64):
        """Blocking host form of rnea_fd_batch: (tau, qdd_out) as [n, B] numpy arrays
        (multibody_rnea_fd_batch_host_f64, or _f32 with dtype=np.float32)."""
        arrs = _host_soa((q, qd, qdd, tau_in), self.n, dtype)
        B = arrs[0].shape[1]
        outs = [np.empty_like(arrs[0]) for _ in range(2)]
        f32 = arrs[0].dtype == np.float32
        fn = getattr(_lib, f"multibody_rnea_fd_batch_host_{'f32' if f32 else 'f64'}")
        ptr = _fp if f32 else _dp
        _check(fn(self._h, *[a.ctypes.data_as(ptr) for a in arrs + outs], B), "rnea_fd_batch_host")
        return outs[0], outs[1]

    def _host_call(self, kind, ins, dtype):
        arrs = _host_soa(ins, self.n, dtype)
        B = arrs[0].shape[1]
        out = np.empty_like(arrs[0])
        f32 = arrs[0].dtype == np.float32
        fn = getattr(_lib, f"multibody_{kind}_batch_host_{'f32' if f32 else 'f64'}")
        ptr = _fp if f32 else _dp
        _check(fn(self._h, *[a.ctypes.data_as(ptr) for a in arrs], out.ctypes.data_as(ptr), B),
               f"{kind}_batch_host")
        return out


def to_tiled(x, stream=None):
    """[rows, B] SoA CUDA tensor -> new [ceil(B/256), rows, 256] tiled tensor (rb_to_tiled_*)."""
    if not isinstance(x, torch.Tensor) or not x.is_cuda or x.dim() != 2 or (x.shape[1] > 1 and x.stride(1) != 1):
        raise TypeError("to_tiled needs a CUDA tensor [rows, B] contiguous along B")
    rows, B = x.shape
    out = torch.empty(((B + TILE - 1) // TILE, rows, TILE), dtype=x.dtype, device=x.device)
    fn = getattr(_lib, f"rb_to_tiled_{_TORCH_SUFFIX[x.dtype]}")
    with torch.cuda.device(x.device):
        _check(fn(x.data_ptr(), _ld(x), out.data_ptr(), rows, B, _stream_ptr(stream, x.device)), "to_tiled")
    return out


def from_tiled(t, B, stream=None):
    """[ceil(B/256), rows, 256] tiled tensor -> new [rows, B] SoA tensor (rb_from_tiled_*)."""
    if not isinstance(t, torch.Tensor) or not t.is_cuda or t.dim() != 3 or t.shape[2] != TILE or \
            t.shape[0] != (B + TILE - 1) // TILE or not t.is_contiguous():
        raise TypeError(f"from_tiled needs a contiguous CUDA tensor [ceil(B/256), rows, 256] for B={B}")
    rows = t.shape[1]
    out = torch.empty((rows, B), dtype=t.dtype, device=t.device)
    fn = getattr(_lib, f"rb_from_tiled_{_TORCH_SUFFIX[t.dtype]}")
    with torch.cuda.device(t.device):
        _check(fn(t.data_ptr(), out.data_ptr(), max(B, 1), rows, B, _stream_ptr(stream, t.device)), "from_tiled")
    return out


def fill_uniform(t, lo, hi, seed, stream=None):
    """rb_fill_uniform_*: t[j, b] = lo[j] + (hi[j]-lo[j]) * u(seed, j, b) on the device."""
    if not isinstance(t, torch.Tensor) or not t.is_cuda or t.dim() != 2 or (t.shape[1] > 1 and t.stride(1) != 1):
        raise TypeError("fill_uniform needs a CUDA tensor [rows, B] contiguous along B")
    rows, B = t.shape
    lo = np.ascontiguousarray(lo, dtype=np.float64)
    hi = np.ascontiguousarray(hi, dtype=np.float64)
    if lo.shape != (rows,) or hi.shape != (rows,):
        raise ValueError("lo/hi must have one value per row")
    fn = getattr(_lib, f"rb_fill_uniform_{_TORCH_SUFFIX[t.dtype]}")
    with torch.cuda.device(t.device):
        _check(fn(t.data_ptr(), rows, B, _ld(t), lo.ctypes.data_as(_dp), hi.ctypes.data_as(_dp),
                  ctypes.c_uint64(seed), _stream_ptr(stream, t.device)), "fill_uniform")
    return t
