"""rigidbody_amd -- host-side mirror of khaninger/rigidbody-rs's hot path on MI355X.

The compute lives in librigidbody_bindings.so (HIP, gfx950) behind the reference's
C ABI (include/rigidbody.h) and its batched extension (include/rigidbody_batch.h).
`rigidbody_amd.ffi` binds it; `rigidbody_amd.chains` builds synthetic chains and the
benchmark input distributions.  `ffi` is loaded lazily so `chains` can be used
without torch or a built library.
"""
from __future__ import annotations

_LAZY = {"Multibody", "RigidBodyError", "fill_uniform", "supported_dofs", "last_error", "version", "ffi"}


def __getattr__(name):
    if name in _LAZY:
        import importlib

        ffi = importlib.import_module(".ffi", __name__)
        return ffi if name == "ffi" else getattr(ffi, name)
    raise AttributeError(name)
