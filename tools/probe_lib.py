"""ctypes loader for the measurement-only bandwidth probe (tools/microbench/probe.hip,
built as tools/microbench/libprobe.so by `make -C tools/microbench`; not part of the product
library).  rb_probe_rows_f32 returns a hipError_t code, 0 on success."""
import ctypes
import os

_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "microbench", "libprobe.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_PATH):
            raise RuntimeError(f"{_PATH} not built: make -C tools/microbench")
        _lib = ctypes.CDLL(_PATH)
        _lib.rb_probe_rows_f32.restype = ctypes.c_int
        _lib.rb_probe_rows_f32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
    return _lib
