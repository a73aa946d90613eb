"""The hipRTC code objects carry kernel-argument preload (tuning.hpp kernarg_preload): the kernel
descriptor of rb_jit_kernel asks the dispatch to place the first 14 argument dwords in SGPRs, so
the kernel does not start with dependent scalar loads of its arguments (13 for the fused pair,
whose next argument, a 64-bit stride, would not fit whole).  hipRTC compiles on the
CPU here; RB_JIT_DUMP (jit.cpp) writes each code object, and this test reads the descriptor
(AMDHSA kernel descriptor: 64 bytes, kernarg_preload at byte 58, length in bits 0-6)."""
import os
import struct
import subprocess
import sys

import pytest

from conftest import PKG, REPO


def _kd_preload(path):
    b = open(path, "rb").read()
    shoff = struct.unpack_from("<Q", b, 0x28)[0]
    shentsize, shnum = struct.unpack_from("<HH", b, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", b, shoff + i * shentsize) for i in range(shnum)]
    symtab = next(s for s in secs if s[1] == 2)  # SHT_SYMTAB
    strtab = secs[symtab[6]]
    for k in range(symtab[5] // 24):
        name_off, _, _, shndx, value, _ = struct.unpack_from("<IBBHQQ", b, symtab[4] + 24 * k)
        end = b.index(b"\0", strtab[4] + name_off)
        if b[strtab[4] + name_off:end] == b"rb_jit_kernel.kd":
            sec = secs[shndx]
            kd = b[sec[4] + value - sec[3]:sec[4] + value - sec[3] + 64]
            return struct.unpack_from("<H", kd, 58)[0] & 0x7F
    raise AssertionError("no rb_jit_kernel.kd in " + path)


@pytest.mark.parametrize("env,want", [({}, (13, 14)), ({"RB_EXPERIMENTAL": "1", "RB_KERNARG_PRELOAD": "0"}, (0,))])
def test_kernarg_preload_in_code_objects(tmp_path, env, want):
    code = ("import sys; sys.path[:0] = [%r, %r]\n"
            "from rigidbody_amd import ffi\n"
            "mb = ffi.Multibody.new()\n"
            "assert mb.jit_compile(f64=True, kind='rnea', batch=1 << 20, tiled=True) > 1000\n"
            "assert mb.jit_compile(f64=False, kind='fd', batch=65536, tiled=True) > 1000\n"
            "assert mb.jit_compile(f64=True, kind='rnea_fd', batch=1 << 17, tiled=True) > 1000\n") % (REPO, PKG)
    e = dict(os.environ, RB_JIT_DUMP=str(tmp_path), **env)
    if not env:
        e.pop("RB_KERNARG_PRELOAD", None)
    r = subprocess.run([sys.executable, "-c", code], env=e, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    cos = sorted(p for p in os.listdir(tmp_path) if p.endswith(".co"))
    assert len(cos) >= 3, cos
    for p in cos:
        assert _kd_preload(str(tmp_path / p)) in want, p
