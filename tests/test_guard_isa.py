"""The input checks survive compilation: the model-specialised kernels compile under
-ffinite-math-only, where the optimizer may treat NaN / Inf results as poison and fold tests on
them.  spatial.hip.hpp InputGuard therefore issues every step of the check as inline assembly
tagged "; rb_guard".  This test compiles the hipRTC source of FR3 kernels for gfx950 with the
options jit.cpp uses (hipcc cross-compiles here, no GPU) and counts the tagged instructions in
the ISA: one v_fma per checked input, one v_mul per joint angle, and per output the add (fp32)
or the NaN test's shift (fp64).  Reference semantics: NaN / Inf flow through
multibody.rs:111-174 (rigidbody_batch.h "Input domain")."""
import os
import re
import subprocess

import pytest

from conftest import PKG

HIPCC = "/opt/rocm/bin/hipcc"
CSRC = os.path.join(PKG, "csrc")

pytestmark = pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")


def _isa(tmp_path, src):
    path = tmp_path / "k.hip"
    path.write_text(src)
    out = tmp_path / "k.s"
    # the options of jit.cpp rtc_compile
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffinite-math-only",
                        "-fno-signed-zeros", "-I", CSRC, "--cuda-device-only", "-S", "-o", str(out), str(path)],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    ops = {}
    for line in out.read_text().splitlines():
        if "rb_guard" in line and not line.lstrip().startswith(";"):
            op = line.split()[0]
            ops[op] = ops.get(op, 0) + 1
    return ops


# (kind, f64, batch, tiled, checked inputs per configuration, angles, outputs, configurations per lane)
CASES = [
    ("rnea", True, 1 << 17, True, 21, 7, 7, 1),    # one per lane
    ("fd", True, 1 << 20, True, 21, 7, 7, 1),      # mass-matrix form: q, qd, tau (qdd = 0 unchecked)
    ("rnea", False, 1 << 17, True, 21, 7, 7, 1),
    ("crba", True, 1 << 20, False, 7, 7, 28, 1),   # upper triangle
    ("rnea_fd", True, 1 << 17, True, 28, 7, 14, 1),
]


@pytest.mark.parametrize("kind,f64,batch,tiled,nin,nang,nout,per", CASES)
def test_guard_instructions_in_isa(tmp_path, kind, f64, batch, tiled, nin, nang, nout, per):
    from rigidbody_amd import ffi

    mb = ffi.Multibody.new()
    src = mb.jit_source(f64, kind, batch=batch, tiled=tiled)
    ops = _isa(tmp_path, src)
    fma = ops.get("v_fma_f32", 0) + ops.get("v_pk_fma_f32", 0)
    mul = ops.get("v_mul_f32", 0) + ops.get("v_pk_mul_f32", 0)
    assert fma >= nin * per, ops
    assert mul >= nang * per, ops
    if f64:
        # one NaN test per distinct running check (the outputs of one configuration share it)
        assert ops.get("v_lshlrev_b32", 0) >= 1, ops
    else:
        assert ops.get("v_add_f32", 0) + ops.get("v_pk_add_f32", 0) >= nout * per, ops


def test_guard_source_has_no_plain_fallback_on_device():
    """The device path of every InputGuard step is the asm form (RB_GUARD_ASM): no compiler-visible
    arithmetic is left for the finite-math optimizer to fold."""
    src = open(os.path.join(CSRC, "spatial.hip.hpp")).read()
    body = src[src.index("struct InputGuard"):src.index("// Paired-lane row access")]
    assert "guard_fma(" in body and "guard_scale(" in body and "guard_add(" in body and "guard_bits2(" in body
    assert not re.search(r"fmadd\(guard_view", body)
