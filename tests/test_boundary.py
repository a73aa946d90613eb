"""The C-ABI boundary on CPU: library loads, exports every declared symbol, and its
host-side model loading (URDF -> per-link constants, run once, no GPU) matches the
oracle's restatement of Multibody::from_urdf (multibody.rs:65-77, joint.rs:53-68).
No compute entry point is called here -- those need a GPU (test_gpu_parity.py)."""
import ctypes
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from conftest import PKG, REPO, load_json

HEADERS = [os.path.join(REPO, "include", "rigidbody.h"), os.path.join(REPO, "include", "rigidbody_batch.h")]


def declared_functions():
    names = []
    for h in HEADERS:
        txt = open(h).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        names += re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w]*\s*\**\s*\**\s*(\w+)\s*\(", txt, flags=re.M)
    return sorted(set(n for n in names if n.startswith(("multibody_", "rb_"))))


@pytest.fixture(scope="module")
def ffi():
    from rigidbody_amd import ffi

    return ffi


def test_headers_declare_reference_abi():
    names = declared_functions()
    for sym in ["multibody_new", "multibody_fwd_kin", "multibody_jac", "multibody_rnea", "multibody_crba",
                "multibody_free"]:
        assert sym in names
    assert len(names) >= 30


def test_library_exports_every_declared_symbol(ffi):
    lib = ffi.lib()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_reference_header_compiles_as_c_and_cpp(tmp_path):
    """rigidbody.h stays a plain C header (the reference's is C++-only) and links."""
    import subprocess

    src = tmp_path / "use.c"
    src.write_text('#include "rigidbody_batch.h"\nint main(void){ Multibody *m = 0; multibody_free(m); return 0; }\n')
    lib = os.path.join(REPO, "rigidbody-rs_amd")
    for cc, f in (("gcc", str(src)), ("g++", str(src))):
        args = [cc, "-x", "c" if cc == "gcc" else "c++", f, "-I", os.path.join(REPO, "include"), "-L", lib,
                "-lrigidbody_bindings", "-o", str(tmp_path / "a.out")]
        r = subprocess.run(args, capture_output=True, text=True)
        assert r.returncode == 0, r.stderr


def test_embedded_fr3_model(ffi):
    mb = ffi.Multibody.new()
    assert mb.n == 7
    assert abs(mb.total_mass - 16.062132) < 1e-12
    lower, upper, vel, eff = mb.limits()
    np.testing.assert_array_equal(eff, [87, 87, 87, 87, 12, 12, 12])
    np.testing.assert_array_equal(lower, [-2.3093, -1.5133, -2.4937, -2.7478, -2.48, 0.8521, -2.6895])
    np.testing.assert_array_equal(vel, [2.0, 1.0, 1.5, 1.25, 3.0, 1.5, 3.0])
    mb.close()


def _blob_links(blob):
    n = int(blob[2])
    return n, blob[5:].reshape(n, 38)  # header: magic, version 3, n, pairing, flags


def test_model_build_matches_oracle(ffi, fr3_text, oracle_mod):
    """Product preprocessing (C++) vs oracle preprocessing (C), field by field."""
    from oracle import urdf_model
    from rigidbody_amd import chains

    for xml in (fr3_text, chains.synthetic_chain_urdf(30), chains.synthetic_chain_urdf(5)):
        raw = urdf_model.model_raw_from_urdf(xml)
        om = oracle_mod.Model(raw)
        ob = np.frombuffer(ctypes.string_at(om._buf, ctypes.sizeof(om._buf)), dtype=np.float64)
        nmax = 64  # ORACLE_MAX_DOF; oracle_model = {int n (8 B with padding), arrays...}
        n = raw["n"]
        off = 1
        o_axis = ob[off:off + nmax * 3].reshape(nmax, 3)[:n]; off += nmax * 3
        o_pq = ob[off:off + nmax * 4].reshape(nmax, 4)[:n]; off += nmax * 4
        o_pt = ob[off:off + nmax * 3].reshape(nmax, 3)[:n]; off += nmax * 3
        o_m = ob[off:off + nmax][:n]; off += nmax
        o_com = ob[off:off + nmax * 3].reshape(nmax, 3)[:n]; off += nmax * 3
        o_ic = ob[off:off + nmax * 9].reshape(nmax, 9)[:n]; off += nmax * 9
        o_io = ob[off:off + nmax * 9].reshape(nmax, 9)[:n]
        mb = ffi.Multibody.from_urdf_string(xml)
        pn, L = _blob_links(mb.blob())
        assert pn == n
        np.testing.assert_array_equal(L[:, 0:3], o_axis)
        np.testing.assert_allclose(L[:, 3:7], o_pq, rtol=0, atol=2e-16)
        np.testing.assert_array_equal(L[:, 7:10], o_pt)
        np.testing.assert_array_equal(L[:, 10], o_m)
        np.testing.assert_array_equal(L[:, 11:14], o_com)
        np.testing.assert_array_equal(L[:, 14:23], o_ic)
        np.testing.assert_allclose(L[:, 23:32], o_io, rtol=1e-15, atol=1e-18)
        mb.close()


def test_blob_round_trip(ffi, fr3_text):
    a = ffi.Multibody.from_urdf_string(fr3_text)
    b = ffi.Multibody.from_blob(a.blob())
    np.testing.assert_array_equal(a.blob(), b.blob())
    with pytest.raises(ffi.RigidBodyError):
        ffi.Multibody.from_blob(a.blob()[:-1])


def test_urdf_file_and_env(ffi, tmp_path, monkeypatch, fr3_text):
    from rigidbody_amd import chains

    p = tmp_path / "c3.urdf"
    p.write_text(chains.synthetic_chain_urdf(3))
    mb = ffi.Multibody.from_urdf(str(p))
    assert mb.n == 3
    monkeypatch.setenv("RIGIDBODY_URDF", str(p))
    assert ffi.Multibody.new().n == 3
    ref = "/root/reference/assets/fr3.urdf"
    if os.path.exists(ref):
        full = ffi.Multibody.from_urdf(ref)
        np.testing.assert_array_equal(full.blob(), ffi.Multibody.from_urdf_string(fr3_text).blob())


@pytest.mark.parametrize("xml,needle", [
    ("<robot><link name='a'/>", "XML parse error"),
    ("<notrobot/>", "not <robot>"),
    ("<robot><link name='a'/><joint name='j' type='fixed'><parent link='a'/><child link='a'/></joint></robot>",
     "no non-fixed joint"),
])
def test_bad_urdf_raises(ffi, xml, needle):
    with pytest.raises(ffi.RigidBodyError, match=needle):
        ffi.Multibody.from_urdf_string(xml)


def test_unsupported_axis_and_dof(ffi):
    from rigidbody_amd import chains

    xml = chains.synthetic_chain_urdf(3).replace('<axis xyz="0 0 1"/>', '<axis xyz="1 0 0"/>', 1)
    with pytest.raises(ffi.RigidBodyError, match="non-z joint axis"):
        ffi.Multibody.from_urdf_string(xml)
    dofs = ffi.supported_dofs()
    assert 7 in dofs and 30 in dofs
    bad = next(k for k in range(1, 64) if k not in dofs)
    with pytest.raises(ffi.RigidBodyError, match="no kernel compiled"):
        ffi.Multibody.from_urdf_string(chains.synthetic_chain_urdf(bad))


def test_null_handle_paths_do_not_abort(ffi):
    """The reference unwraps NULL and aborts (lib.rs:22,37,50,64); here NULL comes back."""
    lib = ffi.lib()
    q = (ctypes.c_double * 7)()
    assert not lib.multibody_rnea(None, q, q, q)
    assert not lib.multibody_crba(None, q)
    assert not lib.multibody_fwd_kin(None, q)
    assert not lib.multibody_jac(None, q)
    lib.multibody_free(None)
    assert lib.multibody_rnea_batch_f32(None, None, None, None, None, 0, 0, None) == 1
    assert "NULL" in ffi.last_error()
    # the tiled q-only entry points: NULL handle, then NULL arrays with a live handle, refused
    # before any device work (no GPU here)
    mb = ffi.Multibody.new()
    for k in ("crba", "fwd_kin", "jac"):
        for t in ("f32", "f64"):
            fn = getattr(lib, f"multibody_{k}_batch_tiled_{t}")
            assert fn(None, None, None, 1, None) == 1, (k, t)
            assert fn(mb.handle, None, None, 1, None) == 1, (k, t)
            assert "NULL" in ffi.last_error()
            assert fn(mb.handle, None, None, 0, None) == 0, (k, t)  # empty batch: nothing to do


def test_index_pairing_detected(ffi):
    """A URDF whose index pairing differs from child pairing still loads (the reference
    pairs by index, multibody.rs:70) -- the product follows the reference."""
    from oracle import urdf_model

    xml = """<robot name="swap">
      <link name="l1"><inertial><origin xyz="0 0 0.1"/><mass value="1"/><inertia ixx="1" ixy="0" ixz="0" iyy="1" iyz="0" izz="1"/></inertial></link>
      <link name="l2"><inertial><origin xyz="0 0 0.2"/><mass value="2"/><inertia ixx="2" ixy="0" ixz="0" iyy="2" iyz="0" izz="2"/></inertial></link>
      <joint name="j2" type="revolute"><parent link="l1"/><child link="l2"/><axis xyz="0 0 1"/></joint>
      <joint name="j1" type="revolute"><parent link="world"/><child link="l1"/><axis xyz="0 0 1"/></joint>
    </robot>"""
    raw = urdf_model.model_raw_from_urdf(xml)
    assert not urdf_model.index_pairing_matches_child(raw)
    mb = ffi.Multibody.from_urdf_string(xml)
    n, L = _blob_links(mb.blob())
    assert mb.blob()[3] == 0.0  # pairing flag recorded
    np.testing.assert_array_equal(L[:, 10], raw["mass"])


def test_version(ffi):
    assert "gfx950" in ffi.version()


def test_golden_fixture_is_self_consistent():
    g = load_json("main_cpp_case.json")
    assert abs(g["total_mass"] - 16.062132) < 1e-12


def test_jit_source_and_compile(ffi, fr3_text):
    """The model-specialised RNEA kernel (hipRTC) builds for gfx950 without a device, and
    its source carries the model with the near-0/+-1 rotation entries snapped."""
    from rigidbody_amd import chains

    mb = ffi.Multibody.from_urdf_string(fr3_text)
    src = mb.jit_source(f64=False)
    assert "constexpr int N = 7" in src and "rnea_lane" in src
    assert "0.333000004f" in src  # fr3_joint1 origin z (fr3.urdf:62) as an fp32 literal
    assert "2.22044605e-16" not in src  # rotation residues snapped to exact 0
    for kind in ("rnea", "fd", "crba", "rollout"):
        for f64 in (False, True):
            assert mb.jit_compile(f64=f64, kind=kind) > 1000
    # FR3 forward dynamics: the mass-matrix form by default, the ABA under fd_form 1
    assert "fdh_lane" in mb.jit_source(kind="fd") and "crba_lane" in mb.jit_source(kind="crba")
    try:
        ffi.set_tuning("fd_form", 1)
        assert "aba_lane" in mb.jit_source(kind="fd")
        assert mb.jit_compile(f64=True, kind="fd") > 1000
    finally:
        ffi.set_tuning("fd_form", -1)
    c30 = ffi.Multibody.from_urdf_string(chains.synthetic_chain_urdf(30))
    assert "rnea_lane" in c30.jit_source(f64=False)  # JIT kernels use the one-per-lane form
    assert "aba_lane" in c30.jit_source(kind="fd")  # long chains keep the ABA
    assert c30.jit_compile(f64=False) > 1000


def test_set_tuning_rejects_unknown_key(ffi):
    with pytest.raises(ffi.RigidBodyError, match="unknown tuning key"):
        ffi.set_tuning("no_such_knob", 1)


def test_set_tuning_experimental_keys_gated(ffi):
    """Only the production knobs (jit, pack, rnea_stream) are writable without
    RB_EXPERIMENTAL=1; the A/B selectors are refused with a message naming the switch, and
    the kernel forms measured and rejected in round 1 no longer exist at all."""
    import os

    if os.environ.get("RB_EXPERIMENTAL") == "1":
        pytest.skip("experimental knobs enabled in this process")
    for key in ("split_rot", "f64_tab", "jit_variant", "rnea_nt", "jit_waves", "opaque_consts"):
        with pytest.raises(ffi.RigidBodyError, match="RB_EXPERIMENTAL"):
            ffi.set_tuning(key, 0)
    for key in ("rnea_seg", "rnea_tiles", "rnea_tile", "fd_stream"):
        with pytest.raises(ffi.RigidBodyError, match="unknown tuning key"):
            ffi.set_tuning(key, 1)
    for key, dflt in (("jit", 1), ("pack", -1), ("rnea_stream", -1)):
        ffi.set_tuning(key, dflt)


def test_jit_kernel_forms_compile(ffi, fr3_text):
    """Every model-specialised kernel form the production knobs select builds for gfx950
    (hipRTC, no device) and its source carries the form: paired fp32 forward-dynamics lanes
    (pack; default for chains up to 8 links), one per lane, or the small-batch split of packed
    waves (pack 4, fp32 mass-matrix form only), table-assisted fp64 sincos,
    split joint rotation for signed-permutation frames."""
    from rigidbody_amd import chains

    mb = ffi.Multibody.from_urdf_string(fr3_text)
    c30 = ffi.Multibody.from_urdf_string(chains.synthetic_chain_urdf(30))
    assert "fdh_lane" in mb.jit_source(False, "fd")             # FR3: mass-matrix FD
    assert "fdh_lane" in mb.jit_source(True, "fd")
    assert "fdh_lane" not in c30.jit_source(False, "fd")        # ... the ABA for 30 links
    c12 = ffi.Multibody.from_urdf_string(chains.synthetic_chain_urdf(12))
    for f64 in (False, True):                                   # 12 links: mass-matrix FD, one per lane
        assert "fdh_lane<" in c12.jit_source(f64, "fd") and "fdh_lane<" in c12.jit_source(f64, "fd", batch=65536)
        assert "RB_ROLLOUT_FDH" not in c12.jit_source(f64, "rollout")  # ... its rollouts the ABA
    assert "rnea_lane<" in mb.jit_source(False, "rnea")         # fp32 RNEA one per lane
    assert "rnea_lane_seq2<" in mb.jit_source(True, "rnea")     # fp64 RNEA: sequential pair
    assert "rnea_lane_rev<" in c30.jit_source(True, "rnea")     # ... up to 8 links; longer: reversed sweep
    try:
        ffi.set_tuning("rnea_rev", 0)
        assert "rnea_lane<" in c30.jit_source(True, "rnea")     # stored-force form on request
    finally:
        ffi.set_tuning("rnea_rev", -1)
    assert "rollout_lane2" in mb.jit_source(False, "rollout")   # paired fp32 rollout
    assert "rollout_lane2" not in mb.jit_source(True, "rollout")
    assert "rollout_lane2" not in c30.jit_source(False, "rollout")
    assert mb.jit_compile(f64=False, kind="rollout") > 1000
    assert "sctab_init" in mb.jit_source(True, "rnea") and "sctab_init" not in mb.jit_source(False, "rnea")
    # the source of the kernel a given launch takes (multibody_jit_source_ex): the auto policy's
    # form, tail and load / store policy per batch size and layout (capi.cpp jit_shape)
    head = mb.jit_source(True, "rnea", batch=1 << 20, tiled=True)
    assert "rnea_lane_seq2<" in head and "rnea_lane<" in head and "S_ =" in head  # pairs + one-per-lane tail
    assert "rnea_lane_seq2<" in mb.jit_source(False, "rnea", batch=1 << 20, tiled=True)
    assert "#define RB_NT 0" in mb.jit_source(False, "rnea", batch=1 << 20, tiled=True)
    assert "#define RB_NT 3" in mb.jit_source(False, "rnea", batch=1 << 20, tiled=False)
    assert "rnea_lane_seq2<" not in mb.jit_source(True, "rnea", batch=1 << 17)
    assert "fdh_split_block1<" in mb.jit_source(False, "fd", batch=1 << 15)
    assert "fdh_split_block1<" in mb.jit_source(False, "fd", batch=65536)
    assert "fdh_split_block1<" in mb.jit_source(False, "fd", batch=1 << 17)
    assert "fdh_lane2<" in mb.jit_source(False, "fd", batch=(1 << 17) + 1)
    assert "rollout_split_block2<" in mb.jit_source(False, "rollout", batch=65536)
    assert mb.jit_compile(f64=True, kind="rnea", batch=1 << 20, tiled=True) > 1000
    # rnea_park (a production knob) is clamped to what 3 blocks per CU leave of the 160 KB LDS
    # (8 links x 6 KB per block) instead of reaching hipRTC, which would fail and drop the launch
    # to the generic kernel
    assert "rnea_lane_park<T, N, true, 8>" in c30.jit_source(False, "rnea")
    try:
        ffi.set_tuning("rnea_park", 40)
        assert "rnea_lane_park<T, N, true, 8>" in c30.jit_source(False, "rnea")
        assert c30.jit_compile(f64=False, kind="rnea") > 1000
        ffi.set_tuning("rnea_park", 5)
        assert "rnea_lane_park<T, N, true, 5>" in c30.jit_source(False, "rnea")
    finally:
        ffi.set_tuning("rnea_park", -1)
    assert "RB_SPLIT_ROT 1" in mb.jit_source(False, "fd")  # FR3 frames are signed permutations
    try:
        for form, pack, marker in ((1, 2, "aba_lane2"), (1, 1, "aba_lane<"), (1, 3, "aba_lane_seq2<"),
                                   (2, 2, "fdh_lane2<"), (2, 1, "fdh_lane<"), (2, 4, "fdh_split_block2<"), (2, 5, "fdh_split_block1<"),
                                   (1, 4, "aba_lane<")):
            ffi.set_tuning("fd_form", form)
            ffi.set_tuning("pack", pack)
            assert marker in mb.jit_source(False, "fd"), (form, pack)
            assert mb.jit_compile(f64=False, kind="fd") > 1000, (form, pack)
        ffi.set_tuning("fd_form", 2)
        ffi.set_tuning("pack", 4)
        assert "fdh_lane<" in mb.jit_source(True, "fd")  # pack 4 has no fp64 form
        ffi.set_tuning("pack", 1)
        assert "rnea_lane<" in mb.jit_source(True, "rnea")
    finally:
        ffi.set_tuning("pack", -1)
        ffi.set_tuning("fd_form", -1)
    for kind in ("rnea", "fd", "crba", "rollout"):
        assert mb.jit_compile(f64=True, kind=kind) > 1000, kind


def test_occupancy_cliff_rebuild(ffi, tmp_path, monkeypatch):
    """jit_compile (jit.hpp "Occupancy cliff"): a kernel built without an occupancy target that
    lands just past 256 registers (one wave per SIMD) is rebuilt with a 2-wave target.  The
    9-joint tree's fp64 RNEA (258 registers) is the case; the FR3 kernels are untouched."""
    import glob
    import subprocess

    from rigidbody_amd import chains

    def vgprs(co):
        notes = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", co], capture_output=True,
                               text=True).stdout
        return int(re.search(r"\.vgpr_count:\s+(\d+)", notes).group(1))

    # The tree kernel lands at 258 registers without kernel-argument preload (with it, the default,
    # at 234 and needs no rebuild): the rebuild is exercised with preload off, in a process of its
    # own (an experimental knob, RB_EXPERIMENTAL=1 at start-up)
    cliff = tmp_path / "cliff"
    cliff.mkdir()
    code = ("import sys; sys.path[:0] = [%r, %r]\n"
            "from rigidbody_amd import chains, ffi\n"
            "tree = ffi.Multibody.from_urdf_string(chains.tree_urdf(), ffi.URDF_TREE | ffi.GENERAL_AXES)\n"
            "assert tree.jit_compile(True, kind='rnea') > 1000\n"
            # multibody_jit_source_ex reports the source of the code object a launch loads: the
            # rebuilt one (it used to return the first-pass source, without the target)
            "assert 'amdgpu_waves_per_eu(2)' in tree.jit_source(True, 'rnea')\n") % (REPO, PKG)
    env = dict(os.environ, RB_JIT_DUMP=str(cliff), RB_EXPERIMENTAL="1", RB_KERNARG_PRELOAD="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    co = sorted(glob.glob(str(cliff / "*.co")), key=os.path.getmtime)[-1]
    assert vgprs(co) <= 256
    assert "amdgpu_waves_per_eu(2)" in open(co[:-3] + ".hip").read()
    monkeypatch.setenv("RB_JIT_DUMP", str(tmp_path))
    tree = ffi.Multibody.from_urdf_string(chains.tree_urdf(), ffi.URDF_TREE | ffi.GENERAL_AXES)
    assert tree.jit_compile(True, kind="rnea") > 1000
    co = sorted(glob.glob(str(tmp_path / "*.co")), key=os.path.getmtime)[-1]
    assert vgprs(co) <= 256  # two waves per SIMD either way
    fr3 = ffi.Multibody.new()
    for f64 in (True, False):
        fr3.jit_compile(f64, kind="rnea")
        co = sorted(glob.glob(str(tmp_path / "*.co")), key=os.path.getmtime)[-1]
        assert vgprs(co) <= 128, f64


def test_host_batch_shapes_checked(ffi):
    """The host batch wrappers check every array is [n, B] before the library copies n*B
    doubles from (and into) them: a short q would overflow the output, a short qd/tau be
    over-read."""
    mb = ffi.Multibody.new()
    n, B = mb.n, 5
    ok = np.zeros((n, B))
    for bad in (np.zeros((n - 1, B)), np.zeros((n, B - 1)), np.zeros(n * B), np.zeros((n, B, 1))):
        for args in ((bad, ok, ok), (ok, bad, ok), (ok, ok, bad)):
            with pytest.raises(ValueError, match=r"\[7, B\]"):
                mb.rnea_batch_host(*args)
            with pytest.raises(ValueError, match=r"\[7, B\]"):
                mb.fd_batch_host(*args)


def test_one_device_per_call(ffi):
    """Arrays of one batched call must share a device (the library launches on the current
    device, which the wrappers set from the arrays); a mix is refused before any launch."""
    import torch

    from rigidbody_amd import ffi as mod

    assert mod._one_device((torch.empty(1), torch.empty(2))) == torch.device("cpu")
    with pytest.raises(ValueError, match="one device"):
        mod._one_device((torch.empty(1), torch.empty(1, device="meta")))


@pytest.mark.parametrize("xml,needle", [
    ("", "XML parse error"),
    ("<robot", "XML parse error"),
    ("<robot name='r'><!-- never closed", "XML parse error"),
    ("<robot name=r></robot>", "XML parse error"),
    ("<robot name='r'></robott>", "mismatched closing tag"),
    ("<robot name='r\x00'><link/></robot>", "no non-fixed joint"),
    ("<" * 5000 + "robot>", "XML parse error"),
    ("<a>" * 100000, "nested too deeply"),
    ("<robot><link name='a'><inertial><mass value='nan'/></inertial></link></robot>", "non-finite"),
    ("<robot><link name='a'><inertial><mass value='1e999'/></inertial></link></robot>", "non-finite"),
    ("<robot><link name='a'><inertial><mass value='abc'/></inertial></link></robot>", "bad number"),
    ("<robot><link name='a'><inertial><origin xyz='1 2'/></inertial></link></robot>", "bad number list"),
    ("<robot><link name='a'><inertial><origin xyz='1 2 3 4'/></inertial></link></robot>", "too many numbers"),
    ("<robot><link name='a'/><joint name='j' type='revolute'><origin rpy='0 0 inf'/>"
     "<parent link='a'/><child link='a'/></joint></robot>", "non-finite"),
])
def test_malformed_urdf_rejected(ffi, xml, needle):
    """Malformed / adversarial URDF text is refused with a message (never a crash): truncation,
    unterminated comments, unquoted attributes, mismatched tags, NUL bytes, deep nesting
    (the parser recurses per level: capped at 256), non-finite or missing numbers.  The
    sanitized build (`make -C rigidbody-rs_amd sanitize`) runs these under ASan/UBSan."""
    with pytest.raises(ffi.RigidBodyError, match=needle):
        ffi.Multibody.from_urdf_string(xml)


def test_mutated_fr3_never_crashes(ffi, fr3_text):
    """600 deterministic mutants of the FR3 URDF (truncations, byte flips, deleted or inserted
    markup characters, duplicated spans): each either loads a model or raises with a message."""
    rng = np.random.default_rng(20250224)
    text = fr3_text.encode()
    loaded = refused = 0
    for k in range(600):
        b = bytearray(text)
        op = k % 5
        at = int(rng.integers(0, len(b)))
        if op == 0:
            b = b[:at]
        elif op == 1:
            b[at] = int(rng.integers(1, 256))
        elif op == 2:
            del b[at:at + int(rng.integers(1, 40))]
        elif op == 3:
            b[at:at] = bytes([ord(c) for c in rng.choice(list("<>/='\" &;"), 3)])
        else:
            n = int(rng.integers(1, 400))
            b[at:at] = b[at:at + n]
        xml = b.decode("latin-1")
        try:
            mb = ffi.Multibody.from_urdf_string(xml)
            assert mb.n >= 1
            loaded += 1
        except ffi.RigidBodyError as e:
            assert str(e)
            refused += 1
    assert loaded + refused == 600 and refused > 100
