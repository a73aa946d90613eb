"""Audit of a model-specialised kernel as hipRTC actually builds it (RB_JIT_DUMP): registers,
LDS, scratch and instruction mix of the code object the library would load.  CPU only.

usage: python tools/jit_rtc_audit.py KIND {f32,f64} [DOF]   (env knobs such as RB_PACK apply)"""
import glob
import os
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rigidbody-rs_amd"))


def main():
    kind, dt = sys.argv[1], sys.argv[2]
    dof = int(sys.argv[3]) if len(sys.argv) > 3 else 7
    d = tempfile.mkdtemp(prefix="rtc_")
    os.environ["RB_JIT_DUMP"] = d
    from rigidbody_amd import chains, ffi

    mb = ffi.Multibody.new() if dof == 7 else ffi.Multibody.from_urdf_string(chains.synthetic_chain_urdf(dof))
    mb.jit_compile(dt == "f64", kind=kind)
    co = sorted(glob.glob(os.path.join(d, "*.co")))[-1]
    notes = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
    for key in (".vgpr_count", ".agpr_count", ".sgpr_count", ".group_segment_fixed_size", ".private_segment_fixed_size"):
        for ln in notes.splitlines():
            if key + ":" in ln:
                print(" ", ln.strip())
    dis = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", co], capture_output=True, text=True).stdout
    ops = [ln.split()[0] for ln in dis.splitlines() if ln.startswith("\t") and ln.split()]
    cls = {}
    for op in ops:
        c = op.split("_")[0] + ("_pk" if op.startswith("v_pk") else "")
        cls[c] = cls.get(c, 0) + 1
    print("  classes:", dict(sorted(cls.items())))
    print("  code object:", co)


if __name__ == "__main__":
    main()
