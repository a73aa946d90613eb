"""A/B parity of a forward-dynamics kernel form (jit_variant V, RB_EXPERIMENTAL) against the
default form and the fp64 kernel, SoA and tiled, at 2^20 and ragged sizes.  usage: streamchk.py [V]"""
import os, sys
os.environ["RB_EXPERIMENTAL"]="1"
sys.path[:0]=[os.getcwd(), os.path.join(os.getcwd(),"rigidbody-rs_amd")]
import torch
from rigidbody_amd import ffi
mb=ffi.Multibody.new(); mb.upload()
V=int(sys.argv[1]) if len(sys.argv)>1 else 128
ok=True
for B in (1<<20, 65536, 1000, 777, 70001, 513, 256):
    g=torch.Generator(device="cuda").manual_seed(B)
    q=torch.rand((7,B),device="cuda",generator=g)*6-3; qd=torch.rand((7,B),device="cuda",generator=g)*4-2; tau=torch.rand((7,B),device="cuda",generator=g)*20-10
    ref=mb.fd_batch(q.double(),qd.double(),tau.double())
    tq,tqd,tt=(ffi.to_tiled(x) for x in (q,qd,tau))
    outs=[];touts=[]
    for v in (0,V):
        ffi.set_tuning("jit_variant",v)
        outs.append(mb.fd_batch(q,qd,tau).clone())
        touts.append(ffi.from_tiled(mb.fd_batch_tiled(tq,tqd,tt,B),B).clone())
    torch.cuda.synchronize()
    for nm,o in (("soa",outs),("tiled",touts)):
        same=torch.equal(o[0],o[1])
        e=[((x.double()-ref).norm(dim=0)/(1+ref.norm(dim=0))).max().item() for x in o]
        nd=(o[0]!=o[1]).sum().item()
        ok&=same or (e[1]<=2*e[0]+1e-6)
        print(B, nm, "bit-identical" if same else f"{nd} differ, max abs {(o[0]-o[1]).abs().max().item():.3g}", f"err vs f64: base {e[0]:.3g} variant {e[1]:.3g}", flush=True)
print("ALL OK" if ok else "MISMATCH")
