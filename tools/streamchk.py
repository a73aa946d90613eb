"""A/B parity of a kernel form (jit_variant V, RB_EXPERIMENTAL) against the default form and
the fp64 kernel, SoA and tiled, fp32 and fp64, at 2^20 and ragged sizes.
usage: streamchk.py [V | key=value] [fd|rnea]   (V: jit_variant; key=value: any experimental tuning key)"""
import os, sys
os.environ["RB_EXPERIMENTAL"]="1"
sys.path[:0]=[os.getcwd(), os.path.join(os.getcwd(),"rigidbody-rs_amd")]
import torch
from rigidbody_amd import ffi
mb=ffi.Multibody.new(); mb.upload()
arg=sys.argv[1] if len(sys.argv)>1 else "128"
KEY,V=(arg.split("=")[0], int(arg.split("=")[1])) if "=" in arg else ("jit_variant", int(arg))
K=sys.argv[2] if len(sys.argv)>2 else "fd"
soa_fn=getattr(mb, K+"_batch"); til_fn=getattr(mb, K+"_batch_tiled")
ok=True
for B in (1<<20, (1<<19)+333, (1<<18)+777, 300001, 65536, 1000, 777, 70001, 513, 256):
    g=torch.Generator(device="cuda").manual_seed(B)
    q=torch.rand((7,B),device="cuda",generator=g)*6-3; qd=torch.rand((7,B),device="cuda",generator=g)*4-2; tau=torch.rand((7,B),device="cuda",generator=g)*20-10
    ffi.set_tuning(KEY,0)
    ref=soa_fn(q.double(),qd.double(),tau.double())
    res={}
    for dt in (torch.float32, torch.float64):
        a,b_,c=(x.to(dt) for x in (q,qd,tau))
        tq,tqd,tt=(ffi.to_tiled(x) for x in (a,b_,c))
        outs=[];touts=[]
        for v in (0,V):
            ffi.set_tuning(KEY,v)
            outs.append(soa_fn(a,b_,c).clone())
            touts.append(ffi.from_tiled(til_fn(tq,tqd,tt,B),B).clone())
        res[f"soa_{str(dt)[-7:]}"]=outs; res[f"tiled_{str(dt)[-7:]}"]=touts
    torch.cuda.synchronize()
    for nm,o in res.items():
        same=torch.equal(o[0],o[1])
        e=[((x.double()-ref).norm(dim=0)/(1+ref.norm(dim=0))).max().item() for x in o]
        nd=(o[0]!=o[1]).sum().item()
        ok&=same or (e[1]<=2*e[0]+1e-6)
        print(B, nm, "bit-identical" if same else f"{nd} differ, max abs {(o[0]-o[1]).abs().max().item():.3g}", f"err vs f64: base {e[0]:.3g} variant {e[1]:.3g}", flush=True)
print("ALL OK" if ok else "MISMATCH")
