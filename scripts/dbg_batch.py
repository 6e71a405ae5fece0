import sys, numpy as np
sys.path.insert(0, '.')
import sparc_ldpc_amd as sp
from oracle import amp_oracle as orc
L,M,P,T=20,8,2.0,20
n=int(L*np.log2(M))
Pl=P/L*np.ones(L)
Ab,Az,_=orc.sparc_transforms(L,M,n)
ys=np.stack([orc.rep_inputs(L,M,n,Pl,0.6,Ab,50+i)[1].reshape(-1) for i in range(9)])
def rel(a,b): return np.linalg.norm(a-b)/np.linalg.norm(b)
for prec in ("fp64","fp32"):
    op=sp.SparcOperator(L,M,n,sp.make_ordering(L,M,n),precision=prec)
    for t in (1,2,5,10,20):
        bb,_=op.amp_batch(ys,Pl,t,early_stop=False)
        r=[rel(bb[i], op.amp_batch(ys[i:i+1],Pl,t,early_stop=False)[0][0]) for i in range(9)]
        print(prec, t, " ".join("%.1e"%v for v in r))
print("--- test order replica")
prec="fp32"
op=sp.SparcOperator(L,M,n,sp.make_ordering(L,M,n),precision=prec)
bb,it=op.amp_batch(ys,Pl,T,early_stop=False)
for i in range(9):
    b1,i1=op.amp_batch(ys[i:i+1],Pl,T,early_stop=False)
    print(i, "%.2e"%rel(bb[i],b1[0]), it[i], i1[0])
bb2,_=op.amp_batch(ys,Pl,T,early_stop=False)
print("rerun batch", [ "%.1e"%rel(bb2[i],bb[i]) for i in range(9)])
