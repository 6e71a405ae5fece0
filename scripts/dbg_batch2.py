import sys, numpy as np
sys.path.insert(0, '.')
import sparc_ldpc_amd as sp
from oracle import amp_oracle as orc
def rel(a,b): return np.linalg.norm(a-b)/np.linalg.norm(b)
for (L,M,B) in [(64,64,5),(48,512,7),(20,8,9)]:
    for prec in ("fp32",):
        P,R,T=2.0,1.0,20
        n=int(L*np.log2(M)/R)
        op=sp.SparcOperator(L,M,n,sp.make_ordering(L,M,n),precision=prec)
        Pl=P/L*np.ones(L)
        Ab,Az,_=orc.sparc_transforms(L,M,n)
        ys=np.stack([orc.rep_inputs(L,M,n,Pl,0.6,Ab,50+i)[1].reshape(-1) for i in range(B)])
        bb,it=op.amp_batch(ys,Pl,T,early_stop=False)
        for i in range(B):
            b1,i1=op.amp_batch(ys[i:i+1],Pl,T,early_stop=False)
            print(L,M,B,i,"%.2e"%rel(bb[i],b1[0]), bb[i][:3])
