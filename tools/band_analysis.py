"""Band values of biComputeTmap's partial fields (FastMarching.py:141-162) against the reference's own
(tests/golden/fmm2d_bidir.npz): the full-field value, the update from popped neighbours alone, and
the band relaxation (fixed point over popped + band cells, every other cell +inf) -- ratio reference /
candidate and the share of band cells matched exactly.  CPU only (oracle/); DESIGN §3.7."""
import sys; sys.path.insert(0,'oracle'); sys.path.insert(0,'.')
import numpy as np, math
import oracle as O
d=np.load('tests/golden/fmm2d_bidir.npz')
def ranks(T):
    n=T.size; f=T.reshape(-1); fin=np.isfinite(f)
    order=np.lexsort((np.arange(n), f)); order=order[fin[order]]
    r=np.full(n, np.iinfo(np.int64).max, np.int64); r[order]=np.arange(order.size); return r.reshape(T.shape)
def godunov(a,b,c):
    if math.isinf(a) and math.isinf(b): return math.inf
    if math.isinf(a): return b+c
    if math.isinf(b): return a+c
    if c < abs(a-b): return min(a,b)+c
    return 0.5*(a+b+math.sqrt(2*c*c-(a-b)**2))
for i in range(6):
    p=f"b{i}_"; cost=d[p+'cost'].astype(float); g=d[p+'goal']; s=d[p+'start']
    FG=O.fmm2d(cost, g); FS=O.fmm2d(cost, s)
    rg, rs = ranks(FG), ranks(FS)
    m=np.maximum(rg, rs); k=m.min()
    for F, r, R, name in ((FG, rg, d[p+'TG'], 'G'), (FS, rs, d[p+'TS'], 'S')):
        closed = r <= k
        H,W=F.shape
        nb=np.zeros_like(closed); nb[1:]|=closed[:-1]; nb[:-1]|=closed[1:]; nb[:,1:]|=closed[:,:-1]; nb[:,:-1]|=closed[:,1:]
        band = nb & ~closed & np.isfinite(R) & np.isfinite(F)
        ys,xs=np.nonzero(band)
        errA=[]; errB=[]
        for y,x in zip(ys,xs):
            ref=R[y,x]
            def cv(yy,xx):
                if 0<=yy<H and 0<=xx<W and closed[yy,xx]: return F[yy,xx]
                return math.inf
            a=min(cv(y,x-1),cv(y,x+1)); b=min(cv(y-1,x),cv(y+1,x))
            B=godunov(a,b,cost[y,x])
            errA.append(ref/F[y,x]); errB.append(ref/B)
        errA=np.array(errA); errB=np.array(errB)
        print(i,name,"band",band.sum(),"full-field: ratio max %.4f exact %.2f"%(errA.max(), np.mean(np.abs(errA-1)<1e-12)),
              "| closed-only: ratio min %.4f max %.4f exact %.2f"%(errB.min(), errB.max(), np.mean(np.abs(errB-1)<1e-12)))
print("---- Jacobi over closed + band (far = inf)")
for i in range(6):
    p=f"b{i}_"; cost=d[p+'cost'].astype(float); g=d[p+'goal']; s=d[p+'start']
    FG=O.fmm2d(cost, g); FS=O.fmm2d(cost, s)
    rg, rs = ranks(FG), ranks(FS)
    m=np.maximum(rg, rs); k=m.min()
    for F, r, R, name in ((FG, rg, d[p+'TG'], 'G'), (FS, rs, d[p+'TS'], 'S')):
        closed = r <= k
        H,W=F.shape
        nb=np.zeros_like(closed); nb[1:]|=closed[:-1]; nb[:-1]|=closed[1:]; nb[:,1:]|=closed[:,:-1]; nb[:,:-1]|=closed[:,1:]
        bandm = nb & ~closed & np.isfinite(F)
        T = np.where(closed, F, np.inf)
        for it in range(200):
            Tn = T.copy()
            for y,x in zip(*np.nonzero(bandm)):
                def v(yy,xx):
                    return T[yy,xx] if (0<=yy<H and 0<=xx<W and (closed[yy,xx] or bandm[yy,xx])) else math.inf
                a=min(v(y,x-1),v(y,x+1)); b=min(v(y-1,x),v(y+1,x))
                Tn[y,x]=min(godunov(a,b,cost[y,x]), T[y,x])
            if np.array_equal(Tn,T): break
            T=Tn
        sel = bandm & np.isfinite(R)
        ratio = R[sel]/T[sel]
        print(i,name,"iters",it,"ratio min %.4f max %.4f exact %.2f"%(ratio.min(), ratio.max(), np.mean(np.abs(ratio-1)<1e-12)))
