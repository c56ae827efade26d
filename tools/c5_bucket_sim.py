"""C5 threshold-mode bucket search, simulated on the CPU (numpy; thresholds from the family maps
in double, so approximate): binary-search steps per pixel ("lane mean") and the per-wave maximum
over 64 lanes for each pixel slot of a chunk ("wave-max"), which is what a divergent loop pays.
"cur" = the shipped map (origin one key below T[1], key clamped at T[cmax]); "ends" = the
map of tools/patches/c5_bucket_ends.patch (origin one bucket below T[1], table run to its end).
"""
import numpy as np
rng=np.random.default_rng(1)
N=1<<20
planes=[rng.lognormal(5,1.5,N).astype(np.float32), rng.normal(0,300,N).astype(np.float32), rng.lognormal(5,1.5,N).astype(np.float32)]
def key(x):
    b=x.view(np.uint32).astype(np.uint64)
    return np.where(b>>31, (~b)&0xFFFFFFFF, b|0x80000000).astype(np.uint64)
def qmap(fam,x,ws,we):
    if fam=='log': f=lambda v: np.log(v)
    elif fam=='p05': f=lambda v: v**0.5
    else: f=lambda v: v**2
    return (f(x)-f(ws))/(f(we)-f(ws))*255
NB=2048
for i,(fam,p) in enumerate(zip(['log','p05','p2'],planes)):
    ws,we=float(np.percentile(p,1)),float(np.percentile(p,99))
    if i==1: ws=max(ws,1.0)
    # thresholds: smallest float with q>=c
    cs=np.arange(1,256)
    xs=np.linspace(ws,we,2000001)
    q=np.floor(np.clip(qmap(fam,xs,ws,we),0,255))
    T=np.array([key(np.array([xs[np.searchsorted(q,c)]],np.float32))[0] for c in cs],np.uint64)
    k=key(p)
    for variant in ['cur','ends']:
        k1=int(T[-1])
        if variant=='cur':
            org=int(T[0])-1; span=k1-org; sh=max(0,span.bit_length()-11); hi=k1
        else:
            sh=0
            while ((k1-int(T[0]))>>sh)>NB-2: sh+=1
            org=int(T[0])-(1<<sh); hi=min(org+(NB<<sh)-1,2**32-1)
        idx=(np.clip(k,org,hi)-org)>>sh
        edges=org+(np.arange(NB+1,dtype=np.uint64)<<sh)
        lo=np.searchsorted(T,edges[:-1],side='right'); hi_=np.searchsorted(T,np.minimum(edges[1:]-1,2**32-1),side='right')
        ln=(hi_-lo)[idx.astype(np.int64)]
        it=np.ceil(np.log2(ln+1)).astype(int)  # binary search iterations
        w=it.reshape(-1,4,64)  # chunk of 4 px per lane? layout: lane holds 4 consecutive px
        w=it.reshape(-1,64,4).transpose(0,2,1)  # waves x j x lanes
        print(fam,variant,'lane mean it',it.mean().round(3),'wave-max mean per j',w.max(axis=2).mean().round(3))
