#!/usr/bin/env python3
"""Row-block backward visits per (b, m) at the bench encoder call (tools/msda_microbench.make, init
regime): query tiles of consecutive queries vs the position order of msda_win.h (QOrder)."""
import torch, sys
sys.path.insert(0, "tools")
from msda_microbench import make
shapes=[1024,512,256,128]; M=8; P=4; B=1
value, loc, aw, gout = make("init", B, 1920, shapes, M, P, torch.float32, torch.device("cpu"))
Lq=1920; QT=32; ntile=Lq//QT
tot=0; totsamp=0
for l,T in enumerate(shapes):
    x = loc[0,:,:,l,:]*T-0.5   # (Lq,M,P) border: rows floor(x), floor(x)+1 clamped
    x = x.clamp(0,T-1)
    lo = x.floor().long(); hi=(lo+1).clamp(max=T-1)
    vis=0; steps=0; per_tile_blocks=[]
    for m in range(M):
        for t in range(ntile):
            a=lo[t*QT:(t+1)*QT,m].min().item(); b=hi[t*QT:(t+1)*QT,m].max().item()
            nb = b//16 - a//16 + 1
            vis += nb
            # samples per block visit -> steps
            for k in range(a//16, b//16+1):
                r0=k*16
                sel=((lo[t*QT:(t+1)*QT,m]>=r0-1)&(lo[t*QT:(t+1)*QT,m]<=r0+15)).sum().item()
                steps += (sel+31)//32
    print(f"level {l} T={T}: visits/(b,m) {vis/M:.0f} steps {steps/M:.0f}  blocks {T//16}")
    tot+=vis/M; totsamp+=steps/M
print("total visits per (b,m)", tot, "mfma steps", totsamp, "min visits", 60*4)
# position-merged query order
perm=[]
for c in range(128):
    for l,T in enumerate(shapes):
        n=T//128; st=sum(shapes[:l])
        perm += [st + c*n + j for j in range(n)]
perm=torch.tensor(perm)
loc2 = loc[:, perm]
tot=0; totsteps=0
for l,T in enumerate(shapes):
    x = (loc2[0,:,:,l,:]*T-0.5).clamp(0,T-1)
    lo = x.floor().long(); hi=(lo+1).clamp(max=T-1)
    vis=0; steps=0
    for m in range(M):
        for t in range(ntile):
            a=lo[t*QT:(t+1)*QT,m].min().item(); b=hi[t*QT:(t+1)*QT,m].max().item()
            vis += b//16 - a//16 + 1
            for k in range(a//16, b//16+1):
                r0=k*16
                sel=((lo[t*QT:(t+1)*QT,m]>=r0-1)&(lo[t*QT:(t+1)*QT,m]<=r0+15)).sum().item()
                steps += (sel+31)//32
    print(f"sorted level {l}: visits {vis/M:.0f} steps {steps/M:.0f}")
    tot+=vis/M; totsteps+=steps/M
print("sorted total", tot, totsteps)
