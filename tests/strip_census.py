"""Strip census at cfg 3 (DESIGN.md §2 "Exact strip masks"): over the instances before each tile's last contributor,
the (instance, 4-row strip) pairs that cell_mask admits (numpy restatement of gsr_common.h strip_mask_exact), that
hold an alpha-passing pixel, and that hold one still compositing (oracle_strip_census), plus the per-strip contributor
bound (bwd_lastc).  Test infrastructure (it runs the oracle): python tests/strip_census.py
"""
import sys, numpy as np, time
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__)))); sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from helpers import scene_inputs, run_oracle
inp=scene_inputs(1_000_000,1920,1080,sh_degree=3,seed=0)
o=run_oracle(inp); run=o[-1]
W,H=1920,1080; gx=(W+15)//16; gy=(H+15)//16; T=gx*gy
pl=run.point_list(); rg=run.ranges(); geo=run.geom(); _,nc=run.image_state()
xy=geo['xy'].astype(np.float32); co=geo['conic_opacity'].astype(np.float32)
ncp=np.zeros((gy*16,gx*16),np.uint32); ncp[:H,:W]=nc
tl=ncp.reshape(gy,16,gx,16).max(axis=(1,3)).reshape(-1)
# instances before each tile's last contributor
tiles=[];gids=[]
for t in range(T):
    a,b=rg[t]; n=int(tl[t])
    if n==0: continue
    gids.append(pl[a:a+n]); tiles.append(np.full(n,t,np.int64))
g=np.concatenate(gids); t=np.concatenate(tiles)
tx=(t%gx).astype(np.float32); ty=(t//gx).astype(np.float32)
row0=ty*16; col0=tx*16
A=co[g,0];B=co[g,1];C=co[g,2];O=co[g,3]; x=xy[g,0]; y=xy[g,1]
# strip_mask_exact (gsr_common.h) in float32
o255=255*O
det=A*C-B*B; hd=0.5*(A-C); lmin=0.5*(A+C)-np.sqrt(hd*hd+B*B)
eps=1e-5*(abs(A)+abs(B)+abs(C))/lmin
tau=(2*np.log(np.maximum(o255*1.00001,1))+1e-3)/(1-eps)
V=np.sqrt(tau*A/det)
uL=col0-x; uR=uL+15
ut=-B*V/A
ic=1/C; ctau=C*tau
vmax=V.copy(); vmin=-V.copy()
m1=~((ut>=uL)&(ut<=uR)); u=np.clip(ut,uL,uR)
vmax=np.where(m1,(-B*u+np.sqrt(np.maximum(ctau-det*u*u,0)))*ic,vmax)
m2=~((-ut>=uL)&(-ut<=uR)); u2=np.clip(-ut,uL,uR)
vmin=np.where(m2,(-B*u2-np.sqrt(np.maximum(ctau-det*u2*u2,0)))*ic,vmin)
mg=1e-2*V+1e-3*(abs(uL)+abs(uR))+0.0625
lo=y+vmin-mg-row0; hi=y+vmax+mg-row0
cnt=0
for k in range(4):
    m=(hi>=4*k)&(lo<=4*k+3)
    keepall=~((o255>=0.999))
    m=np.where(keepall, o255>=0.999, m)  # alpha < 1/255 everywhere -> 0
    bad=~(det>0)|~(lmin>0)|~(eps<1e-2)|~(V<1e6)
    m=m|bad
    cnt+=int(m.sum())
print('cell_mask strips before tile last:', cnt, 'instances', len(g), run.strip_census())
# strip-level last-contributor bound: idx < max n_contrib over the strip's pixels
idx=np.concatenate([np.arange(int(tl[tt])) for tt in range(T) if tl[tt]>0])
smax=ncp.reshape(gy,4,4,gx,16).max(axis=(2,4))  # (gy, 4 strips, gx)
cnt2=0
for k in range(4):
    m=(hi>=4*k)&(lo<=4*k+3)
    m=np.where(~(o255>=0.999), o255>=0.999, m)
    bad=~(det>0)|~(lmin>0)|~(eps<1e-2)|~(V<1e6)
    m=m|bad
    sm=smax[(t//gx).astype(int),k,(t%gx).astype(int)]
    cnt2+=int((m&(idx<sm)).sum())
print('cell_mask & strip lastc bound:', cnt2)
