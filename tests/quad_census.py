"""Skip-unit census at cfg 3 ("8x8 pixel quads instead of 16x4 row strips"): over the instances
before each tile's last contributor, the (instance, unit) pairs holding a pixel whose fp32 alpha passes 1/255, and those
holding one still compositing, for the composites' 16x4 row strips and for 8x8 quads.  Test infrastructure (it runs the
oracle): python tests/quad_census.py
"""
import sys, os, numpy as np, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__)))); sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from helpers import scene_inputs, run_oracle
inp=scene_inputs(1_000_000,1920,1080,sh_degree=3,seed=0)
o=run_oracle(inp); run=o[-1]
W,H=1920,1080; gx=(W+15)//16; gy=(H+15)//16; T=gx*gy
pl=run.point_list(); rg=run.ranges(); geo=run.geom(); _,nc=run.image_state()
xy=geo['xy'].astype(np.float32); co=geo['conic_opacity'].astype(np.float32)
ncp=np.zeros((gy*16,gx*16),np.uint32); ncp[:H,:W]=nc
tl=ncp.reshape(gy,16,gx,16).max(axis=(1,3)).reshape(-1)
tiles=[];gids=[];idxs=[]
for t in range(T):
    a,b=rg[t]; n=int(tl[t])
    if n==0: continue
    gids.append(pl[a:a+n]); tiles.append(np.full(n,t,np.int64)); idxs.append(np.arange(n))
g=np.concatenate(gids); t=np.concatenate(tiles); idx=np.concatenate(idxs)
print('instances', len(g))
ys,xs=np.mgrid[0:16,0:16]
strip=(ys//4)            # 16x4 row strips
quad=(ys//8)*2+(xs//8)   # 8x8 quads
cs=cq=cs_live=cq_live=0
B=200000
t0=time.time()
for s in range(0,len(g),B):
    gg=g[s:s+B]; tt=t[s:s+B]; ii=idx[s:s+B]
    px=(tt%gx)[:,None,None]*16+xs[None]; py=(tt//gx)[:,None,None]*16+ys[None]
    dx=xy[gg,0][:,None,None]-px.astype(np.float32); dy=xy[gg,1][:,None,None]-py.astype(np.float32)
    A=co[gg,0][:,None,None];Bc=co[gg,1][:,None,None];C=co[gg,2][:,None,None];O=co[gg,3][:,None,None]
    power=np.float32(-0.5)*(A*dx*dx+C*dy*dy)-Bc*dx*dy
    alpha=np.minimum(np.float32(0.99),O*np.exp(power))
    ok=(power<=0)&(alpha>=np.float32(1/255))&(px<W)&(py<H)
    live=ok & (ii[:,None,None] < ncp[np.minimum(py,gy*16-1),np.minimum(px,gx*16-1)])
    for m,acc in ((ok,'a'),(live,'l')):
        sc=np.stack([m[:,strip==k].any(1) for k in range(4)],1).sum()
        qc=np.stack([m[:,quad==k].any(1) for k in range(4)],1).sum()
        if acc=='a': cs+=sc; cq+=qc
        else: cs_live+=sc; cq_live+=qc
print('alpha-passing: strips',cs,'quads',cq,' still compositing: strips',cs_live,'quads',cq_live, time.time()-t0)
