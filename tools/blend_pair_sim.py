"""Cost model of the pair-walk blend (k_blend_pw) from the oracle's per-group break points
(og_render group_iters: the full-list entry at which each 4x2 group of a tile breaks): per half-tile unit
the live groups after every 16-entry checkpoint, the current kernel's cost (4 px / lane, then 2 px / lane
once <= 16 of 32 groups live) against pairs of consecutive longest-first units (8 / 4 / 2 px per lane at
> 32 / > 16 / <= 16 live groups), with the longest `singles` units alone.  Wave-instructions per entry
from the ISA: 78 / 42.6 / 38.  usage: python tools/blend_pair_sim.py [config] [orbit angle]"""
import sys, os, numpy as np, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0]=[ROOT, os.path.join(ROOT,'oracle'), os.path.join(ROOT,'gsm-renderer_amd')]
import oracle as O
from gsm_amd import scenes
cfg=sys.argv[1] if len(sys.argv)>1 else "cfg2_1m_sh3_1080p_f16"
ang=float(sys.argv[2]) if len(sys.argv)>2 else 0.0
c=scenes.CONFIGS[cfg]; n,W,H,sh,prec=c["count"],c["width"],c["height"],c["sh"],c["precision"]
wn,hn,cam=scenes.gen_scene(n,W,H,sh,prec,seed=42)
if ang: cam=scenes.orbit_camera(W,H,ang)
t=time.time(); r=O.render(wn,hn,sh,cam,W,H,max_gaussians=n,nthreads=8); print("oracle",time.time()-t,flush=True)
gi=r["group_iters"].astype(np.int64)  # [T,8,8] ly,lx
hd=r["headers"]
T=gi.shape[0]
units=[]
for h in (0,1):
    b=gi[:,:,4*h:4*h+4].reshape(T,32)
    units.append(b)
B=np.concatenate(units,0)  # [2T,32] break index per group
cnt=np.concatenate([hd[:,1],hd[:,1]])
walk=B.max(1)
walk16=np.minimum(((walk+15)//16)*16, ((cnt+15)//16)*16)
C8,C4,C2=78.0,42.6,38.0
def alive(Bu,e):  # groups alive after entry e-1 (i.e. at checkpoint e)
    return (Bu>e).sum(-1)
# current
cur=np.zeros(len(B))
maxw=int(walk16.max())
comp=np.zeros(len(B),bool)
for cp in range(16,maxw+16,16):
    act=walk16>=cp
    cur+=np.where(act, 16*np.where(comp,C2,C4),0)
    comp|= act & (alive(B,cp)<=16)
order=np.argsort(-walk16,kind='stable')
def pairs(singles):
    rest=order[singles:]
    u=rest[0::2]; v=rest[1::2]
    if len(v)<len(u): v=np.append(v,-1)
    Bu=B[u]; Bv=np.where(v[:,None]>=0,B[np.maximum(v,0)],0)
    wu=walk16[u]; wv=np.where(v>=0,walk16[np.maximum(v,0)],0)
    w=np.maximum(wu,wv)
    cost=np.zeros(len(u)); lay=np.full(len(u),8)
    for cp in range(16,int(w.max())+16,16):
        act=w>=cp
        cc=np.select([lay==8,lay==4],[C8,C4],C2)
        cost+=np.where(act,16*cc,0)
        a=np.where(wu>=cp,alive(Bu,cp),0)+np.where(wv>=cp,alive(Bv,cp),0)
        lay=np.where((lay==8)&(a<=32),4,lay)
        lay=np.where((lay==4)&(a<=16),2,lay)
    return cur[order[:singles]].sum()+cost.sum(), cost
tot=cur.sum()
print(cfg,ang,"units",len(B),"walk entries",int(walk16.sum()),"current Minst",round(tot/1e6,2))
for s in (0,1024,3072):
    tp,cost=pairs(s)
    print(" singles",s,"pairs Minst",round(tp/1e6,2),"ratio",round(tp/tot,3),"longest pair job k",round(cost.max()/1e3,1),"longest single k",round(cur.max()/1e3,1))
