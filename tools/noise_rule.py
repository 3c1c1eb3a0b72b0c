"""Simulation behind the noise rule of k_search.hip me_full (development aid):
for synthetic and uniform-noise CIF pictures, SAD(0,0), the lower-bound sum
S(0,0) and the survivor count of the exact search; prints how often the rule
16 S0 - 512 < K SAD(0,0) (with SAD(0,0) > 24*256) sends a block to the dense
pass and whether the bound would have pruned it (<= 256 survivors)."""
import sys, numpy as np
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
import p64_amd
W,H=352,288
def lerp(a,b): return (a+b)>>1
def nested44(P):
    v1=lerp(P[:-1],P[1:]); v2=lerp(v1[:-2],v1[2:]); h1=lerp(v2[:,:-1],v2[:,1:]); return lerp(h1[:,:-2],h1[:,2:])
rng=np.random.default_rng(0)
def analyse(ref,cur,label):
    Rn,Cn=nested44(ref),nested44(cur)
    rows=[]
    for mb in range(0,396,5):
        x0,y0=16*(mb%22),16*(mb//22)
        C=cur[y0:y0+16,x0:x0+16]; cn=Cn[y0:y0+16:4,x0:x0+16:4]
        if cn.max()-cn.min()<12: continue
        sad0=np.abs(ref[y0:y0+16,x0:x0+16]-C).sum()
        S0=np.abs(Rn[y0:y0+16:4,x0:x0+16:4]-cn).sum()
        ehf=np.abs(C-np.repeat(np.repeat(cn,4,0),4,1)).sum()
        best=1<<40; lbs=[];sads=[]
        for dx in range(-15,15):
            for dy in range(-15,15):
                px,py=x0+dx,y0+dy
                if not(0<=px<W-16 and 0<=py<H-16): continue
                sads.append(np.abs(ref[py:py+16,px:px+16]-C).sum())
                lbs.append(16*np.abs(Rn[py:py+16:4,px:px+16:4]-cn).sum()-512)
        lbs=np.array(lbs);sads=np.array(sads)
        cs=np.argmin(lbs);T=min(sads[cs],sad0)
        surv=int((lbs<=T).sum())
        rows.append((sad0,S0,surv,ehf))
    r=np.array(rows)
    for K in (0.3,0.4,0.5):
        pred=(r[:,3] > K*r[:,0]) & (r[:,0]>256*24)
        print(label,K,'n',len(r),'pred_dense',pred.mean().round(3),'actual>256',(r[:,2]>256).mean().round(3),
              'false_dense(surv<=256)',(pred&(r[:,2]<=256)).mean().round(3),'missed',(~pred&(r[:,2]>256)).mean().round(3))
if len(sys.argv) == 1:
  for seed in (1,2,3,4,5,6,9,12):
      t=3
      ref=p64_amd.synth_frame(seed,t-1,W,H)[:W*H].reshape(H,W).astype(np.int64)
      cur=p64_amd.synth_frame(seed,t,W,H)[:W*H].reshape(H,W).astype(np.int64)
      analyse(ref,cur,f'synth{seed}')
  ref=rng.integers(0,256,(H,W)); cur=rng.integers(0,256,(H,W))
  analyse(ref,cur,'noise')

if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "pan15":
    for seed in (1, 2, 3):
        base = p64_amd.synth_frame(seed, 0, W, H)[:W * H].reshape(H, W).astype(np.int64)
        r = (np.roll(base, (15, 15), (0, 1)) + rng.integers(-3, 4, (H, W))).clip(0, 255)
        c = (np.roll(base, (30, 30), (0, 1)) + rng.integers(-3, 4, (H, W))).clip(0, 255)
        analyse(r, c, f"pan15-{seed}")
