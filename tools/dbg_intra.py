import sys, numpy as np
sys.path.insert(0,'.'); sys.path.insert(0,'oracle')
import torch, p64_amd, oracle
for (w,h) in ((176,144),):
    nmb=(w//16)*(h//16)
    f0=p64_amd.synth_frame(1,0,w,h)
    li=torch.zeros(nmb,dtype=torch.uint8,device='cuda')
    r0=torch.zeros(f0.size,dtype=torch.uint8,device='cuda')
    o=p64_amd.encode_frames(torch.from_numpy(f0).cuda(),None,r0,li,width=w,height=h,intra=True,quant=8)
    torch.cuda.synchronize()
    lio=np.zeros(nmb,np.uint8)
    coef,mb,me,rec=oracle.encode_frame(w,h,f0,None,lio,intra=True,quant=8)
    g=r0.cpu().numpy()
    print(w,h,'coef eq',np.array_equal(o.coef.cpu().numpy()[0],coef))
    Y=g[:w*h].reshape(h,w); Yo=rec[:w*h].reshape(h,w)
    d=np.argwhere(Y!=Yo)
    print('luma mismatches',len(d), d[:10], (Y.astype(int)-Yo)[tuple(d[:5].T)] if len(d) else '')
    U=g[w*h:w*h+w*h//4]; Uo=rec[w*h:w*h+w*h//4]
    print('chroma U mismatches', (U!=Uo).sum())
    mbs=set((y//16)*(w//16)+x//16 for y,x in d)
    print('bad MBs', sorted(mbs)[:20], len(mbs))
    print('MB0 gpu rows 0-3 cols 0-23:\n', Y[:4,:24]); print('oracle:\n', Yo[:4,:24])
    print('coded cur:\n', f0[:w*h].reshape(h,w)[:4,:24])
