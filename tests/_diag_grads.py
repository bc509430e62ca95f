import sys, os, torch
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(),'tests'))
import cad_pkg; cad = cad_pkg.load()
from oracle import cad_oracle as O
from conftest import max_rel_err
torch.set_num_threads(16)
dev = torch.device('cuda',0)
for (f,B,H,W) in [(64,1,64,64),(64,2,64,64),(32,1,64,64),(16,1,64,64),(64,1,128,128)]:
    params=O.init_params(f,seed=f); bufs=O.init_buffers(f)
    rgb,gt,K=[torch.from_numpy(a) for a in O.synth_batch(B,H,W)]
    r=O.Trainer(params,bufs).step(rgb,gt,K)
    r64=O.Trainer(params,bufs,dtype=torch.float64).step(rgb,gt,K)
    st=dict(params); st.update(bufs)
    m=cad.BaselineUNet(3,f,10.0,batch=B,height=H,width=W); m.load_state_dict(st)
    L=cad.CombinedDepthLoss(batch=B,height=H,width=W)
    rg,gg,kg=rgb.to(dev),gt.to(dev),K.to(dev)
    pred=m.forward(rg); l5,dp=L.forward_with_intrinsics(pred,gg,rg,kg); m.backward(dp); torch.cuda.synchronize()
    print(f,B,H,W,'pred',max_rel_err(pred.cpu(),r64['pred']),'dpred',max_rel_err(dp.cpu(),r64['dpred']),'dpred32',max_rel_err(r['dpred'],r64['dpred']))
    gr=m.grads(); bad=[]
    for (n,_),g32,g64 in zip(O.param_spec(f),r['grads'],r64['grads']):
        a,b=max_rel_err(gr[n],g64),max_rel_err(g32,g64)
        if a>max(1e-3,3*b): bad.append((n,round(a,6),round(b,8)))
    print('  bad', bad[:12], len(bad))
