import torch, time
dev='cuda'
P=100000
def tm(f, n=20):
    for _ in range(3): f()
    torch.cuda.synchronize(); t=time.perf_counter()
    for _ in range(n): f()
    torch.cuda.synchronize(); return (time.perf_counter()-t)/n*1e6
for (i,o) in [(128,128),(32,128),(128,48),(128,3)]:
    x=torch.randn(P,i,device=dev); dy=torch.randn(P,o,device=dev); w=torch.randn(o,i,device=dev)
    fl=2*P*i*o
    r={}
    r['fwd x@w.T']=tm(lambda: torch.nn.functional.linear(x,w))
    r['dX dy@w']=tm(lambda: dy@w)
    r['dW dy.T@x']=tm(lambda: dy.t()@x)
    for S in (25,100,400):
        def f(S=S):
            return torch.bmm(dy.view(S,P//S,o).transpose(1,2), x.view(S,P//S,i)).sum(0)
        r[f'dW splitK{S}']=tm(f)
    print(i,o, {k:f"{v:.0f}us {fl/v/1e6:.1f}TF" for k,v in r.items()}, flush=True)
