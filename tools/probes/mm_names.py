import torch
dev=torch.device('cuda',0)
for M,N,K in [(8192,8192,8192),(48384,10240,1280),(193536,5120,640)]:
    x=torch.randn(M,K,device=dev,dtype=torch.bfloat16); w=torch.randn(N,K,device=dev,dtype=torch.bfloat16)
    for _ in range(3): y=torch.matmul(x,w.t())
    torch.cuda.synchronize()
