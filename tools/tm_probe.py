import torch
for (M,N,K) in [(32000,1024,12544),(28672,256,1024),(8192,8192,8192),(458752,256,256),(13376*64//64,256,256)]:
    A=torch.randn(M,K,device='cuda'); W=torch.randn(N,K,device='cuda')
    for _ in range(3): C=A@W.t()
    torch.cuda.synchronize()
