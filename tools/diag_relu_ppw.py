import torch, sys
sys.path.insert(0, '/root/repo')
from kubeflow_controller_amd.ops import gemm as G
D = torch.device("cuda")
torch.manual_seed(5)
M, N, K = 4096, 512, 1024
x = (torch.randn(M, K, device=D)).to(torch.bfloat16)
w = (torch.randn(N, K, device=D) * 0.03).to(torch.bfloat16)
b = torch.randn(N, device=D)
y1 = G.gemm_ppp_relu(x, w, b)
y2 = G.gemm_ppw_relu(x, w, b)
y3 = torch.relu(G.gemm_ppp(x, w, probe=9, split=False).float() + b).to(torch.bfloat16)
yr = torch.relu(x.float() @ w.float().t() + b)
print("ppp vs ref", (y1.float()-yr).abs().max().item(), "ppw vs ref", (y2.float()-yr).abs().max().item(), "ppw vs plain+pass", (y2.float()-y3.float()).abs().max().item())
m1, m2, mr = y1 > 0, y2 > 0, yr > 0
print("mask mismatch ppp", (m1 != mr).sum().item(), "ppw", (m2 != mr).sum().item())
bad = (y2.float() - yr).abs() > 0.05
print("bad count", bad.sum().item(), "rows", bad.any(1).nonzero().flatten()[:10].tolist(), "cols", bad.any(0).nonzero().flatten()[:20].tolist())
