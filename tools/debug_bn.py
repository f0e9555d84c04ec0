import torch
from kubeflow_controller_amd.ops.batchnorm import bn_act
from kubeflow_controller_amd.ops import _lib
torch.manual_seed(0)
d = torch.device("cuda")
def ws_nz():
    ws = _lib._ws.get(("cuda:0", "bn"))
    return -1 if ws is None else int((ws.view(torch.float32) != 0).sum())
for (N, C, H, W) in [(2, 256, 7, 7), (4, 64, 14, 14), (2, 256, 7, 7), (2, 256, 7, 7), (4, 64, 14, 14), (2, 128, 7, 7), (2, 256, 7, 7)]:
    x = (torch.randn(N, C, H, W, device=d) * 2 + 3).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g = torch.rand(C, device=d) + 0.5
    b = torch.randn(C, device=d)
    rm, rv = torch.zeros(C, device=d), torch.ones(C, device=d)
    torch.cuda.synchronize()
    before = ws_nz()
    y = bn_act(x, g, b, rm, rv, None, True, 0.1, 1e-5, False)
    torch.cuda.synchronize()
    xf = x.float().permute(0, 2, 3, 1).reshape(-1, C)
    mean = xf.mean(0)
    yf = torch.nn.functional.batch_norm(x.float(), None, None, g, b, True, 0.1, 1e-5)
    bad = ((rm - 0.1 * mean).abs() > 1e-4).nonzero().flatten().tolist()
    print(N, C, H, W, "nz before", before, "rm err", (rm - 0.1 * mean).abs().max().item(), "bad ch", bad[:10],
          "y err", (y.float() - yf).abs().max().item(), "nz after", ws_nz(), flush=True)
