import torch
from kubeflow_controller_amd.models.resnet import ResNet
from kubeflow_controller_amd.ops import conv as convmod
d = torch.device("cuda")
torch.manual_seed(0)
m = ResNet((2, 1, 1, 1), num_classes=10, width=64).to(d).to(memory_format=torch.channels_last)
for p in m.parameters():
    if p.dim() >= 2:
        p.data = p.data.to(torch.bfloat16)
for mod in m.modules():
    if hasattr(mod, "bn3"):
        torch.nn.init.uniform_(mod.bn3.weight, 0.5, 1.5)
x = torch.randn(4, 3, 32, 32, device=d).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
names = ["input"] + [n for n, _ in m.named_parameters()]
res = []
for enabled, joins in ((True, True), (True, False), (False, False)):
    convmod.ENABLED = enabled
    if not joins:
        convmod.GradJoin.branch = lambda self, x: x
        orig = convmod.conv2d
    m.zero_grad(set_to_none=True)
    xr = x.clone().requires_grad_()
    out = m(xr)
    out.float().square().mean().backward()
    res.append([xr.grad.float()] + [p.grad.float() for p in m.parameters()])
for tag, (i, j) in (("igemm+join vs vendor", (0, 2)), ("igemm nojoin vs vendor", (1, 2))):
    print("==", tag)
    for n, a, b in zip(names, res[i], res[j]):
        e = (a - b).abs().max().item(); s = b.abs().max().item()
        if e > 0.05 * max(s, 1e-3):
            print(f"{n:40s} err {e:.4g} scale {s:.4g}")
