"""Probe: stock-PyTorch ResNet-50 training step on one MI355X (bf16, NHWC).

Used once to establish what the vendor path (MIOpen convs, PyTorch BN) costs per
kernel, so the hand-written kernels can be prioritised by measured time.
"""
import time, sys, torch, torch.nn as nn, torch.nn.functional as F

class Bottleneck(nn.Module):
    def __init__(s, cin, mid, cout, stride):
        super().__init__()
        s.c1 = nn.Conv2d(cin, mid, 1, bias=False); s.b1 = nn.BatchNorm2d(mid)
        s.c2 = nn.Conv2d(mid, mid, 3, stride, 1, bias=False); s.b2 = nn.BatchNorm2d(mid)
        s.c3 = nn.Conv2d(mid, cout, 1, bias=False); s.b3 = nn.BatchNorm2d(cout)
        s.down = None
        if stride != 1 or cin != cout:
            s.down = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))
    def forward(s, x):
        y = F.relu(s.b1(s.c1(x))); y = F.relu(s.b2(s.c2(y))); y = s.b3(s.c3(y))
        return F.relu(y + (x if s.down is None else s.down(x)))

class R50(nn.Module):
    def __init__(s):
        super().__init__()
        s.stem = nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(), nn.MaxPool2d(3, 2, 1))
        L = []; cin = 64
        for mid, n, st in [(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)]:
            for i in range(n):
                L.append(Bottleneck(cin, mid, mid * 4, st if i == 0 else 1)); cin = mid * 4
        s.layers = nn.Sequential(*L); s.fc = nn.Linear(2048, 1000)
    def forward(s, x):
        x = s.layers(s.stem(x)); return s.fc(x.mean((2, 3)))

def main():
    bs = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    torch.backends.cudnn.benchmark = True
    m = R50().cuda().to(memory_format=torch.channels_last).to(torch.bfloat16)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
    x = torch.randn(bs, 3, 224, 224, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (bs,), device="cuda")
    def step():
        opt.zero_grad(set_to_none=True)
        loss = F.cross_entropy(m(x).float(), y); loss.backward(); opt.step()
    for _ in range(5): step()
    torch.cuda.synchronize(); t = time.time()
    for _ in range(steps): step()
    torch.cuda.synchronize(); dt = (time.time() - t) / steps
    print(f"torch-r50 bs={bs} ms/step={dt*1e3:.2f} img/s={bs/dt:.1f}", flush=True)

if __name__ == "__main__":
    main()
