"""Does hipBLASLt kernel selection depend on the weight's alignment inside the flat buffer?"""
import torch


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it


d = torch.device("cuda")
for (M, N, K) in [(16384, 3072, 768), (16384, 2304, 768), (16384, 768, 3072), (16384, 768, 768)]:
    x = torch.randn(M, K, device=d, dtype=torch.bfloat16)
    dy = torch.randn(M, N, device=d, dtype=torch.bfloat16)
    row = []
    for off in (0, 8, 64, 128, 256):
        buf = torch.randn(N * K + 512, device=d, dtype=torch.bfloat16)
        w = torch.as_strided(buf, (N, K), (K, 1), off)
        fl = 2 * M * N * K
        tf = t(lambda: torch.mm(x, w.t()))
        td = t(lambda: torch.mm(dy, w))
        gw = torch.as_strided(torch.zeros_like(buf), (N, K), (K, 1), off)
        tw = t(lambda: gw.addmm_(dy.t(), x))
        row.append(f"off{off}: fwd {fl / tf / 1e9:.0f} dgrad {fl / td / 1e9:.0f} wgrad {fl / tw / 1e9:.0f}")
    print(M, N, K, " | ".join(row), flush=True)
