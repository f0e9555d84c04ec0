import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.ops.conv import wgrad_into
d = torch.device("cuda")
for rows, co, ci in [(5120, 30528, 768), (5120, 768, 768), (5120, 768, 30528)]:
    x = torch.randn(rows, ci, device=d).to(torch.bfloat16)
    dy = torch.randn(rows, co, device=d).to(torch.bfloat16)
    out = torch.zeros(co, ci, device=d)
    f = lambda: wgrad_into(x, dy, out, 1, 1, rows, ci, 1, rows, co, 1, 1, 1, 0, accumulate=True)
    for _ in range(3): f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    best = 1e9
    for _ in range(3):
        e0.record()
        for _ in range(10): f()
        e1.record(); torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / 10)
    print(f"PP={os.environ.get('KFA_WGRAD_PP', '1')} {rows}x{co}x{ci}: {best*1e3:8.1f} us {2*rows*co*ci/best/1e9:6.0f} TF/s", flush=True)
