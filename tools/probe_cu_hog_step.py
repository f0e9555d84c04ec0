"""Throughput of the ResNet-50 training step while a CU-holding kernel emulates
RCCL's resident collective kernels (VERDICT r4 "multi-GPU readiness you can test
on one GPU").

On an 8-GPU node the gradient all-reduces run as RCCL kernels that stay resident
on a few CUs per channel for most of the backward pass.  Here ``kfa_cu_hog``
(csrc/kernels/diag.hip: blocks of 96 KB LDS that sleep-spin for a fixed wall
time, one per CU) is launched on a side stream at the start of every step and
holds ``--hog`` CUs for ``--hog-ms``; the step time is measured with and without
it.  Run once per ``KFA_CONV_OVERSUB`` mode (the conv grid policy is read once per
process): 1 = persistent grids (2 blocks per CU), 2 = twice the resident slots,
0 = one block per tile.  The mode whose step time degrades least under the hog is
the one ``trainer/engine.py`` should set for ``world > 1``.

    KFA_CONV_OVERSUB=1 python tools/probe_cu_hog_step.py --hog 0,16,32
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--hog", default="0,16,32", help="CUs held per step (comma list)")
    ap.add_argument("--hog-ms", type=float, default=12.0, help="wall time each hog block holds its CU")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--batch", type=int, default=256)
    args = ap.parse_args()
    from kubeflow_controller_amd.models.resnet import resnet50
    from kubeflow_controller_amd.ops import _lib
    from kubeflow_controller_amd.ops.loss import cross_entropy
    from kubeflow_controller_amd.trainer.engine import DistInfo, Engine
    _lib.register("kfa_cu_hog", [_lib.I, _lib.L, _lib.P, _lib.P])
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    eng = Engine(resnet50(), lambda m, x, y: cross_entropy(m(x), y), optimizer="sgd", lr=0.1, momentum=0.9,
                 dist_info=DistInfo(device=dev))
    x = torch.randn(args.batch, 3, 224, 224, device=dev, dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (args.batch,), device=dev)
    side = torch.cuda.Stream(device=dev)
    flags = torch.zeros(1024, dtype=torch.int32, device=dev)
    for _ in range(args.warmup):
        eng.train_step(x, y)
    torch.cuda.synchronize()
    out = {"oversub": os.environ.get("KFA_CONV_OVERSUB", "1"), "hog_ms": args.hog_ms, "ms_per_step": {}}
    for hog in [int(h) for h in args.hog.split(",")]:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(args.steps):
            if hog:
                side.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(side):
                    _lib.call("kfa_cu_hog", hog, int(args.hog_ms * 1000), _lib.ptr(flags), _lib.stream())
            eng.train_step(x, y)
        torch.cuda.current_stream(dev).wait_stream(side)
        e1.record()
        torch.cuda.synchronize()
        out["ms_per_step"][hog] = round(e0.elapsed_time(e1) / args.steps, 3)
        print(f"[hog {hog} CUs x {args.hog_ms} ms] {out['ms_per_step'][hog]} ms/step", file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
