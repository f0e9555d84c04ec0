#!/usr/bin/env python3
"""Per-launch GPU time of every own-kernel call of one training step, with the call's
integer arguments (shapes), by wrapping ``ops/_lib.call`` in CUDA events:

    python tools/launch_profile.py --model resnet50 [--filter conv] > out.txt

Each launch is bracketed by events on the current stream, so a time is that launch's
kernels (plus any library kernel the same C entry point issues).  Only the main
stream's order is meaningful; side-stream launches (weight gradients) are timed on
their own stream.  Prints one line per launch and a per-entry-point summary."""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--filter", default="")
    ap.add_argument("--warmup", type=int, default=3)
    args = ap.parse_args()
    from kubeflow_controller_amd.ops import _lib
    from kubeflow_controller_amd.models.resnet import resnet50
    from kubeflow_controller_amd.ops.loss import cross_entropy
    from kubeflow_controller_amd.trainer.engine import DistInfo, Engine
    d = torch.device("cuda")
    torch.manual_seed(0)
    eng = Engine(resnet50(), lambda m, x, y: cross_entropy(m(x), y), optimizer="sgd", lr=0.1, momentum=0.9,
                 dist_info=DistInfo(device=d))
    x = torch.randn(args.batch, 3, 224, 224, device=d).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (args.batch,), device=d)
    for _ in range(args.warmup):
        eng.train_step(x, y)
    torch.cuda.synchronize()
    recs = []
    orig = _lib.call

    def timed(name, *a):
        if args.filter and args.filter not in name:
            return orig(name, *a)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        orig(name, *a)
        e1.record()
        ints = [v for v in a if isinstance(v, int) and abs(v) < 1 << 20]
        recs.append((name, tuple(ints), e0, e1))
    _lib.call = timed
    eng.train_step(x, y)
    torch.cuda.synchronize()
    _lib.call = orig
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    for i, (name, ints, e0, e1) in enumerate(recs):
        ms = e0.elapsed_time(e1)
        tot[name] += ms
        cnt[name] += 1
        print(f"{i:4d} {name:34s} {ms * 1e3:9.1f} us  {ints}")
    print("\n# per entry point (ms / step, launches)")
    for n, t in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"{n:34s} {t:8.3f} ms  {cnt[n]:4d}")


if __name__ == "__main__":
    main()
