#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 training images/sec (whole node) on MI355X.

BASELINE.json metric "images/sec (whole node) ResNet-50 TFJob at 1/2/4/8
workers on MI355X".  One process per GPU (``torchrun --nproc-per-node N``),
data-parallel over RCCL/xGMI, bf16 compute with fp32 master weights, fused
SGD+momentum, synthetic ImageNet batch (random-init weights, 224x224, 1000
classes) — weak scaling: the per-GPU batch is fixed as N grows.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W`` prints ONE
JSON line on rank 0.  Every timed step is a full step: forward, loss, backward,
gradient all-reduce, optimizer update.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from kubeflow_controller_amd.models.resnet import resnet50  # noqa: E402
from kubeflow_controller_amd.ops.loss import cross_entropy  # noqa: E402
from kubeflow_controller_amd.trainer.engine import Engine, init_distributed, timed_steps  # noqa: E402

BASELINE_VALUE = None  # BASELINE.json "published": {} — the reference publishes no number


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch (weak scaling)")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--bucket-mb", type=float, default=16.0)
    ap.add_argument("--lr", type=float, default=0.1)
    args = ap.parse_args(argv)

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world_env}; using WORLD_SIZE", file=sys.stderr)
    info = init_distributed()
    if info.device.type != "cuda":
        raise SystemExit("bench.py needs an MI355X (no GPU visible)")
    torch.manual_seed(1234 + info.rank)
    torch.backends.cudnn.benchmark = True

    model = resnet50()
    engine = Engine(model, lambda m, x, y: cross_entropy(m(x), y), optimizer="sgd", lr=args.lr, momentum=0.9,
                    weight_decay=5e-5, bucket_mb=args.bucket_mb, dist_info=info)
    B = args.batch
    x = torch.randn(B, 3, args.image, args.image, device=info.device, dtype=torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (B,), device=info.device)

    r = timed_steps(engine, (x, y), args.steps, args.warmup)
    ms = r["elapsed"] / args.steps * 1e3
    ips = B * info.world * args.steps / r["elapsed"]
    if info.rank == 0:
        out = {
            "metric": "images/sec (whole node) ResNet-50 TFJob at 1/2/4/8 workers on MI355X",
            "value": round(ips, 2),
            "unit": "images/sec",
            "n_gpus": info.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (round(ips / BASELINE_VALUE, 4) if BASELINE_VALUE else None),
            "dtype": "bf16",
            "data": "synthetic (random ImageNet-shaped batch, random-init weights)",
            "config": {"model": "ResNet-50 v1.5", "global_batch": B * info.world, "seq_len": None,
                       "image": args.image, "per_gpu_batch": B,
                       "parallelism": f"dp{info.world}" if info.world > 1 else "single",
                       "optimizer": "SGD momentum 0.9 (fused HIP), fp32 master",
                       "loss": r["loss"]},
        }
        print(json.dumps(out), flush=True)
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
