#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 training images/sec (whole node) on MI355X.

BASELINE.json metric "images/sec (whole node) ResNet-50 TFJob at 1/2/4/8
workers on MI355X".  One process per GPU, data-parallel over RCCL/xGMI, bf16
compute with fp32 master weights, fused SGD+momentum, synthetic ImageNet batch
(random-init weights, 224x224, 1000 classes) — weak scaling: the per-GPU batch
is fixed as N grows.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W`` prints ONE
JSON line.  Every timed step is a full step: forward, loss, backward, gradient
all-reduce (fp32 buckets overlapped with backward), optimizer update.

Launch modes:

* under ``torchrun`` (``WORLD_SIZE`` set): this process is one rank;
  ``WORLD_SIZE`` must equal ``--gpus``.
* plain ``python bench.py --gpus N`` with N > 1: the parent — which never
  touches the GPU — starts ``python -m torch.distributed.run --nproc-per-node N
  bench.py ...`` as a CHILD process (no exec), relays rank 0's JSON line and
  exits non-zero if any rank failed or the line does not say ``n_gpus == N``.
  This mirrors how the controller wires a multi-replica TFJob
  (reference ``pkg/tensorflow/distributed.go:127-159``, ``examples/tfjob/dist.yml``).

``KFA_DIST_BACKEND=gloo`` rehearses the multi-rank path with several ranks on
one GPU (or on the CPU with ``--device cpu --model resnet_tiny``: the CPU test).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_VALUE = None  # BASELINE.json "published": {} — the reference publishes no number
METRIC = "images/sec (whole node) ResNet-50 TFJob at 1/2/4/8 workers on MI355X"


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch (weak scaling)")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--grad-reduce", choices=["fp32", "bf16"], default="fp32",
                    help="dtype of the cross-rank gradient sum (fp32: bf16 grads are widened per bucket)")
    ap.add_argument("--model", choices=["resnet50", "resnet_tiny"], default="resnet50",
                    help="resnet_tiny only for the launcher's CPU/plumbing test")
    ap.add_argument("--device", choices=["auto", "cpu"], default="auto")
    ap.add_argument("--port", type=int, default=0, help="rendezvous port for the self-launch (0 = pick one)")
    ap.add_argument("--graph", choices=["auto", "on", "off"], default=os.environ.get("KFA_GRAPH", "off"),
                    help="replay the whole step as one HIP graph after the warm-up (Engine.capture); "
                         "auto/on: where Engine.graph_ok allows it (1 rank, SGD)")
    return ap.parse_args(argv)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args, argv) -> int:
    """Parent side of ``--gpus N`` without torchrun: run N ranks as a child job.

    Nothing here initialises the GPU (no torch import at all), so starting the
    child is safe on the GPU box."""
    port = args.port or _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "4")
    env["KFA_BENCH_CHILD"] = "1"
    print("bench: launching " + " ".join(cmd), file=sys.stderr, flush=True)
    p = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, text=True)
    line = None
    for out in p.stdout:  # stream: long runs keep printing progress to stderr, stdout carries the result
        s = out.strip()
        if s.startswith("{") and '"metric"' in s:
            line = s
        else:
            print(out, end="", file=sys.stderr, flush=True)
    rc = p.wait()
    if rc != 0:
        print(f"bench: rank job failed with exit code {rc}", file=sys.stderr)
        return rc
    if line is None:
        print("bench: no result line from rank 0", file=sys.stderr)
        return 1
    res = json.loads(line)
    if res.get("n_gpus") != args.gpus:
        print(f"bench: rank job reported n_gpus={res.get('n_gpus')} but --gpus {args.gpus}", file=sys.stderr)
        return 1
    print(line, flush=True)
    return 0


def run_rank(args) -> int:
    import torch

    from kubeflow_controller_amd.models.resnet import resnet50, resnet_tiny
    from kubeflow_controller_amd.ops.loss import cross_entropy
    from kubeflow_controller_amd.trainer.engine import Engine, init_distributed, timed_steps

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world_env}", file=sys.stderr)
        return 2
    info = init_distributed(prefer_gpu=(args.device != "cpu"))
    on_gpu = info.device.type == "cuda"
    if not on_gpu and args.model == "resnet50":
        raise SystemExit("bench.py needs an MI355X for ResNet-50 (no GPU visible)")
    torch.manual_seed(1234 + info.rank)
    model = resnet50() if args.model == "resnet50" else resnet_tiny(10)
    ncls = 1000 if args.model == "resnet50" else 10
    dtype = torch.bfloat16 if on_gpu else torch.float32
    engine = Engine(model, lambda m, x, y: cross_entropy(m(x), y), optimizer="sgd", lr=args.lr, momentum=0.9,
                    weight_decay=5e-5, bucket_mb=args.bucket_mb, dist_info=info,
                    compute_dtype=(torch.bfloat16 if on_gpu else None),
                    grad_reduce_dtype=(torch.float32 if args.grad_reduce == "fp32" else None))
    B = args.batch
    x = torch.randn(B, 3, args.image, args.image, device=info.device, dtype=dtype)
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, ncls, (B,), device=info.device)

    r = timed_steps(engine, (x, y), args.steps, args.warmup, graph=args.graph != "off")
    ms = r["elapsed"] / args.steps * 1e3
    ips = B * info.world * args.steps / r["elapsed"]
    if info.rank == 0:
        out = {
            "metric": METRIC,
            "value": round(ips, 2),
            "unit": "images/sec",
            "n_gpus": info.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (round(ips / BASELINE_VALUE, 4) if BASELINE_VALUE else None),
            "dtype": "bf16" if on_gpu else "fp32",
            "data": "synthetic (random ImageNet-shaped batch, random-init weights)",
            "config": {"model": "ResNet-50 v1.5" if args.model == "resnet50" else "resnet_tiny (CPU plumbing)",
                       "global_batch": B * info.world, "seq_len": None,
                       "image": args.image, "per_gpu_batch": B,
                       "parallelism": f"dp{info.world}" if info.world > 1 else "single",
                       "grad_reduce": args.grad_reduce if info.world > 1 else None,
                       "backend": (torch.distributed.get_backend() if torch.distributed.is_initialized()
                                   else None),
                       "optimizer": "SGD momentum 0.9 (fused HIP), fp32 master",
                       "hip_graph": engine._graph is not None,
                       "loss": r["loss"]},
        }
        print(json.dumps(out), flush=True)
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()
    return 0


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    if args.gpus < 1:
        print("bench: --gpus must be >= 1", file=sys.stderr)
        return 2
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args, argv)
    return run_rank(args)


if __name__ == "__main__":
    sys.exit(main())
