#!/usr/bin/env python3
"""Throughput of the non-headline BASELINE.json configs (BERT-base pre-training,
Wide&Deep) on MI355X: same contract as ``bench.py`` (W warmup, K timed full
steps bracketed by barrier + device sync, MAX over ranks, ONE JSON line).

    python tools/bench_model.py --model bert_base --batch 64 --seq 128
    torchrun --nproc-per-node N tools/bench_model.py --model bert_base --ps 2

``--ps P`` runs the parameter-server layout (P shard owners, reduce-scatter
push / owner-side fused Adam / all-gather pull) instead of all-reduce.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kubeflow_controller_amd.trainer.engine import Engine, init_distributed, timed_steps  # noqa: E402


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--model", default="bert_base", choices=["bert_base", "bert_large", "bert_tiny", "wide_deep",
                                                             "wide_deep_tiny"])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64, help="per-GPU batch")
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--ps", type=int, default=0, help="parameter-server shard owners (0 = all-reduce)")
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    args = ap.parse_args(argv)
    info = init_distributed()
    if info.device.type != "cuda":
        raise SystemExit("bench_model.py needs an MI355X")
    torch.manual_seed(1234)
    g = torch.Generator().manual_seed(1234 + info.rank)
    if args.model.startswith("bert"):
        from kubeflow_controller_amd.models.bert import (BertConfig, BertForPreTraining, bert_loss, flops_per_step,
                                                         synthetic_mlm_batch)
        cfg = {"bert_base": BertConfig.base, "bert_large": BertConfig.large, "bert_tiny": BertConfig.tiny}[args.model]()
        model = BertForPreTraining(cfg)
        batch = synthetic_mlm_batch(cfg, args.batch, args.seq, g, info.device)
        loss_fn, unit, flops = bert_loss, "sequences/sec", flops_per_step(cfg, args.batch, args.seq)
        metric = f"{args.model} pre-training sequences/sec (seq {args.seq}, whole node)"
    else:
        from kubeflow_controller_amd.models.wide_deep import (WideDeep, WideDeepConfig, prepare_batch, synthetic_batch,
                                                              wide_deep_loss)
        cfg = WideDeepConfig() if args.model == "wide_deep" else WideDeepConfig.tiny()
        model = WideDeep(cfg, device=info.device)
        batch = prepare_batch(model, *synthetic_batch(cfg, args.batch, g, "cpu"), info.device)
        loss_fn, unit, flops = wide_deep_loss, "examples/sec", None
        metric = f"{args.model} training examples/sec (whole node)"
    engine = Engine(model, loss_fn, optimizer="adam", lr=args.lr, weight_decay=0.01, bucket_mb=args.bucket_mb,
                    dist_info=info, channels_last=False, ps=args.ps)
    from kubeflow_controller_amd.ops import routes as _routes
    r = timed_steps(engine, batch, args.steps, args.warmup)
    ms = r["elapsed"] / args.steps * 1e3
    value = args.batch * info.world * args.steps / r["elapsed"]
    if info.rank == 0:
        out = {"metric": metric, "value": round(value, 2), "unit": unit, "n_gpus": info.world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
               "vs_baseline": None, "dtype": "bf16", "data": "synthetic (random ids / features, random-init weights)",
               "config": {"model": args.model, "global_batch": args.batch * info.world,
                          "seq_len": args.seq if args.model.startswith("bert") else None,
                          "parallelism": (f"{info.world}w+{args.ps}ps" if args.ps else f"dp{info.world}"),
                          "routes": _routes.summary(), "loss": r["loss"]}}
        if flops:
            out["tflops_per_gpu"] = round(flops / (ms / 1e3) / 1e12, 1)
        print(json.dumps(out), flush=True)
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
