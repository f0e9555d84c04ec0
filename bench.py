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
    ap.add_argument("--ps", type=int, default=0,
                    help="parameter-server shard owners (K < N): gradients reduce-scattered to the owners, "
                         "owner-side fused optimizer, all-gather pull — the 'N workers + K PS' TFJob layout "
                         "(reference examples/tfjob/dist.yml); 0 = all-reduce data parallel")
    ap.add_argument("--watchdog", type=float, default=float(os.environ.get("KFA_BENCH_WATCHDOG", "900")),
                    help="seconds before a hung run is killed with every rank's stack dumped (0 = off)")
    ap.add_argument("--init-timeout", type=float, default=float(os.environ.get("KFA_DIST_INIT_TIMEOUT", "300")),
                    help="torch.distributed init / collective timeout (seconds)")
    return ap.parse_args(argv)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_pids(pid: int):
    """PIDs of the python rank processes under the torchrun child (psutil)."""
    try:
        import psutil
        return [c.pid for c in psutil.Process(pid).children(recursive=True)]
    except Exception:
        return []


def launch_ranks(args, argv) -> int:
    """Parent side of ``--gpus N`` without torchrun: run N ranks as a child job.

    Nothing here initialises the GPU (no torch import at all), so starting the
    child is safe on the GPU box.  Each rank writes its stderr to
    ``<logdir>/rank<R>.err``; this parent streams those files to its own stderr
    with a ``[rank R]`` prefix, so a failure or a hang names the rank.  A
    wall-clock watchdog (``--watchdog`` seconds) asks every rank to dump its
    Python stacks (SIGUSR1, ``faulthandler``), prints each rank's last stderr
    lines and kills the whole child job (its own process group), exit 124."""
    import signal
    import tempfile
    import time

    port = args.port or _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]
    logdir = tempfile.mkdtemp(prefix="kfa_bench_")
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "4")
    env["KFA_BENCH_CHILD"] = "1"
    env["KFA_BENCH_RANKLOG_DIR"] = logdir
    print("bench: launching " + " ".join(cmd), file=sys.stderr, flush=True)
    p = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, text=True, start_new_session=True)
    lines: list = []

    def _read_stdout():
        for out in p.stdout:
            lines.append(out)

    import threading
    reader = threading.Thread(target=_read_stdout, daemon=True)
    reader.start()
    offsets = {}

    def _pump(final: bool = False):
        for r in range(args.gpus):
            path = os.path.join(logdir, f"rank{r}.err")
            if not os.path.exists(path):
                continue
            with open(path, "r", errors="replace") as f:
                f.seek(offsets.get(r, 0))
                chunk = f.read()
                offsets[r] = f.tell()
            if final and chunk and not chunk.endswith("\n"):
                chunk += "\n"
            body = chunk if final else chunk[:chunk.rfind("\n") + 1]
            offsets[r] -= len(chunk) - len(body)
            for ln in body.splitlines():
                print(f"[rank {r}] {ln}", file=sys.stderr, flush=True)

    def _tail(r: int, n: int = 25) -> str:
        path = os.path.join(logdir, f"rank{r}.err")
        if not os.path.exists(path):
            return "(no stderr file: the rank never started)"
        with open(path, "r", errors="replace") as f:
            return "".join(f.readlines()[-n:])

    # the ranks' own watchdogs fire first (stack dump + exit); this one is the backstop
    deadline = time.monotonic() + (args.watchdog + 60 if args.watchdog > 0 else float("inf"))
    timed_out = False
    while p.poll() is None:
        time.sleep(0.5)
        _pump()
        for ln in lines[:]:
            s = ln.strip()
            if not (s.startswith("{") and '"metric"' in s):
                print(ln, end="", file=sys.stderr, flush=True)
                lines.remove(ln)
        if time.monotonic() > deadline:
            timed_out = True
            break
    if timed_out:
        print(f"bench: WATCHDOG: rank job still running after {args.watchdog:.0f} s; dumping rank stacks "
              "and killing it", file=sys.stderr, flush=True)
        for pid in _rank_pids(p.pid):
            try:
                os.kill(pid, signal.SIGUSR1)
            except OSError:
                pass
        time.sleep(3.0)
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except OSError:
            pass
        p.wait()
    rc = p.wait()
    reader.join(timeout=5)
    _pump(final=True)
    line = None
    for out in lines:
        s = out.strip()
        if s.startswith("{") and '"metric"' in s:
            line = s
        else:
            print(out, end="", file=sys.stderr, flush=True)
    if timed_out or rc != 0:
        why = "timed out (watchdog)" if timed_out else f"failed with exit code {rc}"
        print(f"bench: rank job {why}; last stderr lines per rank:", file=sys.stderr)
        for r in range(args.gpus):
            print(f"---- rank {r} ----\n{_tail(r)}", file=sys.stderr)
        return 124 if timed_out else rc
    if line is None:
        print("bench: no result line from rank 0", file=sys.stderr)
        return 1
    res = json.loads(line)
    if res.get("n_gpus") != args.gpus:
        print(f"bench: rank job reported n_gpus={res.get('n_gpus')} but --gpus {args.gpus}", file=sys.stderr)
        return 1
    print(line, flush=True)
    return 0


def _arm_rank_watchdog(args, rank: int) -> None:
    """Per-rank hang guard, also under the driver's own torchrun (which never
    goes through ``launch_ranks``): after ``--watchdog`` seconds every thread's
    Python stack goes to stderr and the rank exits non-zero, so a wedged RCCL
    collective ends the job with a diagnosis instead of burning the driver's
    timeout.  SIGUSR1 (the launcher's watchdog) and SIGTERM (torchrun stopping
    the survivors of a failed rank) dump the stacks too.
    With ``KFA_BENCH_RANKLOG_DIR`` (set by ``launch_ranks``) stderr goes to
    ``rank<R>.err`` there."""
    import faulthandler
    import signal
    d = os.environ.get("KFA_BENCH_RANKLOG_DIR")
    if d:
        fd = os.open(os.path.join(d, f"rank{rank}.err"), os.O_WRONLY | os.O_CREAT | os.O_APPEND, 0o644)
        os.dup2(fd, 2)
        os.close(fd)
        sys.stderr = os.fdopen(2, "w", buffering=1, closefd=False)
    faulthandler.enable()
    faulthandler.register(signal.SIGUSR1, all_threads=True)
    # torchrun SIGTERMs the surviving ranks when one fails: show where they were
    faulthandler.register(signal.SIGTERM, all_threads=True, chain=True)
    if args.watchdog > 0:
        faulthandler.dump_traceback_later(args.watchdog, exit=True)


def _test_hang(rank: int) -> None:
    """Test hook (``KFA_BENCH_HANG_RANK=r``): rank r stops before the timed
    region, as a rank stuck in a collective would; the others then wait in the
    barrier.  Exercised by ``tests/test_dist_cpu.py``."""
    if os.environ.get("KFA_BENCH_HANG_RANK") == str(rank):
        import time
        print(f"bench: rank {rank} hanging on purpose (KFA_BENCH_HANG_RANK)", file=sys.stderr, flush=True)
        while True:
            time.sleep(1.0)


def run_rank(args) -> int:
    import torch

    from kubeflow_controller_amd.models.resnet import resnet50, resnet_tiny
    from kubeflow_controller_amd.ops import routes
    from kubeflow_controller_amd.ops.loss import cross_entropy
    from kubeflow_controller_amd.trainer.engine import Engine, init_distributed, timed_steps

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world_env}", file=sys.stderr)
        return 2
    if args.ps >= args.gpus and args.gpus > 1:
        print(f"bench: --ps {args.ps} needs fewer PS shard owners than ranks ({args.gpus})", file=sys.stderr)
        return 2
    _arm_rank_watchdog(args, int(os.environ.get("RANK", "0")))
    info = init_distributed(prefer_gpu=(args.device != "cpu"), timeout_s=args.init_timeout)
    on_gpu = info.device.type == "cuda"
    if not on_gpu and args.model == "resnet50":
        raise SystemExit("bench.py needs an MI355X for ResNet-50 (no GPU visible)")
    torch.manual_seed(1234 + info.rank)
    model = resnet50() if args.model == "resnet50" else resnet_tiny(10)
    ncls = 1000 if args.model == "resnet50" else 10
    dtype = torch.bfloat16 if on_gpu else torch.float32
    engine = Engine(model, lambda m, x, y: cross_entropy(m(x), y), optimizer="sgd", lr=args.lr, momentum=0.9,
                    weight_decay=5e-5, bucket_mb=args.bucket_mb, dist_info=info, ps=args.ps,
                    compute_dtype=(torch.bfloat16 if on_gpu else None),
                    grad_reduce_dtype=(torch.float32 if args.grad_reduce == "fp32" else None))
    B = args.batch
    x = torch.randn(B, 3, args.image, args.image, device=info.device, dtype=dtype)
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, ncls, (B,), device=info.device)

    _test_hang(info.rank)
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
                       "parallelism": (f"{info.world}w{args.ps}ps" if (args.ps and info.world > 1) else
                                       f"dp{info.world}" if info.world > 1 else "single"),
                       "grad_reduce": args.grad_reduce if info.world > 1 else None,
                       "backend": (torch.distributed.get_backend() if torch.distributed.is_initialized()
                                   else None),
                       # layer / default group / RCCL transport per peer, and the per-step
                       # compute-stream wait for the gradient collectives after backward
                       "comm": dict(engine.comm_info(), comm_wait_ms=r["comm_wait_ms"]),
                       "routes": routes.summary(),
                       "optimizer": "SGD momentum 0.9 (fused HIP), fp32 master",
                       "hip_graph": engine._graph is not None,
                       "loss": r["loss"]},
        }
        print(json.dumps(out), flush=True)
    engine.comm.destroy()
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()
    import faulthandler
    faulthandler.cancel_dump_traceback_later()
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
