"""The TFJob replica runtime: what every Worker / PS / Local process runs.

MI355X-native replacement of the reference's TensorFlow-1.x workload scripts
(``examples/workdir/mnist_replica.py``, ``mnist_softmax.py``) — same CLI flags,
same roles, same log lines, PyTorch-ROCm + hand-written HIP kernels + RCCL inside:

  python -m kubeflow_controller_amd.trainer.replica --model mnist_mlp \\
      --worker_hosts=... --ps_hosts=... --job_name=worker --task_index=0 \\
      [--train_steps 200 --batch_size 100 --learning_rate 0.01 --sync_replicas]

Roles (``mnist_replica.py:107-122``):
* ``local`` — single process, no collectives (the Local TFJob).
* ``worker`` — joins the worker collective (RCCL on a GPU, gloo on CPU) via
  the chief's endpoint; trains; reports to the coordination store.
* ``ps`` — coordinator: attaches to the chief's store, tracks the global step
  and exits 0 once every worker reported done.  The reference's PS
  ``server.join()``s forever; here the job completes.
  Parameter shards are owned by worker ranks (``parallel/ps.py``).

Update semantics (``--ps_mode``):
* ``async`` — the reference's default (no ``--sync_replicas``): PS tasks hold
  the variables and Adam state and serve pull/push requests from any worker
  (``parallel/async_ps.py``); workers run at their own pace and stop once the
  global step (advanced by every push) reaches ``train_steps``.
* ``collective`` — push = RCCL reduce-scatter -> owner-side fused optimizer ->
  pull = all-gather on the worker GPUs (PS processes coordinate only;
  co-located PS); without PS, bucketed all-reduce.  Used for
  ``--sync_replicas`` and for the large models (``auto``), where moving the
  variables through host memory every step would dominate.
"""
from __future__ import annotations

import argparse
import datetime
import json
import math
import os
import sys
import time
from typing import Optional

import torch
import torch.distributed as dist

from .cluster import ClusterSpec, add_cluster_flags, local_device, parse_cluster

STEP_KEY = "kfa/global_step"
DONE_KEY = "kfa/workers_done"


def _log(msg: str) -> None:
    print(msg, flush=True)


def _use_gpu(args) -> bool:
    if args.device == "cpu":
        return False
    vis = os.environ.get("HIP_VISIBLE_DEVICES")
    if vis is not None and vis.strip() == "":
        return False  # the supervisor bound no GPU to this replica
    return torch.cuda.is_available()


_armed_at = [0.0]


def _arm_watchdog(args) -> None:
    """(Re-)arm the replica's hang guard: if the next ``--hang_timeout`` seconds
    pass without another call (one per training step; the rendezvous and the
    first, kernel-tuning step get the same budget), every thread's Python stack
    goes to stderr (the replica log) and the process exits 1, so the supervisor
    applies the replica's restartPolicy (``dist.yml:45`` OnFailure) instead of
    the job hanging on a wedged collective or a dead peer."""
    t = getattr(args, "hang_timeout", 0)
    now = time.monotonic()
    # re-arming costs ~0.1 ms (a timer thread restart): at most 8 times per timeout period
    if t > 0 and now - _armed_at[0] >= t / 8:
        import faulthandler
        try:
            faulthandler.dump_traceback_later(t, exit=True)
        except (ValueError, OSError, RuntimeError, AttributeError):  # stderr without a file descriptor (in-process)
            return
        _armed_at[0] = now


def _disarm_watchdog() -> None:
    import faulthandler
    faulthandler.cancel_dump_traceback_later()
    _armed_at[0] = 0.0


def _install_stack_dumps() -> None:
    """SIGTERM (the supervisor stopping a replica) and SIGUSR1 print all stacks first."""
    import faulthandler
    import signal
    try:
        faulthandler.enable()
        faulthandler.register(signal.SIGUSR1, all_threads=True)
        faulthandler.register(signal.SIGTERM, all_threads=True, chain=True)
    except (AttributeError, ValueError, RuntimeError, OSError):  # in-process caller without a real stderr fd
        pass


def _test_hang(spec: ClusterSpec, step: int) -> None:
    """Test hook: ``KFA_TEST_HANG=<job_name>:<task_index>:<step>`` stops that replica
    at that step as a replica stuck in a collective would (tests/test_e2e_cpu.py)."""
    v = os.environ.get("KFA_TEST_HANG")
    if v and v == f"{spec.job_name}:{spec.task_index}:{step}":
        _log(f"{spec.job_name} {spec.task_index}: hanging at step {step} on purpose (KFA_TEST_HANG)")
        while True:
            time.sleep(1.0)


def _pg_timeout(args) -> datetime.timedelta:
    return datetime.timedelta(seconds=getattr(args, "dist_timeout", 300.0))


def _store(spec: ClusterSpec, is_master: bool, timeout: float = 300.0):
    host, port = spec.rendezvous()
    return dist.TCPStore(host, port, spec.num_workers if is_master else None, is_master,
                         timeout=datetime.timedelta(seconds=timeout), wait_for_workers=False)


# ------------------------------------------------------------------ models
def build(args, device):
    from ..models import mnist
    from ..ops.loss import clipped_sum_cross_entropy, cross_entropy
    name = args.model
    # --loss sum_clipped: mnist_replica.py:168's -reduce_sum(y_ * log(clip(y, 1e-10, 1)));
    # mean: mnist_softmax.py:57-58's mean softmax cross-entropy (every other model)
    xent = clipped_sum_cross_entropy if getattr(args, "loss", "mean") == "sum_clipped" else cross_entropy
    if name == "mnist_softmax":
        data = mnist.SyntheticMNIST(seed=args.seed)
        return mnist.MnistSoftmax(), data, lambda m, x, y: xent(m(x).float(), y)
    if name == "mnist_mlp":
        data = mnist.SyntheticMNIST(seed=args.seed)
        return mnist.MnistMLP(args.hidden_units), data, lambda m, x, y: xent(m(x).float(), y)
    if name in ("resnet50", "resnet_tiny"):
        from ..models.resnet import resnet50, resnet_tiny
        model = resnet50() if name == "resnet50" else resnet_tiny(10)
        return model, None, lambda m, x, y: cross_entropy(m(x), y)
    if name in ("bert_base", "bert_tiny"):
        from ..models.bert import BertConfig, BertForPreTraining, bert_loss
        cfg = BertConfig.base() if name == "bert_base" else BertConfig.tiny()
        return BertForPreTraining(cfg), None, bert_loss
    if name in ("wide_deep", "wide_deep_tiny"):
        from ..models.wide_deep import WideDeep, WideDeepConfig, wide_deep_loss
        cfg = WideDeepConfig() if name == "wide_deep" else WideDeepConfig.tiny()
        # table rows interleave over every worker rank (balanced sparse-update work);
        # --embedding_owners ps keeps them on the ranks co-located with the PS tasks
        cfg.owners = (getattr(args, "num_ps", 0) or None) if getattr(args, "embedding_owners", "all") == "ps" \
            else None
        return WideDeep(cfg, device=device), None, wide_deep_loss
    raise SystemExit(f"unknown --model {name}")


def synthetic_batch(args, model, device, rank: int):
    g = torch.Generator(device="cpu").manual_seed(args.seed + 1000 * rank)
    B = args.batch_size
    if args.model.startswith("resnet"):
        s = 224 if args.model == "resnet50" else 32
        x = torch.randn(B, 3, s, s, generator=g).to(device)
        x = x.to(torch.bfloat16 if device.type == "cuda" else torch.float32)
        x = x.contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 1000 if args.model == "resnet50" else 10, (B,), generator=g).to(device)
        return (x, y)
    if args.model.startswith("bert"):
        from ..models.bert import synthetic_mlm_batch
        return synthetic_mlm_batch(model.cfg, B, args.seq_len, g, device)
    if args.model.startswith("wide_deep"):
        from ..models.wide_deep import prepare_batch
        from ..models.wide_deep import synthetic_batch as wd_batch
        return prepare_batch(model, *wd_batch(model.cfg, B, g, "cpu"), device)
    raise ValueError(args.model)


def _aggregate(spec: ClusterSpec, args) -> int:
    """Gradients per update on the PS service loop: 0 = async (the reference's
    default); ``--sync_replicas`` aggregates ``--replicas_to_aggregate``
    (default: every worker), ``mnist_replica.py:172-182``."""
    if not args.sync_replicas:
        return 0
    n = args.replicas_to_aggregate if args.replicas_to_aggregate is not None else spec.num_workers
    if not 1 <= n <= spec.num_workers:
        raise SystemExit(f"--replicas_to_aggregate {n}: must be in 1..{spec.num_workers} (the number of workers)")
    return n


def _async_mode(spec: ClusterSpec, args) -> bool:
    """True: the PS service loop (``parallel/async_ps.py``) — async pushes, or
    ``--sync_replicas`` aggregation of N < W gradients with stale ones dropped.
    False: the collective path (RCCL reduce-scatter / all-gather or all-reduce),
    which always aggregates every worker's gradient, so it refuses N != W."""
    n = args.replicas_to_aggregate
    partial = args.sync_replicas and n is not None and n != spec.num_workers
    if spec.is_local or not spec.ps:
        if partial and not spec.is_local:
            raise SystemExit(f"--replicas_to_aggregate {n} with {spec.num_workers} workers needs PS tasks: the "
                             "all-reduce path sums every worker's gradient (no PS to drop stale ones)")
        return False
    if args.ps_mode == "auto":  # the reference's default update mode is async (no --sync_replicas)
        if partial:
            return True
        return not args.sync_replicas and (args.model.startswith("mnist") or args.ps_transport == "device")
    if args.ps_mode == "collective" and partial:
        raise SystemExit(f"--replicas_to_aggregate {n} != {spec.num_workers} workers is not supported by "
                         "--ps_mode collective (reduce-scatter aggregates every worker); use --ps_mode async")
    return args.ps_mode == "async"


# ------------------------------------------------------------------ roles
TRANSPORT_KEY = "kfa/async_ps/transport"


def _ps_transport(args, has_gpu: bool) -> str:
    if args.ps_transport == "auto":
        return "device" if has_gpu else "host"
    if args.ps_transport == "device" and not has_gpu:
        raise SystemExit("--ps_transport device: this PS replica has no GPU (set KFA_PS_COLOCATE=1 in its template)")
    return args.ps_transport


def run_ps_async(spec: ClusterSpec, args) -> int:
    """PS task of the async mode: own the round-robin-placed variables, serve pulls/pushes."""
    from ..parallel.async_ps import AsyncPSServer, DeviceAsyncPSServer
    W, P = spec.num_workers, len(spec.ps)
    rank = W + spec.task_index
    _log(f"PS {spec.task_index}: async parameter server, rank {rank} of {W} workers + {P} ps at "
         f"{'%s:%d' % spec.rendezvous()}")
    t0 = time.time()
    store = None
    while store is None:
        try:
            store = _store(spec, False, timeout=args.ps_connect_timeout)
        except Exception as e:  # chief not up yet
            if time.time() - t0 > args.ps_connect_timeout:
                _log(f"PS {spec.task_index}: chief unreachable ({e}); exiting")
                return 1
            time.sleep(0.5)
    dist.init_process_group("gloo", store=store, rank=rank, world_size=W + P, timeout=_pg_timeout(args))
    torch.manual_seed(args.seed)  # same initial values as every worker's model
    use_gpu = _use_gpu(args)
    transport = _ps_transport(args, use_gpu)
    if spec.task_index == 0:
        store.set(TRANSPORT_KEY, transport)
    model, _, _ = build(args, torch.device("cpu"))
    agg = _aggregate(spec, args)
    if transport == "device":
        torch.cuda.set_device(local_device())
        server = DeviceAsyncPSServer(list(model.named_parameters()), W, P, spec.task_index, store,
                                     torch.device("cuda", local_device()), lr=args.learning_rate, optimizer=args.optimizer,
                                     aggregate=agg, channels_last=model.__class__.__name__ == "ResNet")
    else:
        server = AsyncPSServer(list(model.named_parameters()), W, P, spec.task_index, lr=args.learning_rate,
                               optimizer=args.optimizer, aggregate=agg)
    _log(f"PS {spec.task_index}: serving {len(server.names)} variables ({server.w.numel()} values), "
         f"{transport}-resident ({'GPU HBM, HIP IPC pull/push' if transport == 'device' else 'host memory'}; "
         f"requests over {server.p2p!r}), "
         + (f"sync replicas: mean of {agg} of {W} workers' gradients per update, stale ones dropped" if agg
            else "async updates"))
    pushes = server.serve(log=_log)
    server.close()
    _log(f"PS {spec.task_index}: all {W} workers done; {pushes} gradients applied in {server.global_step} updates, "
         f"{server.dropped} stale dropped; exiting")
    dist.destroy_process_group()
    return 0


def run_worker_async(spec: ClusterSpec, args) -> int:
    """Between-graph replicated async training against the PS tasks (``mnist_replica.py:251-264``)."""
    from ..ops.loss import accuracy, cross_entropy
    from ..parallel.async_ps import AsyncPSClient, DeviceAsyncPSClient
    W, P = spec.num_workers, len(spec.ps)
    use_gpu = _use_gpu(args)
    device = torch.device("cuda", local_device()) if use_gpu else torch.device("cpu")
    if not use_gpu and not os.environ.get("OMP_NUM_THREADS"):
        torch.set_num_threads(max(1, (os.cpu_count() or 1) // (W + P)))
    if use_gpu:
        torch.cuda.set_device(local_device())
    store = _store(spec, spec.is_chief)
    dist.init_process_group("gloo", store=store, rank=spec.task_index, world_size=W + P, timeout=_pg_timeout(args))
    torch.manual_seed(args.seed)
    args.num_ps = P
    model, data, loss_fn = build(args, device)
    model = model.to(device)
    if use_gpu and args.bf16:  # the compute copy: bf16 matrices, fp32 vectors (the PS keeps fp32 masters)
        for p in model.parameters():
            if p.dim() >= 2:
                p.data = p.data.to(torch.bfloat16)
        if model.__class__.__name__ == "ResNet":
            model = model.to(memory_format=torch.channels_last)
    transport = store.get(TRANSPORT_KEY).decode()  # PS 0 decides (waits for it to come up)
    if transport == "device" and not use_gpu:
        raise SystemExit("device-resident async PS needs GPU workers")
    if transport == "device":
        client = DeviceAsyncPSClient(list(model.named_parameters()), W, P, spec.task_index, store, log=_log)
        zero_grad = client.zero_grad
        transport = "+".join(sorted(set(client.transports))) + " transport; " + "; ".join(client.transport_desc)
    else:
        client = AsyncPSClient(list(model.named_parameters()), W, P)
        zero_grad = lambda: model.zero_grad(set_to_none=False)  # noqa: E731
    agg = _aggregate(spec, args)
    _log(f"Worker {spec.task_index}: {W} workers, {P} ps, device {device}, model {args.model}, "
         f"{sum(p.numel() for p in model.parameters())} params, "
         f"{'sync replicas (%d of %d aggregated)' % (agg, W) if agg else 'async'} parameter server "
         f"({transport if transport.endswith(')') else transport + ' transport'})")
    fixed = None if data is not None else synthetic_batch(args, model, device, spec.task_index)
    t_begin = time.time()
    _log(f"Training begins @ {t_begin:f}")
    local_step, global_step, t_first, loss = 0, 0, None, None
    while global_step < args.train_steps:
        _arm_watchdog(args)
        _test_hang(spec, local_step)
        if data is not None:
            xb, yb = data.next_batch(args.batch_size)
            batch = (xb.to(device), yb.to(device))
        else:
            batch = fixed
        client.pull()
        zero_grad()
        loss = loss_fn(model, *batch)
        loss.backward()
        global_step = client.push()
        local_step += 1
        if t_first is None:
            t_first = time.time()
        if args.log_every and local_step % args.log_every == 0:
            _log(f"{time.time():f}: Worker {spec.task_index}: training step {local_step} done "
                 f"(global step: {global_step})")
    t_end = time.time()
    _log(f"Training ends @ {t_end:f}")
    _log(f"Training elapsed time: {t_end - t_begin:f} s")
    if t_first is not None and local_step > 1:
        sps = (local_step - 1) / max(t_end - t_first, 1e-9)
        _log(f"Steady-state: {sps:.1f} steps/s/worker, {sps * args.batch_size:.1f} examples/s (this worker)")
    if agg:
        _log(f"Worker {spec.task_index}: {local_step} pushes, {client.pushes_dropped} dropped as stale")
    client.pull()  # evaluate the PS's current variables, as the reference's session does
    client.done()
    client.close()
    if data is not None:
        with torch.no_grad():
            model.eval()
            vx, vy = data.validation
            ce = float(cross_entropy(model(vx.to(device)).float(), vy.to(device))) * vx.shape[0]
            _log(f"After {global_step} training step(s), validation cross entropy = {ce:g}")
            tx, ty = data.test
            _log(f"Test accuracy: {float(accuracy(model(tx.to(device)).float(), ty.to(device))):.4f}")
    elif loss is not None:
        _log(f"Final loss: {float(loss):.5f}")
    dist.destroy_process_group()
    return 0


def run_ps(spec: ClusterSpec, args) -> int:
    """PS coordinator: follow the global step until every worker is done."""
    _log(f"PS {spec.task_index}: joining job with {spec.num_workers} workers at "
         f"{'%s:%d' % spec.rendezvous()}")
    t0 = time.time()
    store = None
    while store is None:
        try:
            store = _store(spec, False, timeout=args.ps_connect_timeout)
        except Exception as e:  # chief not up yet
            if time.time() - t0 > args.ps_connect_timeout:
                _log(f"PS {spec.task_index}: chief unreachable ({e}); exiting")
                return 1
            time.sleep(0.5)
    last = -1
    while True:
        try:
            done = int(store.add(DONE_KEY, 0))
            step = int(store.add(STEP_KEY, 0))
        except Exception:
            # the chief's store is gone: the job finished (workers exit after reporting)
            _log(f"PS {spec.task_index}: store closed at global step {last}; done")
            return 0
        if step != last and step % max(1, args.log_every) == 0:
            _log(f"PS {spec.task_index}: global step {step}")
        last = step
        if done >= spec.num_workers:
            _log(f"PS {spec.task_index}: all {done} workers done at global step {step}; exiting")
            return 0
        time.sleep(0.2)


GRAPH_AUTO_MS = float(os.environ.get("KFA_GRAPH_AUTO_MS", "5"))


def run_worker(spec: ClusterSpec, args) -> int:
    """Worker / Local replica on the shared training engine (``trainer/engine.py``):
    the same step ``bench.py`` times, plus the reference's logging, global-step
    bookkeeping, validation and ``spec.modelDir`` checkpoints."""
    from ..ops.loss import accuracy, cross_entropy
    from ..parallel.ps import ps_assignment, ps_owner_ranks
    from . import checkpoint
    from .engine import DistInfo, Engine

    use_gpu = _use_gpu(args)
    device = torch.device("cuda", local_device()) if use_gpu else torch.device("cpu")
    if not use_gpu and not spec.is_local and not os.environ.get("OMP_NUM_THREADS"):
        # CPU replicas of one job share the node: don't oversubscribe the cores
        torch.set_num_threads(max(1, (os.cpu_count() or 1) // (spec.num_workers + len(spec.ps))))
    if use_gpu:
        torch.cuda.set_device(local_device())
    world = 1 if spec.is_local else spec.num_workers
    rank = 0 if spec.is_local else spec.task_index
    if (args.sync_replicas and args.replicas_to_aggregate is not None and not spec.is_local
            and args.replicas_to_aggregate != world):
        raise SystemExit(f"--replicas_to_aggregate {args.replicas_to_aggregate} != {world} workers: the collective "
                         "path aggregates every worker's gradient; use --ps_mode async with PS tasks")
    store = None
    if not spec.is_local:
        if world > 1:
            os.environ.setdefault("KFA_CONV_OVERSUB", "2")  # see engine.init_distributed
        store = _store(spec, spec.is_chief)
        # GPU replicas: a control-only gloo group, gradients on the native RCCL layer
        # (parallel/comm.py: one RCCL communicator per process); KFA_COMM=torch: nccl
        from ..parallel.comm import init_default_group
        init_default_group(rank, world, device, _pg_timeout(args), store=store)
    torch.manual_seed(args.seed)  # identical init everywhere (+ broadcast in the engine)
    num_ps = 0 if spec.is_local else len(spec.ps)
    args.num_ps = num_ps
    model, data, loss_fn = build(args, device)
    model = model.to(device)
    engine = Engine(model, loss_fn, optimizer=args.optimizer, lr=args.learning_rate, momentum=args.momentum,
                    weight_decay=args.weight_decay, compute_dtype=torch.bfloat16 if (use_gpu and args.bf16) else None,
                    bucket_mb=args.bucket_mb, dist_info=DistInfo(rank, world, 0, device),
                    channels_last=model.__class__.__name__ == "ResNet", ps=num_ps, ps_placement=args.ps_placement,
                    grad_reduce_dtype=None if args.grad_reduce == "bf16" else torch.float32)
    model = engine.model
    resumed = engine.restore(args.model_dir) if args.model_dir else 0
    if resumed:
        _log(f"Worker {rank}: resumed from {args.model_dir} at global step {resumed}")
    if engine.sharded and spec.is_chief:
        placement = ps_assignment(list(model.named_parameters()), num_ps)
        counts = [sum(1 for v in placement.values() if v == p) for p in range(num_ps)]
        where = (f"variables of PS task p on worker rank {ps_owner_ranks(world, num_ps)}[p]"
                 if args.ps_placement == "ps" else f"shards owned by worker ranks 0..{world - 1}")
        _log(f"PS placement over {num_ps} PS tasks ({args.ps_placement}): tensors per PS = {counts}; {where}; "
             f"{len(engine.sync.buckets)} buckets; optimizer state {engine.optimizer_bytes() / 2**20:.1f} MiB "
             f"on this rank")

    inc = 1 if (args.sync_replicas or spec.is_local) else world
    steps_per_worker = max(0, math.ceil((args.train_steps - resumed) / inc))
    fixed = None if data is not None else synthetic_batch(args, model, device, rank)
    _log(f"Worker {rank}: {'local' if spec.is_local else f'{world} workers, {num_ps} ps'}, device {device}, "
         f"model {args.model}, {sum(p.numel() for p in model.parameters())} params, "
         f"{'push/pull to ' + args.ps_placement + ' owners (pull waits: ' + getattr(engine.sync, 'pull_mode', '?') + ')' if engine.sharded else 'all-reduce'}")
    t_begin = time.time()
    _log(f"Training begins @ {t_begin:f}")
    global_step = resumed
    t_first = None
    loss = None

    def _save():
        engine.save(args.model_dir, global_step, is_chief=False)
        if store is not None:
            dist.barrier()  # every rank's file is on disk before the manifest names the step
        if spec.is_chief:
            checkpoint.write_manifest(args.model_dir, global_step, world)

    # HIP graph replay of the whole step (Engine.capture) for single-replica GPU
    # jobs: the reference's MNIST steps are a few tiny kernels each, so launch
    # overhead is the step time; the batch is copied into the captured inputs.
    # "auto" captures only launch-bound steps: step 1 is timed (synchronized) and a
    # step of more than GRAPH_AUTO_MS keeps eager launches (ResNet-50 at batch 256:
    # 21.8 ms eager, replay measured 0.5 % slower; the reference's MNIST: 0.2 ms).
    use_graph = args.graph == "on" or (args.graph == "auto" and world == 1 and device.type == "cuda")
    cap_step = 1 if args.graph == "on" else 2
    if data is not None and device.type == "cuda" and hasattr(data, "to"):
        data.to(device)  # dataset resident in HBM: no host copy per step
    # steady-state window: from the end of the warm-up steps (step 0 tunes the
    # per-shape kernels, the capture step records the graph), GPU drained first
    warm = min(cap_step + 1 if use_graph else 1, max(1, steps_per_worker - 1))
    for local_step in range(steps_per_worker):
        _arm_watchdog(args)
        _test_hang(spec, local_step)
        if data is not None:
            xb, yb = data.next_batch(args.batch_size)
            batch = (xb.to(device), yb.to(device))
        else:
            batch = fixed
        if use_graph and local_step == 1 and args.graph == "auto":
            torch.cuda.synchronize()
            t1 = time.time()
            loss = engine.train_step(*batch)
            torch.cuda.synchronize()
            use_graph = (time.time() - t1) * 1e3 < GRAPH_AUTO_MS
        elif use_graph and local_step == cap_step and engine.graph_ok() is None:
            loss = engine.capture(*(b.clone() for b in batch))  # its warm-up step trains on this batch
            _log(f"Worker {rank}: step captured as a HIP graph; replaying it from step {cap_step + 1} on")
        else:
            loss = engine.train_step(*batch)
        global_step += inc
        if store is not None and spec.is_chief:
            store.add(STEP_KEY, inc)
        if local_step == 0 and engine.sharded and spec.is_chief:  # decided by the first forward
            _log(f"Worker {rank}: pull waits after the first forward: {getattr(engine.sync, 'pull_mode', '?')}")
        if local_step + 1 == warm:
            if device.type == "cuda":
                torch.cuda.synchronize()
            t_first = time.time()
        if args.model_dir and args.checkpoint_every and (local_step + 1) % args.checkpoint_every == 0:
            _save()
        if args.log_every and (local_step % args.log_every == 0 or local_step == steps_per_worker - 1):
            if spec.is_local:
                _log(f"step: {local_step}")
            else:
                _log(f"{time.time():f}: Worker {rank}: training step {local_step + 1} done "
                     f"(global step: {global_step})")
    engine.wait()
    if device.type == "cuda":
        torch.cuda.synchronize()
    t_end = time.time()
    _log(f"Training ends @ {t_end:f}")
    _log(f"Training elapsed time: {t_end - t_begin:f} s")
    if t_first is not None and steps_per_worker > warm:
        sps = (steps_per_worker - warm) / max(t_end - t_first, 1e-9)
        _log(f"Steady-state: {sps:.1f} steps/s/worker, {sps * args.batch_size * world:.1f} examples/s (job)")
    if data is not None:
        with torch.no_grad():
            model.eval()
            vx, vy = data.validation
            z = model(vx.to(device)).float()
            ce = float(cross_entropy(z, vy.to(device))) * vx.shape[0]
            _log(f"After {global_step} training step(s), validation cross entropy = {ce:g}")
            tx, ty = data.test
            acc = float(accuracy(model(tx.to(device)).float(), ty.to(device)))
            _log(f"Test accuracy: {acc:.4f}")
    elif loss is not None:
        _log(f"Final loss: {float(loss):.5f}")
    if args.model_dir:
        _save()
    if store is not None:
        store.add(DONE_KEY, 1)
        dist.barrier()
        dist.destroy_process_group()
    return 0


def _flag(v) -> bool:
    """TF-style boolean flag value: ``--x``, ``--x=true``, ``--x false``."""
    if isinstance(v, bool):
        return v
    if str(v).lower() in ("1", "true", "yes", "t", "y"):
        return True
    if str(v).lower() in ("0", "false", "no", "f", "n"):
        return False
    raise argparse.ArgumentTypeError(f"expected a boolean, got {v!r}")


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    add_cluster_flags(ap)
    ap.add_argument("--model", default="mnist_mlp",
                    help="mnist_softmax | mnist_mlp | resnet50 | resnet_tiny | bert_base | bert_tiny | "
                         "wide_deep | wide_deep_tiny")
    ap.add_argument("--train_steps", type=int, default=200)
    ap.add_argument("--batch_size", type=int, default=100)
    ap.add_argument("--learning_rate", type=float, default=0.01)
    ap.add_argument("--optimizer", default="adam", choices=["adam", "sgd"])
    ap.add_argument("--momentum", type=float, default=0.0)
    ap.add_argument("--weight_decay", type=float, default=0.0)
    ap.add_argument("--hidden_units", type=int, default=100)
    ap.add_argument("--seq_len", type=int, default=128)
    ap.add_argument("--sync_replicas", action="store_true")
    ap.add_argument("--ps_mode", default="auto", choices=["auto", "async", "collective"],
                    help="async: PS tasks own variables + Adam (reference default); collective: RCCL "
                         "reduce-scatter/all-gather on the workers; auto: async for MNIST without "
                         "--sync_replicas, collective otherwise")
    ap.add_argument("--ps_transport", default="auto", choices=["auto", "host", "device"],
                    help="async PS payloads: device = variables in the co-located GPU's HBM, pulled / pushed by "
                         "HIP IPC device copies; host = CPU tensors over gloo; auto = device when the PS has a GPU")
    ap.add_argument("--replicas_to_aggregate", type=int, default=None,
                    help="with --sync_replicas: gradients averaged per update (default: number of workers); "
                         "N < workers runs the PS service loop, which drops stale gradients")
    ap.add_argument("--existing_servers", type=_flag, nargs="?", const=True, default=False,
                    help="accepted for compatibility (no in-process gRPC server exists here; the job's "
                         "rendezvous store plays that part)")
    ap.add_argument("--download_only", type=_flag, nargs="?", const=True, default=False,
                    help="prepare the data set and exit 0 (synthetic data: nothing to download)")
    ap.add_argument("--num_gpus", type=int, default=1, help="accepted (one GPU per replica)")
    ap.add_argument("--data_dir", default="", help="accepted (synthetic data; no network)")
    ap.add_argument("--model_dir", default=os.environ.get("KFA_MODEL_DIR", ""),
                    help="checkpoint / resume directory (TFJob spec.modelDir via $KFA_MODEL_DIR)")
    ap.add_argument("--checkpoint_every", type=int, default=0, help="local steps between checkpoints")
    ap.add_argument("--device", default="auto", choices=["auto", "cpu", "gpu"])
    ap.add_argument("--bf16", type=int, default=1)
    ap.add_argument("--bucket_mb", type=float, default=32.0)
    ap.add_argument("--ps_placement", default="ps", choices=["ps", "sharded"],
                    help="collective mode with PS tasks: ps = each gradient bucket owned by one PS task's "
                         "co-located rank (replica_device_setter round-robin); sharded = every worker owns 1/W")
    ap.add_argument("--embedding_owners", default="all", choices=["all", "ps"],
                    help="Wide&Deep table rows: interleaved over all workers, or only the PS-co-located ranks")
    ap.add_argument("--grad_reduce", default="fp32", choices=["fp32", "bf16"],
                    help="dtype of the cross-rank gradient sum")
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                    help="replay the training step as one HIP graph after step 1 (auto: single-replica GPU jobs)")
    ap.add_argument("--log_every", type=int, default=1)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--ps_connect_timeout", type=float, default=300.0)
    ap.add_argument("--dist_timeout", type=float, default=float(os.environ.get("KFA_DIST_INIT_TIMEOUT", "300")),
                    help="torch.distributed init / collective timeout (seconds)")
    ap.add_argument("--hang_timeout", type=float, default=float(os.environ.get("KFA_REPLICA_HANG_TIMEOUT", "900")),
                    help="seconds without progress (rendezvous, one training step) before the replica dumps "
                         "every thread's stack and exits 1 (0 = off)")
    ap.add_argument("--loss", default="mean", choices=["mean", "sum_clipped"],
                    help="MNIST loss: mean softmax cross-entropy (mnist_softmax.py) or the summed "
                         "cross-entropy of clipped probabilities (mnist_replica.py:168)")
    return ap


def main(argv: Optional[list] = None) -> int:
    args = build_parser().parse_args(argv)
    if args.download_only:  # mnist_replica.py:94-96: read the data set, then exit before any cluster work
        if args.model.startswith("mnist"):
            from ..models import mnist
            d = mnist.SyntheticMNIST(seed=args.seed)
            _log(f"data ready: synthetic MNIST, {len(d.train[0])} training examples (--download_only)")
        else:
            _log(f"data ready: synthetic {args.model} batches are generated in-process (--download_only)")
        return 0
    spec = parse_cluster(args)
    if not spec.is_local:
        _aggregate(spec, args)  # validates --replicas_to_aggregate before any connection is made
    _install_stack_dumps()
    if _async_mode(spec, args):
        if spec.is_ps:  # a PS serves for as long as the workers train: no step-level guard
            return run_ps_async(spec, args)
        _arm_watchdog(args)
        try:
            return run_worker_async(spec, args)
        finally:  # an in-process caller must not be left with a live exit=True timer
            _disarm_watchdog()
    elif spec.is_ps:
        return run_ps(spec, args)
    _arm_watchdog(args)
    try:
        return run_worker(spec, args)
    finally:
        _disarm_watchdog()


if __name__ == "__main__":
    sys.exit(main())
