"""Asynchronous parameter server — the reference's DEFAULT update mode
(``mnist_replica.py`` without ``--sync_replicas``: between-graph replication,
variables round-robin on PS tasks via ``replica_device_setter`` :137-141, every
worker's ``sess.run(train_step)`` pulls the variables, computes gradients
against that (possibly stale) copy and pushes them to the PS, which applies
Adam immediately :184,:256; the global step advances once per push) — and its
``--sync_replicas --replicas_to_aggregate N`` form (``SyncReplicasOptimizer``
:172-195) on the same service loop.

Transport (SURVEY §5.8 "Async PS = send/recv to the owner rank", H5): a
process group over workers AND PS tasks (ranks ``0..W-1`` workers, ``W..W+P-1``
PS tasks).  Each PS runs a single-threaded service loop that receives request
headers ``[op, step_tag]`` from ANY worker (``recv(src=None)``), so workers
progress independently — no collective, no lock-step:

* ``PULL``  → PS sends its shard (all owned tensors, flattened fp32);
* ``PUSH``  → PS receives the gradient for its shard and applies Adam/SGD to it
  in place (owner-side apply: optimizer state lives only on the PS); the reply
  is ``[global_step, applied]`` (PS 0's counter is the job's global step);
* ``PUSH_DEV`` → the same with the gradient already in the worker's device
  mailbox (device transport, below); ``PUSH_SIG``: the mailbox copies are still
  in flight and the PS's stream waits on the worker's event before reading it;
* ``DONE``  → a worker finished; the PS exits when every worker has.

Aggregation (``aggregate = N``, the ``SyncReplicasOptimizer`` semantics): a
push tagged with a step older than the PS's current step is DROPPED (stale;
reply ``applied = 0`` at once); fresh pushes are summed, and the N-th one
applies their MEAN, advances the step and releases every waiting pusher (the
token queue).  When every still-active worker is waiting (fewer than N left,
e.g. at the end of training) the partial sum is applied so no one blocks
forever.  ``aggregate = 0``: every push applies at once (async).

Headers and payloads use distinct tags, and every request from one worker is
sequential, so a PS never interleaves two workers' payloads.  The request channel
(``parallel/comm.py:P2P``) is the first-party host transport by default —
``csrc/comm`` TCP streams per rank pair with an any-source receive for the PS
loop (``kfc_recv_any``), where the per-pair message order stands in for the tags
— or gloo (``KFA_PS_P2P=torch``).  Two payload transports:

* **host** (:class:`AsyncPSServer` / :class:`AsyncPSClient`): payloads are CPU
  tensors on the request channel — TF's gRPC PS in spirit, for CPU replicas;
* **device** (:class:`DeviceAsyncPSServer` / :class:`DeviceAsyncPSClient`): the
  PS task keeps its variables, Adam slots and one gradient mailbox per worker
  in the HBM of the GPU it is co-located with and exports them by HIP IPC
  (dmabuf handles published in the job's TCPStore as JSON — nothing is
  unpickled).  The worker holds its weights and gradients in per-PS flat
  buffers laid out exactly like the PS's, so a pull is ONE device copy (+cast)
  per PS and dtype run straight out of the PS's fp32 variables and a push is
  one copy into the mailbox followed by a ``PUSH_DEV`` header.  Before using a
  PS's memory the client verifies the mapping against a canary pattern the PS
  published (value + nonce); if the import fails or reads wrong data (e.g. the
  PS's GPU is not visible to this replica) that PS is served over the host
  transport instead, with a loud log line — the server speaks both.

  Hand-offs ordered ON THE DEVICES instead of by host waits
  (``KFA_PS_DEVICE_SIGNAL=1``, opt-in; the PS publishes its choice): each
  worker records an interprocess HIP event (``hipIpcGetEventHandle``) after its
  mailbox copies and the PS's stream waits on it before reading the mailbox;
  the PS records its own interprocess event after every update and replies at
  once, and the worker's stream waits on that event before its next pull (so it
  reads the update) and before it rewrites the mailbox (so the update has read
  it).  A PS that cannot see the worker's GPU (an isolated PS replica) cannot
  wait on the worker's event: that worker host-waits its copies and sends
  ``PUSH_DEV`` instead (every PS publishes the GPUs it sees).  The request /
  reply headers stay on the host channel; the steady-state push / pull path has
  no host synchronisation (``tests/test_async_ps_cpu_src.py`` checks the
  sources).  Measured SLOWER, so not the default: BERT-base 2 workers + 1 PS on
  one MI355X (``tools/async_rehearsal.py``) 3,377-3,643 ex/s with device
  signalling vs 5,188-5,320 with host waits.  The host time it spends is
  negligible (43 stream waits 1.3 ms, 3 event imports 0.17 s per run); the loss
  is head-of-line blocking on the PS's one stream (an update queued behind
  another worker's still-running mailbox copy) and workers' waits covering other
  workers' updates — a host-waited header only reaches the PS once its data is
  there.  ROCm's interprocess events also stop working after 31 records
  (``tools/probe_ipc_event4.py``), hence the event chains below.
  Default (``KFA_PS_DEVICE_SIGNAL`` unset / 0): host waits on recorded events
  (the round-4 protocol).

The synchronous collective modes (``--sync_replicas`` with N = W, or no PS) use
RCCL reduce / reduce-scatter / all-gather on the GPUs instead
(``parallel/ps.py``, ``parallel/ddp.py``).
"""
from __future__ import annotations

import base64
import json
import math
import os
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .comm import make_p2p
from .ps import ps_assignment

PULL, PUSH, DONE, PUSH_DEV, PUSH_SIG = 1, 2, 3, 4, 5
TAG_HDR, TAG_DATA, TAG_REPLY = 11, 12, 13
ALIGN = 8  # = parallel/flat.py ALIGN: device-layout offsets match the worker's FlatGroups


def _layout(shapes: Sequence[Tuple[str, torch.Size]], assignment: Dict[str, int], ps: int):
    """names owned by PS ``ps`` in declaration order, and the flat size."""
    names = [n for n, _ in shapes if assignment[n] == ps]
    sizes = {n: int(torch.Size(s).numel()) for n, s in shapes}
    return names, sum(sizes[n] for n in names)


def _round_up(n: int, m: int) -> int:
    return (n + m - 1) // m * m


def device_layout(shapes: Sequence[Tuple[str, torch.Size]], assignment: Dict[str, int], ps: int):
    """Layout of PS ``ps``'s variables in the device transport: the matrices
    (dim >= 2, bf16 on the worker) first, then the vectors, each run laid out as
    ``parallel.flat.FlatGroup`` lays it (offsets rounded up to ``ALIGN``, run
    length padded to ``ALIGN``).  Returns ``[(names, offsets, run_start,
    run_len)]`` for the two runs (empty runs omitted) and the total length."""
    names, _ = _layout(shapes, assignment, ps)
    dims = {n: len(s) for n, s in shapes}
    sizes = {n: int(torch.Size(s).numel()) for n, s in shapes}
    runs, start = [], 0
    for sel in ([n for n in names if dims[n] >= 2], [n for n in names if dims[n] < 2]):
        if not sel:
            continue
        offs, off = [], 0
        for n in sel:
            offs.append(off)
            off = _round_up(off + sizes[n], ALIGN)
        length = _round_up(max(off, 1), ALIGN)
        runs.append((sel, offs, start, length))
        start += length
    return runs, start


def _flat_order(t: torch.Tensor, channels_last: bool) -> torch.Tensor:
    """``t`` flattened in the worker's memory order (NHWC for channels-last convs)."""
    if channels_last and t.dim() == 4:
        return t.permute(0, 2, 3, 1).reshape(-1)
    return t.reshape(-1)


class _Service:
    """The PS service loop shared by both transports (see module docstring)."""

    W: int
    idx: int
    aggregate: int

    def _init_service(self, aggregate: int) -> None:
        if aggregate < 0 or aggregate > self.W:
            raise ValueError(f"replicas_to_aggregate must be in 1..{self.W} (num workers), got {aggregate}")
        self.aggregate = aggregate
        self.global_step = 0
        self.t = 0
        self.dropped = 0
        self.applied_pushes = 0
        self.update_sizes: List[int] = []  # gradients averaged into each aggregated update

    # transport hooks
    def _send_vars(self, src: int) -> None: ...
    def _recv_grad(self, src: int, op: int, seq: int = 0) -> torch.Tensor: ...
    def _apply(self, g: torch.Tensor, scale: float) -> None: ...
    def _acc_reset(self) -> None: ...
    def _acc_add(self, g: torch.Tensor) -> None: ...
    def _acc(self) -> torch.Tensor: ...
    def _reply(self, dst: int, applied: int) -> None:
        # [global step, applied, this PS's update-event sequence number (0: no device signalling)]
        self.p2p.send(torch.tensor([self.global_step, applied, getattr(self, "ps_seq", 0)], dtype=torch.int64), dst,
                      tag=TAG_REPLY)

    def close(self) -> None:
        """Release the request channel (after :meth:`serve`)."""
        self.p2p.destroy()

    def serve(self, log: Optional[Callable[[str], None]] = None) -> int:
        """Run until every worker sent DONE; returns the number of pushes applied."""
        active = self.W
        hdr = torch.zeros(3, dtype=torch.int64)  # [op, step tag, the pusher's mailbox-event sequence number]
        waiting: List[int] = []
        count = 0
        if self.aggregate:
            self._acc_reset()

        def flush():
            nonlocal count
            self._apply(self._acc(), 1.0 / count)
            self.update_sizes.append(count)
            self.global_step += 1
            for w in waiting:
                self._reply(w, 1)
            waiting.clear()
            count = 0
            self._acc_reset()

        while active > 0:
            src = self.p2p.recv_any(hdr, tag=TAG_HDR)
            op, tag, seq = int(hdr[0]), int(hdr[1]), int(hdr[2])
            if op == PULL:
                self._send_vars(src)
            elif op in (PUSH, PUSH_DEV, PUSH_SIG):
                g = self._recv_grad(src, op, seq)
                if not self.aggregate:
                    self._apply(g, 1.0)
                    self.applied_pushes += 1
                    self.global_step += 1
                    self._reply(src, 1)
                elif tag < self.global_step:  # computed on variables older than the current step
                    self.dropped += 1
                    self._reply(src, 0)
                else:
                    self._acc_add(g)
                    self.applied_pushes += 1
                    count += 1
                    waiting.append(src)
                    if count >= self.aggregate:
                        flush()
                if log and self.global_step and self.global_step % 50 == 0 and not waiting:
                    log(f"PS {self.idx}: applied {self.global_step} updates")
            elif op == DONE:
                active -= 1
            else:
                raise RuntimeError(f"PS {self.idx}: bad request {op} from rank {src}")
            if self.aggregate and waiting and len(waiting) >= active:
                flush()  # nobody left who could complete the aggregate
        return self.applied_pushes


class AsyncPSServer(_Service):
    """Service loop of PS task ``ps_index`` (rank ``num_workers + ps_index``), host memory."""

    def __init__(self, init_params: Sequence[Tuple[str, torch.Tensor]], num_workers: int, num_ps: int, ps_index: int,
                 lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, optimizer: str = "adam", group=None,
                 aggregate: int = 0, p2p=None):
        self.W, self.P, self.idx = num_workers, num_ps, ps_index
        shapes = [(n, p.shape) for n, p in init_params]
        self.assignment = ps_assignment(list(init_params), num_ps)
        self.names, n = _layout(shapes, self.assignment, ps_index)
        src = dict(init_params)
        self.w = torch.cat([src[k].detach().float().reshape(-1).cpu() for k in self.names]) if self.names \
            else torch.zeros(0)
        self.m = torch.zeros_like(self.w)
        self.v = torch.zeros_like(self.w)
        self.grad = torch.empty_like(self.w)
        self.lr, self.betas, self.eps, self.opt = lr, betas, eps, optimizer
        self.group = group
        self._init_service(aggregate)
        self.p2p = p2p if p2p is not None else make_p2p(group=group)

    def _apply(self, g: torch.Tensor, scale: float = 1.0) -> None:
        self.t += 1
        if scale != 1.0:
            g = g * scale
        if self.opt == "sgd":
            self.w.add_(g, alpha=-self.lr)
            return
        b1, b2 = self.betas
        self.m.mul_(b1).add_(g, alpha=1 - b1)
        self.v.mul_(b2).addcmul_(g, g, value=1 - b2)
        step = self.lr * math.sqrt(1 - b2 ** self.t) / (1 - b1 ** self.t)  # TF AdamOptimizer form
        self.w.addcdiv_(self.m, self.v.sqrt().add_(self.eps), value=-step)

    def _send_vars(self, src: int) -> None:
        self.p2p.send(self.w, src, tag=TAG_DATA)

    def _recv_grad(self, src: int, op: int, seq: int = 0) -> torch.Tensor:
        if op != PUSH:
            raise RuntimeError(f"PS {self.idx}: host server got a device push from rank {src}")
        self.p2p.recv(self.grad, src, tag=TAG_DATA)
        return self.grad

    def _acc_reset(self) -> None:
        self.acc = torch.zeros_like(self.w)

    def _acc_add(self, g: torch.Tensor) -> None:
        self.acc.add_(g)

    def _acc(self) -> torch.Tensor:
        return self.acc


class _ClientSteps:
    """Per-PS step tags: the PS's step as last reported to this worker."""

    def _init_steps(self, num_ps: int) -> None:
        self.tags = [0] * num_ps
        self.pushes_dropped = 0
        self._hdr = torch.zeros(3, dtype=torch.int64)
        self._reply = torch.zeros(3, dtype=torch.int64)
        self.ps_seq = [0] * num_ps  # each PS's update-event sequence number as last replied

    def close(self) -> None:
        """Release the request channel (after :meth:`done`)."""
        self.p2p.destroy()

    def _header(self, rank: int, op: int, tag: int = 0, seq: int = 0) -> None:
        self._hdr[0], self._hdr[1], self._hdr[2] = op, tag, seq
        self.p2p.send(self._hdr, rank, tag=TAG_HDR)

    def _await_reply(self, k: int, rank: int) -> int:
        self.p2p.recv(self._reply, rank, tag=TAG_REPLY)
        step, applied = int(self._reply[0]), int(self._reply[1])
        self.tags[k] = step
        self.ps_seq[k] = int(self._reply[2])
        if not applied:
            self.pushes_dropped += 1
        return step


class AsyncPSClient(_ClientSteps):
    """Worker side: pull variables from / push gradients to every PS task (host transport)."""

    def __init__(self, params: Sequence[Tuple[str, torch.nn.Parameter]], num_workers: int, num_ps: int, group=None,
                 p2p=None):
        self.W, self.P, self.group = num_workers, num_ps, group
        self.params = list(params)
        self.assignment = ps_assignment(self.params, num_ps)
        shapes = [(n, p.shape) for n, p in self.params]
        by_name = dict(self.params)
        self.plan: List[Tuple[int, List[torch.nn.Parameter], torch.Tensor]] = []
        for k in range(num_ps):
            names, n = _layout(shapes, self.assignment, k)
            self.plan.append((num_workers + k, [by_name[x] for x in names], torch.zeros(n)))
        self._init_steps(num_ps)
        self.p2p = p2p if p2p is not None else make_p2p(group=group)

    def pull(self) -> None:
        for rank, ps, buf in self.plan:
            if not ps:
                continue
            self._header(rank, PULL)
            self.p2p.recv(buf, rank, tag=TAG_DATA)
            off = 0
            with torch.no_grad():
                for p in ps:
                    n = p.numel()
                    p.copy_(buf[off:off + n].view_as(p))
                    off += n

    def push(self) -> int:
        """Send every PS its gradient shard (all shards first, then the replies, so the
        PS tasks apply concurrently); returns the global step reported by PS 0."""
        live = []
        for k, (rank, ps, buf) in enumerate(self.plan):
            if not ps:
                continue
            off = 0
            for p in ps:
                n = p.numel()
                if p.grad is None:
                    buf[off:off + n].zero_()
                else:
                    buf[off:off + n].copy_(p.grad.reshape(-1))
                off += n
            self._header(rank, PUSH, self.tags[k])
            self.p2p.send(buf, rank, tag=TAG_DATA)
            live.append((k, rank))
        step = -1
        for k, rank in live:
            s = self._await_reply(k, rank)
            if k == 0:
                step = s
        return step

    def done(self) -> None:
        for rank, _, _ in self.plan:
            self._header(rank, DONE)


# ---------------------------------------------------------------------------
# device-resident transport (HIP IPC)
def _ipc_key(ps: int, what: str) -> str:
    return f"kfa/async_ps/{ps}/{what}"


_TENSOR_CLS = {"Tensor": torch.Tensor, "Parameter": torch.nn.Parameter}
_STORAGE_CLS = {"UntypedStorage": torch.UntypedStorage, "TypedStorage": torch.storage.TypedStorage}


def _enc(v):
    if isinstance(v, (bytes, bytearray)):
        return {"b64": base64.b64encode(bytes(v)).decode()}
    if isinstance(v, torch.Size):
        return list(v)
    if isinstance(v, tuple):
        return list(v)
    return v


def _dec(v):
    if isinstance(v, dict) and set(v) == {"b64"}:
        return base64.b64decode(v["b64"])
    return v


def _export(store, key: str, t: torch.Tensor) -> None:
    """Publish a CUDA tensor to the other processes of the job (HIP IPC handle)
    as JSON: plain ints / strings and base64 handle bytes, no pickled objects."""
    from torch.multiprocessing.reductions import reduce_tensor
    _, a = reduce_tensor(t)
    (tensor_cls, size, stride, offset, storage_cls, dtype, device, handle, size_bytes, offset_bytes, req_grad,
     ref_handle, ref_offset, ev_handle, ev_sync) = a
    rec = {"tensor_cls": tensor_cls.__name__, "size": list(size), "stride": list(stride), "offset": int(offset),
           "storage_cls": storage_cls.__name__, "dtype": str(dtype).replace("torch.", ""), "device": int(device),
           "handle": _enc(handle), "size_bytes": int(size_bytes), "offset_bytes": int(offset_bytes),
           "requires_grad": bool(req_grad), "ref_handle": _enc(ref_handle), "ref_offset": int(ref_offset),
           "event_handle": _enc(ev_handle), "event_sync": bool(ev_sync)}
    store.set(key, json.dumps(rec))


def _export_event(store, key: str, ev: "torch.cuda.Event") -> None:
    """Publish an interprocess HIP event (recorded at least once) as base64 text."""
    store.set(key, base64.b64encode(bytes(ev.ipc_handle())).decode())


def _import_event(store, key: str, device: int) -> "torch.cuda.Event":
    """Open an event another process published with :func:`_export_event`;
    ``device``: this process's ordinal of the exporter's GPU."""
    return torch.cuda.Event.from_ipc_handle(torch.device("cuda", device), base64.b64decode(store.get(key)))


class _EventChain:
    """The producer side of a cross-process "done up to here" signal: an
    interprocess HIP event per generation of ``G`` records, re-created and
    published under ``key/<generation>`` when a generation is full.  ROCm's
    interprocess event stops working after 31 records (every later
    ``hipStreamWaitEvent`` on it fails with invalid argument, whatever the pacing:
    ``tools/probe_ipc_event4.py``), so no event is recorded more than G = 16 times.
    ``record`` returns the record's sequence number (1, 2, ...); the last
    ``KEEP`` generations stay alive for consumers that open them late."""
    G, KEEP = 16, 8

    def __init__(self, store, key: str):
        self.store, self.key, self.n = store, key, 0
        self.gens: List[torch.cuda.Event] = []

    def record(self, stream) -> int:
        if self.n % self.G == 0:
            ev = torch.cuda.Event(interprocess=True)
            ev.record(stream)
            _export_event(self.store, f"{self.key}/{self.n // self.G}", ev)
            self.gens = (self.gens + [ev])[-self.KEEP:]
        else:
            self.gens[-1].record(stream)
        self.n += 1
        return self.n


class _EventWaiter:
    """The consumer side: order a stream after record ``seq`` of another process's
    :class:`_EventChain` (a wait on that record's generation event waits for its
    latest record, which is ``seq`` or a later one)."""

    def __init__(self, store, key: str, device: int):
        self.store, self.key, self.device = store, key, device
        self.cache: Dict[int, torch.cuda.Event] = {}

    STATS = {"imports": 0, "import_s": 0.0, "waits": 0, "wait_s": 0.0}  # host time (KFA_PS_SIGNAL_STATS=1)

    def wait(self, stream, seq: int) -> None:
        if seq <= 0:
            return
        import time
        t0 = time.perf_counter()
        gen = (seq - 1) // _EventChain.G
        ev = self.cache.get(gen)
        if ev is None:
            ev = _import_event(self.store, f"{self.key}/{gen}", self.device)
            self.cache = {g: e for g, e in self.cache.items() if g >= gen - 1}
            self.cache[gen] = ev
            self.STATS["imports"] += 1
            self.STATS["import_s"] += time.perf_counter() - t0
        t1 = time.perf_counter()
        stream.wait_event(ev)
        self.STATS["waits"] += 1
        self.STATS["wait_s"] += time.perf_counter() - t1


def _worker_key(rank: int, what: str) -> str:
    return f"kfa/async_ps/worker/{rank}/{what}"


def device_signal_enabled() -> bool:
    return os.environ.get("KFA_PS_DEVICE_SIGNAL", "0") == "1"


def _host_wait(ev: "torch.cuda.Event", stream) -> None:
    """The KFA_PS_DEVICE_SIGNAL=0 protocol: record on ``stream`` and block the host."""
    ev.record(stream)
    ev.synchronize()


def _import(store, key: str, device: Optional[int] = None) -> torch.Tensor:
    """Map a tensor another process of this job exported with :func:`_export`.
    ``device``: this process's ordinal of the exporter's GPU (the record holds the
    EXPORTER's ordinal, which differs whenever the two see different GPU lists)."""
    from torch.multiprocessing.reductions import rebuild_cuda_tensor
    r = json.loads(store.get(key).decode())
    if device is not None:
        r["device"] = int(device)
    dtype = getattr(torch, r["dtype"])
    if not isinstance(dtype, torch.dtype):
        raise ValueError(f"bad dtype {r['dtype']!r} in {key}")
    return rebuild_cuda_tensor(_TENSOR_CLS[r["tensor_cls"]], torch.Size(r["size"]), tuple(r["stride"]),
                               int(r["offset"]), _STORAGE_CLS[r["storage_cls"]], dtype, int(r["device"]),
                               _dec(r["handle"]), int(r["size_bytes"]), int(r["offset_bytes"]),
                               bool(r["requires_grad"]), _dec(r["ref_handle"]), int(r["ref_offset"]),
                               _dec(r["event_handle"]), bool(r["event_sync"]))


CANARY_N = 64


def physical_gpu() -> str:
    """Physical index of this process's own GPU (entry ``local_device()`` of the
    supervisor's ``KFA_GPUS`` / ``HIP_VISIBLE_DEVICES`` list: the first one when the
    replica is isolated, its ``KFA_LOCAL_DEVICE`` ordinal when every GPU is
    visible); "" when not pinned."""
    from ..trainer.cluster import local_device
    vis = [v.strip() for v in (os.environ.get("KFA_GPUS") or os.environ.get("HIP_VISIBLE_DEVICES") or "").split(",")]
    i = local_device()
    return vis[i] if i < len(vis) else ""


def local_ordinal(phys: str) -> Tuple[Optional[int], str]:
    """This process's device ordinal of physical GPU ``phys`` (None + the reason
    when it is not visible here).  ``phys == ""`` (exporter not pinned): ordinal 0."""
    if phys == "":
        return 0, "exporter GPU unknown: assuming this process's cuda:0"
    vis = os.environ.get("KFA_GPUS") or os.environ.get("HIP_VISIBLE_DEVICES")
    if vis is None or not vis.strip():
        return int(phys), f"all GPUs visible: cuda:{phys}"
    lst = [v.strip() for v in vis.split(",") if v.strip()]
    if phys in lst:
        return lst.index(phys), f"GPU {phys} = cuda:{lst.index(phys)} (visible {','.join(lst)})"
    return None, f"its GPU {phys} is not visible to this worker (HIP_VISIBLE_DEVICES={vis})"


def _canary_values(nonce: int) -> torch.Tensor:
    return torch.arange(CANARY_N, dtype=torch.float32) * 0.5 + float(nonce % 1000003)


class DeviceAsyncPSServer(_Service):
    """PS task ``ps_index`` with its variables in GPU memory (see module docstring)."""

    def __init__(self, init_params: Sequence[Tuple[str, torch.Tensor]], num_workers: int, num_ps: int, ps_index: int,
                 store, device, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, optimizer: str = "adam",
                 group=None, aggregate: int = 0, channels_last: bool = False, p2p=None):
        self.W, self.P, self.idx = num_workers, num_ps, ps_index
        shapes = [(n, p.shape) for n, p in init_params]
        self.assignment = ps_assignment(list(init_params), num_ps)
        self.runs, n = device_layout(shapes, self.assignment, ps_index)
        self._shapes = shapes
        self.names = [x for run in self.runs for x in run[0]]
        src = dict(init_params)
        self.device = device
        npad = max(_round_up(n, ALIGN), ALIGN)  # the fused Adam kernel moves 8 values per thread
        self.w = torch.zeros(npad, dtype=torch.float32, device=device)
        for names, offs, start, _ in self.runs:
            for name, o in zip(names, offs):
                t = _flat_order(src[name].detach().float(), channels_last)
                self.w[start + o:start + o + t.numel()].copy_(t)
        self.m = torch.zeros_like(self.w)
        self.v = torch.zeros_like(self.w)
        self.mail = torch.zeros(num_workers, npad, dtype=torch.float32, device=device)
        self.stage = torch.empty(npad, dtype=torch.float32)  # host-transport payloads
        self.lr, self.betas, self.eps, self.opt = lr, betas, eps, optimizer
        self.group = group
        self._init_service(aggregate)
        nonce = int.from_bytes(os.urandom(4), "little")
        self.canary = _canary_values(nonce).to(device)
        torch.cuda.synchronize(device)
        _export(store, _ipc_key(ps_index, "w"), self.w)
        _export(store, _ipc_key(ps_index, "mail"), self.mail)
        _export(store, _ipc_key(ps_index, "canary"), self.canary)
        store.set(_ipc_key(ps_index, "nonce"), str(nonce))
        store.set(_ipc_key(ps_index, "gpu"), physical_gpu())
        self._done = torch.cuda.Event()
        # device-side hand-offs (module doc): this PS's "update recorded" event, and the
        # workers' "mailbox written" events, opened at their first device push
        self.signal = device_signal_enabled()
        self._store = store
        self._wev: Dict[int, _EventWaiter] = {}
        self.ps_seq = 0
        self._done_chain = _EventChain(store, _ipc_key(ps_index, "done")) if self.signal else None
        store.set(_ipc_key(ps_index, "signal"), "1" if self.signal else "0")
        store.set(_ipc_key(ps_index, "visible"),
                  os.environ.get("KFA_GPUS") or os.environ.get("HIP_VISIBLE_DEVICES") or "")
        store.set(_ipc_key(ps_index, "ready"), "1")
        # after the buffers are published: the workers join the channel once they mapped them
        self.p2p = p2p if p2p is not None else make_p2p(store, group=group)

    def _apply(self, g: torch.Tensor, scale: float = 1.0) -> None:
        from ..ops import _lib, optim  # noqa: F401  (optim registers kfa_adam_step)
        self.t += 1
        n = self.w.numel()
        if self.opt == "sgd":
            self.w.add_(g, alpha=-self.lr * scale)
        else:
            b1, b2 = self.betas
            bc1, bc2 = 1.0 - b1 ** self.t, 1.0 - b2 ** self.t
            # TF AdamOptimizer form (eps outside the bias-corrected sqrt) with the fused HIP kernel
            _lib.call("kfa_adam_step", _lib.ptr(self.w), None, _lib.ptr(g), 0, _lib.ptr(self.m), _lib.ptr(self.v), n,
                      self.lr, b1, b2, self.eps / math.sqrt(bc2), 0.0, bc1, bc2, scale, None, _lib.stream())
        self._after_update()

    def _after_update(self) -> None:
        """The reply that follows tells the pusher its mailbox may be rewritten and its
        next pull sees this update: with device signalling the PS records its event
        (the worker's stream waits on it) and replies at once; else a host wait on
        THIS update's completion event (not the stream)."""
        stream = torch.cuda.current_stream(self.device)
        if self.signal:
            self.ps_seq = self._done_chain.record(stream)  # replied to the pusher(s): they wait on it
        else:
            _host_wait(self._done, stream)

    def _send_vars(self, src: int) -> None:  # a host-transport client (IPC mapping failed on its side)
        self.stage.copy_(self.w)
        self.p2p.send(self.stage, src, tag=TAG_DATA)

    def _recv_grad(self, src: int, op: int, seq: int = 0) -> torch.Tensor:
        if op == PUSH_SIG:  # the mailbox copies (record `seq` of the pusher's chain) are ordered first
            w = self._wev.get(src)
            if w is None:
                dev, why = local_ordinal(self._store.get(_worker_key(src, "gpu")).decode())
                if dev is None:
                    raise RuntimeError(f"PS {self.idx}: PUSH_SIG from rank {src}, whose GPU I cannot see ({why})")
                w = self._wev[src] = _EventWaiter(self._store, _worker_key(src, "copied"), dev)
            w.wait(torch.cuda.current_stream(self.device), seq)
            return self.mail[src]
        if op == PUSH_DEV:
            return self.mail[src]
        self.p2p.recv(self.stage, src, tag=TAG_DATA)
        self.mail[src].copy_(self.stage, non_blocking=False)
        return self.mail[src]

    def variables(self) -> Dict[str, torch.Tensor]:
        """name -> view of this PS's fp32 variable (worker memory order, flattened)."""
        out = {}
        shapes = dict(self._shapes)
        for names, offs, start, _ in self.runs:
            for name, o in zip(names, offs):
                n = int(torch.Size(shapes[name]).numel())
                out[name] = self.w[start + o:start + o + n]
        return out

    def _acc_reset(self) -> None:
        if not hasattr(self, "acc"):
            self.acc = torch.zeros_like(self.w)
        else:
            self.acc.zero_()

    def _acc_add(self, g: torch.Tensor) -> None:
        self.acc.add_(g)
        # the pusher may reuse its mailbox once replied to: the add that read it is ordered first
        self._after_update()

    def _acc(self) -> torch.Tensor:
        return self.acc


class DeviceAsyncPSClient(_ClientSteps):
    """Worker side of the device transport.

    The worker's parameters are re-homed into per-PS flat buffers
    (``parallel.flat.FlatGroup``: one for the bf16 matrices, one for the fp32
    vectors, laid out like :func:`device_layout`), their gradients too, so each
    pull / push is one device copy per PS and run.  Each PS's mapping is
    checked against its canary first; a PS whose memory cannot be mapped is
    served over the host transport (``transports[k] == "host"``)."""

    def __init__(self, params: Sequence[Tuple[str, torch.nn.Parameter]], num_workers: int, num_ps: int, rank: int,
                 store, group=None, timeout: float = 300.0, log: Optional[Callable[[str], None]] = None,
                 p2p=None):
        import time

        from .flat import FlatGroup
        self.W, self.P, self.rank, self.group = num_workers, num_ps, rank, group
        self.params = list(params)
        self.assignment = ps_assignment(self.params, num_ps)
        shapes = [(n, p.shape) for n, p in self.params]
        by_name = dict(self.params)
        self.plan = []
        self.applied: List[Optional[_EventWaiter]] = []  # per PS: waits on its "update recorded" chain
        self.sig: List[bool] = []  # per PS: it waits on this worker's "mailbox written" event (PUSH_SIG)
        self.transports: List[str] = []
        self.transport_desc: List[str] = []
        log = log or (lambda s: print(s, flush=True))
        t0 = time.time()
        for k in range(num_ps):
            runs, total = device_layout(shapes, self.assignment, k)
            groups = []
            for names, _, start, length in runs:
                g = FlatGroup([by_name[x] for x in names], pad_to=ALIGN, master=False, name=f"ps{k}")
                assert g.numel == length, (g.numel, length)
                groups.append((g, start))
            while True:  # the PS publishes its buffers once its variables are on the GPU
                try:
                    if store.check([_ipc_key(k, "ready")]):
                        break
                except Exception:
                    pass
                if time.time() - t0 > timeout:
                    raise TimeoutError(f"PS {k} did not publish its device buffers")
                time.sleep(0.05)
            w = mail = None
            try:
                phys = store.get(_ipc_key(k, "gpu")).decode() if store.check([_ipc_key(k, "gpu")]) else ""
                dev, where = local_ordinal(phys)
                if dev is None:
                    raise RuntimeError(where)
                nonce = int(store.get(_ipc_key(k, "nonce")).decode())
                canary = _import(store, _ipc_key(k, "canary"), dev)
                got = canary.cpu()
                if not torch.equal(got, _canary_values(nonce)):
                    raise RuntimeError(f"canary mismatch (read {got[:4].tolist()}...)")
                w = _import(store, _ipc_key(k, "w"), dev)
                mail = _import(store, _ipc_key(k, "mail"), dev)[rank]
                if w.numel() < total:
                    raise RuntimeError(f"PS buffer has {w.numel()} values, layout needs {total}")
                self.transports.append("device")
                self.transport_desc.append(f"PS {k}: device ({where})")
            except Exception as e:  # noqa: BLE001 — any mapping failure: fall back, loudly
                log(f"Worker {rank}: WARNING: HIP IPC mapping of PS {k}'s device buffers failed ({e}); "
                    f"using the HOST transport for PS {k} (payloads over the request channel, slower)")
                self.transports.append("host")
                self.transport_desc.append(f"PS {k}: host ({e})")
                w = mail = None
            stage = torch.empty(max(_round_up(total, ALIGN), ALIGN), dtype=torch.float32) \
                if self.transports[-1] == "host" else None
            applied, sig = None, False
            if w is not None and store.get(_ipc_key(k, "signal")).decode() == "1":
                applied = _EventWaiter(store, _ipc_key(k, "done"), dev)  # the PS's "update recorded" chain
                vis = [v.strip() for v in store.get(_ipc_key(k, "visible")).decode().split(",") if v.strip()]
                sig = not vis or physical_gpu() in vis  # the PS can open this worker's event
            self.applied.append(applied)
            self.sig.append(sig)
            self.plan.append((num_workers + k, groups, w, mail, stage))
        self._ev: Dict[torch.device, torch.cuda.Event] = {}
        self._copied = None
        if any(self.sig):  # this worker's "mailboxes written" chain, and its GPU (the PS opens the events there)
            self._copied = _EventChain(store, _worker_key(rank, "copied"))
            store.set(_worker_key(rank, "gpu"), physical_gpu())
        self._init_steps(num_ps)
        self.p2p = p2p if p2p is not None else make_p2p(store, group=group)

    def zero_grad(self) -> None:
        for _, groups, *_ in self.plan:
            for g, _ in groups:
                g.zero_grad()

    @torch.no_grad()
    def pull(self) -> None:
        cur = torch.cuda.current_stream() if torch.cuda.is_available() else None
        for k, (rank, groups, w, _, stage) in enumerate(self.plan):
            if not groups:
                continue
            if stage is not None:
                self._header(rank, PULL)
                self.p2p.recv(stage, rank, tag=TAG_DATA)
                src = stage
            else:
                src = w
                if self.applied[k] is not None:  # the PS's update last replied to this worker first
                    self.applied[k].wait(cur, self.ps_seq[k])
            for g, start in groups:
                g.data.copy_(src[start:start + g.numel])  # D2D (peer) copy + cast, or H2D

    @torch.no_grad()
    def push(self) -> int:
        """Every PS shard at once: all mailbox copies (peer D2D writes over xGMI) are
        enqueued first and covered by ONE host wait per device, then every PS gets its
        header, then the replies are collected — the PS tasks apply their shards
        concurrently instead of one after another (round 4 did copy / wait / header /
        reply per PS in turn)."""
        live = [(k, rank, groups, mail, stage) for k, (rank, groups, _, mail, stage) in enumerate(self.plan) if groups]
        devs = set()
        for k, rank, groups, mail, stage in live:
            dst = stage if stage is not None else mail
            if stage is None and self.applied[k] is not None:
                # the PS's previous update (which read this mailbox) is ordered first
                self.applied[k].wait(torch.cuda.current_stream(), self.ps_seq[k])
            for g, start in groups:
                dst[start:start + g.numel].copy_(g.grad)
            if stage is None and not self.sig[k]:
                devs |= {mail.device, groups[0][0].grad.device}
        seq = 0
        if self._copied is not None:  # PUSH_SIG: the PS's stream waits on this record before it reads the mailbox
            seq = self._copied.record(torch.cuda.current_stream())
        # PUSH_DEV (signalling off, or the PS cannot see this GPU): the mailboxes are
        # written before any header (host waits)
        for d in devs:
            _host_wait(self._ev.setdefault(d, torch.cuda.Event()), torch.cuda.current_stream(d))
        for k, rank, groups, mail, stage in live:
            if stage is None:
                self._header(rank, PUSH_SIG if self.sig[k] else PUSH_DEV, self.tags[k], seq if self.sig[k] else 0)
            else:
                self._header(rank, PUSH, self.tags[k])
                self.p2p.send(stage, rank, tag=TAG_DATA)
        step = -1
        for k, rank, *_ in live:
            s = self._await_reply(k, rank)
            if k == 0:
                step = s
        return step

    def done(self) -> None:
        if os.environ.get("KFA_PS_SIGNAL_STATS") == "1":
            print(f"[async ps] worker {self.rank} device-signal host time: {_EventWaiter.STATS}", flush=True)
        for rank, *_ in self.plan:
            self._header(rank, DONE)
