"""Asynchronous parameter server — the reference's DEFAULT update mode
(``mnist_replica.py`` without ``--sync_replicas``: between-graph replication,
variables round-robin on PS tasks via ``replica_device_setter`` :137-141, every
worker's ``sess.run(train_step)`` pulls the variables, computes gradients
against that (possibly stale) copy and pushes them to the PS, which applies
Adam immediately :184,:256; the global step advances once per push).

Transport (SURVEY §5.8 "Async PS = send/recv to the owner rank", H5): a
process group over workers AND PS tasks (ranks ``0..W-1`` workers, ``W..W+P-1``
PS tasks).  Each PS runs a single-threaded service loop that receives request
headers from ANY worker (``recv(src=None)``), so workers progress
independently — no collective, no lock-step:

* ``PULL``  → PS sends its shard (all owned tensors, flattened fp32);
* ``PUSH``  → PS receives the gradient for its shard, applies Adam to it in
  place (owner-side apply, optimizer state lives only on the PS) and replies
  with the new global step (PS 0 owns the global step counter);
* ``DONE``  → a worker finished; the PS exits when every worker has.

Headers and payloads use distinct tags, and every request from one worker is
sequential, so a PS never interleaves two workers' payloads.  Two transports:

* **host** (:class:`AsyncPSServer` / :class:`AsyncPSClient`): payloads are CPU
  tensors over gloo — TF's gRPC PS in spirit, for CPU replicas;
* **device** (:class:`DeviceAsyncPSServer` / :class:`DeviceAsyncPSClient`): the
  PS task keeps its variables, Adam slots and one gradient mailbox per worker
  in GPU memory on the GPU it is co-located with, and exports them to the
  workers by HIP IPC (dmabuf handles published in the job's TCPStore).  A pull
  is a device-to-device copy straight out of the PS's fp32 variables (over
  xGMI when the PS sits on another GPU of the node; no PS involvement, and —
  like TF's ``use_locking=False`` Adam — it may overlap an update); a push is a
  device-to-device write into the worker's mailbox followed by a PUSH header;
  the PS applies the fused HIP Adam kernel to the mailbox and replies with the
  global step.  Only headers and step numbers cross the host.

The synchronous modes (``--sync_replicas``, or no PS) use RCCL reduce /
reduce-scatter / all-gather on the GPUs instead (``parallel/ps.py``,
``parallel/ddp.py``).
"""
from __future__ import annotations

import math
from typing import Dict, List, Sequence, Tuple

import torch
import torch.distributed as dist

from .ps import ps_assignment

PULL, PUSH, DONE = 1, 2, 3
TAG_HDR, TAG_DATA, TAG_REPLY = 11, 12, 13


def _layout(shapes: Sequence[Tuple[str, torch.Size]], assignment: Dict[str, int], ps: int):
    """names owned by PS ``ps`` in declaration order, and the flat size."""
    names = [n for n, _ in shapes if assignment[n] == ps]
    sizes = {n: int(torch.Size(s).numel()) for n, s in shapes}
    return names, sum(sizes[n] for n in names)


class AsyncPSServer:
    """Service loop of PS task ``ps_index`` (rank ``num_workers + ps_index``)."""

    def __init__(self, init_params: Sequence[Tuple[str, torch.Tensor]], num_workers: int, num_ps: int, ps_index: int,
                 lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, optimizer: str = "adam", group=None):
        self.W, self.P, self.idx = num_workers, num_ps, ps_index
        shapes = [(n, p.shape) for n, p in init_params]
        self.assignment = ps_assignment(list(init_params), num_ps)
        self.names, n = _layout(shapes, self.assignment, ps_index)
        src = dict(init_params)
        self.w = torch.cat([src[k].detach().float().reshape(-1).cpu() for k in self.names]) if self.names \
            else torch.zeros(0)
        self.m = torch.zeros_like(self.w)
        self.v = torch.zeros_like(self.w)
        self.lr, self.betas, self.eps, self.opt = lr, betas, eps, optimizer
        self.t = 0
        self.global_step = 0
        self.group = group

    def _apply(self, g: torch.Tensor) -> None:
        self.t += 1
        if self.opt == "sgd":
            self.w.add_(g, alpha=-self.lr)
            return
        b1, b2 = self.betas
        self.m.mul_(b1).add_(g, alpha=1 - b1)
        self.v.mul_(b2).addcmul_(g, g, value=1 - b2)
        step = self.lr * math.sqrt(1 - b2 ** self.t) / (1 - b1 ** self.t)  # TF AdamOptimizer form
        self.w.addcdiv_(self.m, self.v.sqrt().add_(self.eps), value=-step)

    def serve(self, log=None) -> int:
        """Run until every worker sent DONE; returns the number of pushes applied."""
        active = self.W
        hdr = torch.zeros(2, dtype=torch.int64)
        grad = torch.empty_like(self.w)
        pushes = 0
        while active > 0:
            src = dist.recv(hdr, src=None, group=self.group, tag=TAG_HDR)
            op = int(hdr[0])
            if op == PULL:
                dist.send(self.w, src, group=self.group, tag=TAG_DATA)
            elif op == PUSH:
                dist.recv(grad, src, group=self.group, tag=TAG_DATA)
                self._apply(grad)
                pushes += 1
                self.global_step += 1
                dist.send(torch.tensor([self.global_step], dtype=torch.int64), src, group=self.group,
                          tag=TAG_REPLY)
                if log and self.global_step % 50 == 0:
                    log(f"PS {self.idx}: applied {self.global_step} updates")
            elif op == DONE:
                active -= 1
            else:
                raise RuntimeError(f"PS {self.idx}: bad request {op} from rank {src}")
        return pushes


class AsyncPSClient:
    """Worker side: pull variables from / push gradients to every PS task."""

    def __init__(self, params: Sequence[Tuple[str, torch.nn.Parameter]], num_workers: int, num_ps: int, group=None):
        self.W, self.P, self.group = num_workers, num_ps, group
        self.params = list(params)
        self.assignment = ps_assignment(self.params, num_ps)
        shapes = [(n, p.shape) for n, p in self.params]
        by_name = dict(self.params)
        self.plan: List[Tuple[int, List[torch.nn.Parameter], torch.Tensor]] = []
        for k in range(num_ps):
            names, n = _layout(shapes, self.assignment, k)
            self.plan.append((num_workers + k, [by_name[x] for x in names], torch.zeros(n)))
        self._hdr = torch.zeros(2, dtype=torch.int64)

    def pull(self) -> None:
        for rank, ps, buf in self.plan:
            if not ps:
                continue
            self._hdr[0] = PULL
            dist.send(self._hdr, rank, group=self.group, tag=TAG_HDR)
            dist.recv(buf, rank, group=self.group, tag=TAG_DATA)
            off = 0
            with torch.no_grad():
                for p in ps:
                    n = p.numel()
                    p.copy_(buf[off:off + n].view_as(p))
                    off += n

    def push(self) -> int:
        """Send every PS its gradient shard; returns the global step reported by PS 0."""
        step = -1
        reply = torch.zeros(1, dtype=torch.int64)
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
            self._hdr[0] = PUSH
            dist.send(self._hdr, rank, group=self.group, tag=TAG_HDR)
            dist.send(buf, rank, group=self.group, tag=TAG_DATA)
            dist.recv(reply, rank, group=self.group, tag=TAG_REPLY)
            if k == 0:
                step = int(reply[0])
        return step

    def done(self) -> None:
        self._hdr[0] = DONE
        for rank, _, _ in self.plan:
            dist.send(self._hdr, rank, group=self.group, tag=TAG_HDR)


# ---------------------------------------------------------------------------
# device-resident transport (HIP IPC)
def _ipc_key(ps: int, what: str) -> str:
    return f"kfa/async_ps/{ps}/{what}"


def _export(store, key: str, t: torch.Tensor) -> None:
    """Publish a CUDA tensor to other processes of the job (HIP IPC handle)."""
    import pickle
    from torch.multiprocessing.reductions import reduce_tensor
    _, args = reduce_tensor(t)
    store.set(key, pickle.dumps(args))


def _import(store, key: str) -> torch.Tensor:
    import pickle
    from torch.multiprocessing.reductions import rebuild_cuda_tensor
    return rebuild_cuda_tensor(*pickle.loads(store.get(key)))  # bytes this job's own PS wrote


class DeviceAsyncPSServer:
    """PS task ``ps_index`` with its variables in GPU memory (see module docstring)."""

    def __init__(self, init_params: Sequence[Tuple[str, torch.Tensor]], num_workers: int, num_ps: int, ps_index: int,
                 store, device, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, optimizer: str = "adam",
                 group=None):
        self.W, self.P, self.idx = num_workers, num_ps, ps_index
        shapes = [(n, p.shape) for n, p in init_params]
        self.assignment = ps_assignment(list(init_params), num_ps)
        self.names, n = _layout(shapes, self.assignment, ps_index)
        src = dict(init_params)
        self.device = device
        npad = (n + 7) // 8 * 8  # the fused Adam kernel moves 8 values per thread; the tail stays 0
        self.w = torch.zeros(npad, dtype=torch.float32, device=device)
        if self.names:
            self.w[:n].copy_(torch.cat([src[k].detach().float().reshape(-1) for k in self.names]))
        self.m = torch.zeros_like(self.w)
        self.v = torch.zeros_like(self.w)
        self.mail = torch.zeros(num_workers, max(npad, 8), dtype=torch.float32, device=device)
        self.lr, self.betas, self.eps, self.opt = lr, betas, eps, optimizer
        self.t = 0
        self.global_step = 0
        self.group = group
        torch.cuda.synchronize(device)
        _export(store, _ipc_key(ps_index, "w"), self.w)
        _export(store, _ipc_key(ps_index, "mail"), self.mail)
        store.set(_ipc_key(ps_index, "ready"), "1")

    def _apply(self, g: torch.Tensor) -> None:
        from ..ops import _lib, optim  # noqa: F401  (optim registers kfa_adam_step)
        self.t += 1
        n = self.w.numel()
        if n == 0:
            return
        if self.opt == "sgd":
            self.w.add_(g, alpha=-self.lr)
            return
        b1, b2 = self.betas
        bc1, bc2 = 1.0 - b1 ** self.t, 1.0 - b2 ** self.t
        # TF AdamOptimizer form (eps outside the bias-corrected sqrt) with the fused HIP kernel
        _lib.call("kfa_adam_step", _lib.ptr(self.w), None, _lib.ptr(g), 0, _lib.ptr(self.m), _lib.ptr(self.v), n,
                  self.lr, b1, b2, self.eps / math.sqrt(bc2), 0.0, bc1, bc2, 1.0, None, _lib.stream())

    def serve(self, log=None) -> int:
        active = self.W
        hdr = torch.zeros(2, dtype=torch.int64)
        pushes = 0
        n = self.w.numel()  # padded length (the mailbox tail beyond the variables is never written: 0)
        while active > 0:
            src = dist.recv(hdr, src=None, group=self.group, tag=TAG_HDR)
            op = int(hdr[0])
            if op == PUSH:
                self._apply(self.mail[src, :n])
                torch.cuda.current_stream(self.device).synchronize()  # mailbox consumed, update visible
                pushes += 1
                self.global_step += 1
                dist.send(torch.tensor([self.global_step], dtype=torch.int64), src, group=self.group,
                          tag=TAG_REPLY)
                if log and self.global_step % 50 == 0:
                    log(f"PS {self.idx}: applied {self.global_step} updates")
            elif op == DONE:
                active -= 1
            else:
                raise RuntimeError(f"PS {self.idx}: bad request {op} from rank {src}")
        return pushes


class DeviceAsyncPSClient:
    """Worker side of the device transport: pulls and pushes are D2D copies."""

    def __init__(self, params: Sequence[Tuple[str, torch.nn.Parameter]], num_workers: int, num_ps: int, rank: int,
                 store, group=None, timeout: float = 300.0):
        import time
        self.W, self.P, self.rank, self.group = num_workers, num_ps, rank, group
        self.params = list(params)
        self.assignment = ps_assignment(self.params, num_ps)
        shapes = [(n, p.shape) for n, p in self.params]
        by_name = dict(self.params)
        self.plan = []
        t0 = time.time()
        for k in range(num_ps):
            names, n = _layout(shapes, self.assignment, k)
            while True:  # the PS publishes its buffers once its variables are on the GPU
                try:
                    if store.check([_ipc_key(k, "ready")]):
                        break
                except Exception:
                    pass
                if time.time() - t0 > timeout:
                    raise TimeoutError(f"PS {k} did not publish its device buffers")
                time.sleep(0.05)
            w = _import(store, _ipc_key(k, "w"))
            mail = _import(store, _ipc_key(k, "mail"))
            self.plan.append((num_workers + k, [by_name[x] for x in names], w, mail[rank], n))
        self._hdr = torch.zeros(2, dtype=torch.int64)

    @torch.no_grad()
    def pull(self) -> None:
        for _, ps, w, _, n in self.plan:
            off = 0
            for p in ps:
                k = p.numel()
                p.copy_(w[off:off + k].view_as(p))   # device-to-device (peer) copy + cast
                off += k

    @torch.no_grad()
    def push(self) -> int:
        step = -1
        reply = torch.zeros(1, dtype=torch.int64)
        for k, (rank, ps, _, mail, n) in enumerate(self.plan):
            if not ps:
                continue
            off = 0
            for p in ps:
                c = p.numel()
                if p.grad is None:
                    mail[off:off + c].zero_()
                else:
                    mail[off:off + c].copy_(p.grad.reshape(-1))
                off += c
            torch.cuda.current_stream(mail.device).synchronize()  # the mailbox is written before the header
            self._hdr[0] = PUSH
            dist.send(self._hdr, rank, group=self.group, tag=TAG_HDR)
            dist.recv(reply, rank, group=self.group, tag=TAG_REPLY)
            if k == 0:
                step = int(reply[0])
        return step

    def done(self) -> None:
        self._hdr[0] = DONE
        for rank, *_ in self.plan:
            dist.send(self._hdr, rank, group=self.group, tag=TAG_HDR)
