"""Communicators for the gradient / parameter traffic (SURVEY §1.2 L0 comm, §2.5, §2.7, §5.8).

Two implementations of one small interface (``all_reduce``, ``reduce_scatter_tensor``,
``all_gather_into_tensor``, ``broadcast``, ``reduce``, ``all_to_all_single``,
``send`` / ``recv``, ``barrier``; every collective takes ``async_op`` and returns a
work object with ``wait()``):

* :class:`Communicator` — the first-party layer, ``csrc/comm/comm.cpp``
  (``parallel/_kfc_comm.so``).  Bootstrap: rank 0 (the chief) opens a TCP
  listener and publishes ``host:port`` in the job's rendezvous store — the store
  every replica already reaches on the chief's cluster-spec endpoint, the
  kube-dns stand-in of ``kubelet/endpoints.py``; every other rank connects and
  receives the RCCL unique id (one exchange per communicator, the analogue of the
  reference's ``tf.train.Server`` bind, ``mnist_replica.py:117-122``).  Then
  RCCL's collectives run directly on the caller's flat buffers on this
  communicator's OWN HIP stream: it first waits for the caller's stream (the
  kernels that produced the bucket), and hands the result back through an event
  that ``Work.wait()`` makes the caller's stream wait on — the optimizer (or the
  next forward) waits for exactly the buckets it reads.  On a CPU the same C++
  layer runs its host-TCP backend (``backend="host"``) so it is tested against
  gloo without a GPU (``tests/test_comm_cpu.py``).
* :class:`TorchComm` — ``torch.distributed`` on a process group (gloo on the
  CPU: the test double; ``KFA_COMM=torch`` also selects it on GPUs for A/B).

:func:`make_comm` picks one: ``KFA_COMM`` = ``native`` | ``torch``; default
native on GPUs (RCCL), torch (gloo) on the CPU.

ONE RCCL communicator per process: a GPU job whose gradient traffic runs on the
native layer initialises ``torch.distributed`` with **gloo** (:func:`dist_backend`)
and uses it for control scalars only — tuner agreement (``routes._agree_index``,
``conv._agree``), the timing MAX, barriers, the native layer's keep/fall-back vote
— always on CPU tensors (:func:`control_device`).  No torch RCCL communicator is
created unless the native layer fails on some rank; then every rank falls back
together to a torch ``nccl`` group created at that point.  ``KFA_COMM=torch``
keeps the old layout (nccl default group, torch's communicator for everything)
for A/B.  RCCL's transport choice per peer (P2P/IPC over xGMI vs SHM / NET) is
read from its INIT/P2P log at bring-up (:attr:`Communicator.transport`) and
reported in ``bench.py``'s ``config.comm``.
"""
from __future__ import annotations

import ctypes
import itertools
import os
import re
import sys
import tempfile
from typing import Dict, Optional, Sequence

import torch
import torch.distributed as dist

_P, _L, _I, _S = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_size_t
_LIB = None

_DT = {torch.int8: 0, torch.uint8: 1, torch.int32: 2, torch.int64: 4, torch.float16: 6, torch.float32: 7,
       torch.float64: 8, torch.bfloat16: 9, torch.bool: 1}
_OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3, "avg": 4}


def _op_code(op) -> int:
    if isinstance(op, str):
        return _OPS[op.lower()]
    name = str(op).split(".")[-1].lower()   # dist.ReduceOp.SUM / RedOpType.SUM
    for k, v in (("sum", 0), ("product", 1), ("prod", 1), ("max", 2), ("min", 3), ("avg", 4)):
        if name.startswith(k):
            return v
    raise ValueError(f"unsupported reduction op {op!r}")


def lib() -> ctypes.CDLL:
    """The comm library (built in-tree by ``_build.build_comm``; built here if
    missing and a compiler is present — it is plain C++, no ROCm toolchain)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    from .. import _build
    # rebuilt when comm.cpp changed since the library was built (source stamp, under
    # the build lock, atomic replace): a stale .so would bind a different ABI
    path = _build.build_comm()
    L = ctypes.CDLL(path)
    sig = {
        "kfc_last_error": ([], ctypes.c_char_p), "kfc_listen": ([ctypes.c_char_p, _I, ctypes.POINTER(_I)], _I),
        "kfc_close_fd": ([_I], None), "kfc_rccl_path": ([], ctypes.c_char_p), "kfc_rccl_version": ([], _I),
        "kfc_comm_init": ([ctypes.c_char_p, _I, _I, ctypes.c_char_p, _I, _I, _I], _P),
        "kfc_backend": ([_P], ctypes.c_char_p),
        "kfc_all_reduce": ([_P, _P, _P, _S, _I, _I, _P], _I),
        "kfc_reduce_scatter": ([_P, _P, _P, _S, _I, _I, _P], _I),
        "kfc_all_gather": ([_P, _P, _P, _S, _I, _P], _I),
        "kfc_broadcast": ([_P, _P, _P, _S, _I, _I, _P], _I),
        "kfc_reduce": ([_P, _P, _P, _S, _I, _I, _I, _P], _I),
        "kfc_send": ([_P, _P, _S, _I, _I, _P], _I), "kfc_recv": ([_P, _P, _S, _I, _I, _P], _I),
        "kfc_recv_any": ([_P, _P, _S, _I, ctypes.POINTER(_I), _I], _I),
        "kfc_all_to_all_v": ([_P, _P, _P, _P, _P, _P, _P, _I, _P], _I),
        "kfc_group_start": ([_P], _I), "kfc_group_end": ([_P], _I), "kfc_async_error": ([_P], _I),
        "kfc_comm_abort": ([_P], None), "kfc_comm_destroy": ([_P], None),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes, f.restype = args, res
    _LIB = L
    return L


class CommError(RuntimeError):
    pass


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise CommError(f"{what}: {lib().kfc_last_error().decode(errors='replace')} (code {rc})")


class Work:
    """Completion of one collective: ``wait()`` orders the caller's CURRENT stream
    after it (no host wait); CPU collectives are complete on return."""
    __slots__ = ("event", "device")

    def __init__(self, event=None, device=None):
        self.event, self.device = event, device

    def wait(self) -> bool:
        if self.event is not None:
            torch.cuda.current_stream(self.device).wait_event(self.event)
        return True

    def is_completed(self) -> bool:
        return self.event is None or self.event.query()


def _ptr(t: torch.Tensor):
    return ctypes.c_void_p(t.data_ptr())


_KEYS = itertools.count()


class Communicator:
    """One communicator of the first-party layer (see the module docstring)."""

    native = True

    def __init__(self, handle, rank: int, world: int, device: torch.device, backend: str,
                 debug_log: Optional[str] = None):
        self._h = handle
        self.rank, self.world, self.device, self.backend = rank, world, device, backend
        self.stream = torch.cuda.Stream(device=device) if device.type == "cuda" else None
        self._debug_log = debug_log   # RCCL's INIT/P2P log of this process (transport capture)
        self._transport: Optional[Dict] = None

    @classmethod
    def create(cls, store, rank: int, world: int, device: torch.device, backend: Optional[str] = None,
               advertise_host: Optional[str] = None, key: Optional[str] = None,
               timeout_s: float = 300.0) -> "Communicator":
        """Collective over every rank: rank 0 listens and publishes its address under
        ``key`` in ``store`` (a ``torch.distributed`` Store); the others read it and
        connect.  Every rank must create its communicators in the same order.

        Rank 0 publishes the key even when it fails before listening (``ERR:<why>``),
        so the other ranks fail at once instead of waiting out the store timeout."""
        backend = backend or ("rccl" if device.type == "cuda" else "host")
        key = key or f"kfc/comm/{next(_KEYS)}"
        tmo = int(timeout_s * 1000)
        if rank == 0:
            try:
                L = lib()
                port = ctypes.c_int(0)
                fd = L.kfc_listen(b"", 0, ctypes.byref(port))
                if fd < 0:
                    _check(-fd, "kfc_listen")
            except Exception as e:  # noqa: BLE001 - tell the peers, then raise
                store.set(key, f"ERR:{e}")
                raise
            host = advertise_host or os.environ.get("MASTER_ADDR", "127.0.0.1")
            store.set(key, f"{host}:{port.value}")
            log = _arm_rccl_log(key) if backend == "rccl" else None
            h = L.kfc_comm_init(backend.encode(), world, 0, None, 0, fd, tmo)
            _disarm_rccl_log()
        else:
            addr = store.get(key).decode()
            if addr.startswith("ERR:"):
                raise CommError(f"rank 0 could not open the communicator: {addr[4:]}")
            L = lib()
            host, _, port = addr.rpartition(":")
            log = _arm_rccl_log(key) if backend == "rccl" else None
            h = L.kfc_comm_init(backend.encode(), world, rank, host.encode(), int(port), -1, tmo)
            _disarm_rccl_log()
        if not h:
            raise CommError(f"kfc_comm_init({backend}, rank {rank}/{world}): {L.kfc_last_error().decode()}")
        return cls(h, rank, world, device, backend, debug_log=log)

    @property
    def transport(self) -> Dict:
        """RCCL's transport per connection of this rank, from its INIT/P2P log:
        ``{"via": {"P2P/IPC": n, ...}, "peers": {peer: transport}}`` (P2P/IPC =
        direct xGMI peer access; SHM / NET = a fallback through host memory / sockets);
        ``{"via": "unknown"}`` when the log was not available (``NCCL_DEBUG`` set by
        the user, or RCCL's logging already initialised in this process)."""
        if self._transport is None and self.backend == "rccl":
            t = parse_rccl_transport(self._debug_log, self.rank)
            if t.get("via") != "unknown":
                self._transport = t
            return t
        return self._transport or {"via": self.backend}

    # -------------------------------------------------------------- plumbing
    def _stream_arg(self):
        return ctypes.c_void_p(self.stream.cuda_stream) if self.stream is not None else None

    def _run(self, tensors: Sequence[torch.Tensor], fn, what: str, async_op: bool) -> Work:
        if self._h is None:
            raise CommError("communicator destroyed")
        if self.stream is None:
            _check(fn(None), what)
            return Work()
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)           # the producing kernels first
        _check(fn(self._stream_arg()), what)
        for t in tensors:                       # keep the caching allocator off these until the comm stream is done
            t.record_stream(self.stream)
        ev = torch.cuda.Event()
        ev.record(self.stream)
        w = Work(ev, self.device)
        if not async_op:
            cur.wait_event(ev)
        return w

    @staticmethod
    def _dt(t: torch.Tensor) -> int:
        if t.dtype not in _DT:
            raise CommError(f"unsupported dtype {t.dtype}")
        if not t.is_contiguous():
            raise CommError("collective buffers must be contiguous")
        return _DT[t.dtype]

    # -------------------------------------------------------------- collectives
    def all_reduce(self, t: torch.Tensor, op="sum", async_op: bool = False) -> Work:
        dt, oc = self._dt(t), _op_code(op)
        return self._run([t], lambda s: lib().kfc_all_reduce(self._h, _ptr(t), _ptr(t), t.numel(), dt, oc, s),
                         "all_reduce", async_op)

    def reduce_scatter_tensor(self, out: torch.Tensor, inp: torch.Tensor, op="sum", async_op: bool = False) -> Work:
        dt, oc = self._dt(inp), _op_code(op)
        if out.dtype != inp.dtype or inp.numel() != out.numel() * self.world:
            raise CommError(f"reduce_scatter: input {inp.numel()} != world {self.world} x output {out.numel()}")
        return self._run([out, inp], lambda s: lib().kfc_reduce_scatter(self._h, _ptr(inp), _ptr(out), out.numel(),
                                                                         dt, oc, s), "reduce_scatter", async_op)

    def all_gather_into_tensor(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False) -> Work:
        dt = self._dt(inp)
        if out.dtype != inp.dtype or out.numel() != inp.numel() * self.world:
            raise CommError(f"all_gather: output {out.numel()} != world {self.world} x input {inp.numel()}")
        return self._run([out, inp], lambda s: lib().kfc_all_gather(self._h, _ptr(inp), _ptr(out), inp.numel(), dt,
                                                                     s), "all_gather", async_op)

    def broadcast(self, t: torch.Tensor, src: int, async_op: bool = False) -> Work:
        dt = self._dt(t)
        return self._run([t], lambda s: lib().kfc_broadcast(self._h, _ptr(t), _ptr(t), t.numel(), dt, src, s),
                         "broadcast", async_op)

    def reduce(self, t: torch.Tensor, dst: int, op="sum", async_op: bool = False) -> Work:
        dt, oc = self._dt(t), _op_code(op)
        return self._run([t], lambda s: lib().kfc_reduce(self._h, _ptr(t), _ptr(t), t.numel(), dt, oc, dst, s),
                         "reduce", async_op)

    def send(self, t: torch.Tensor, dst: int, async_op: bool = False) -> Work:
        dt = self._dt(t)
        return self._run([t], lambda s: lib().kfc_send(self._h, _ptr(t), t.numel(), dt, dst, s), "send", async_op)

    def recv(self, t: torch.Tensor, src: int, async_op: bool = False) -> Work:
        dt = self._dt(t)
        return self._run([t], lambda s: lib().kfc_recv(self._h, _ptr(t), t.numel(), dt, src, s), "recv", async_op)

    def recv_any(self, t: torch.Tensor, timeout_s: Optional[float] = None) -> int:
        """Receive one message from whichever rank sends first (host backend, CPU
        tensors); returns that rank.  Every rank's messages to this one arrive in
        the order it sent them."""
        if self.device.type != "cpu":
            raise CommError("recv_any: host-memory tensors only")
        src = ctypes.c_int(-1)
        _check(lib().kfc_recv_any(self._h, _ptr(t), t.numel(), self._dt(t), ctypes.byref(src),
                                  int((timeout_s or 0) * 1000)), "recv_any")
        return src.value

    def all_to_all_single(self, out: torch.Tensor, inp: torch.Tensor, out_splits: Sequence[int],
                          in_splits: Sequence[int], async_op: bool = False) -> Work:
        """Rows of ``inp`` (``in_splits[p]`` of them to rank p) -> rows of ``out``
        (``out_splits[p]`` from rank p): one grouped send / recv batch, the local
        block copied on the communicator's stream."""
        dt = self._dt(inp)
        row = inp[0].numel() if inp.dim() > 1 and inp.shape[0] else (out[0].numel() if out.dim() > 1 and out.shape[0]
                                                                    else 1)
        W = self.world
        sc = (ctypes.c_int64 * W)(*[int(n) * row for n in in_splits])
        rc = (ctypes.c_int64 * W)(*[int(n) * row for n in out_splits])
        so = (ctypes.c_int64 * W)(*[sum(in_splits[:p]) * row for p in range(W)])
        ro = (ctypes.c_int64 * W)(*[sum(out_splits[:p]) * row for p in range(W)])
        r = self.rank

        def fn(s):
            rc_ = lib().kfc_all_to_all_v(self._h, _ptr(inp), sc, so, _ptr(out), rc, ro, dt, s)
            if rc_ == 0 and in_splits[r]:
                src = inp.reshape(-1)[so[r]:so[r] + sc[r]]
                dst = out.reshape(-1)[ro[r]:ro[r] + rc[r]]
                if self.stream is not None:
                    with torch.cuda.stream(self.stream):
                        dst.copy_(src)
                else:
                    dst.copy_(src)
            return rc_
        return self._run([out, inp], fn, "all_to_all", async_op)

    def barrier(self) -> None:
        t = torch.ones(1, dtype=torch.int32, device=self.device)
        self.all_reduce(t)
        if self.stream is not None:
            torch.cuda.current_stream(self.device).synchronize()
        if int(t.item()) != self.world:
            raise CommError(f"barrier: {int(t.item())} of {self.world} ranks")

    def check(self) -> None:
        """Raise if the backend recorded an asynchronous error (RCCL)."""
        _check(lib().kfc_async_error(self._h), "async error")

    def destroy(self, abort: bool = False) -> None:
        if self._h is not None:
            (lib().kfc_comm_abort if abort else lib().kfc_comm_destroy)(self._h)
            self._h = None

    def __repr__(self) -> str:
        return f"Communicator({self.backend}, rank {self.rank}/{self.world}, {self.device})"


_RCCL_LOG_VARS = ("NCCL_DEBUG", "NCCL_DEBUG_SUBSYS", "NCCL_DEBUG_FILE")


def _arm_rccl_log(key: str) -> Optional[str]:
    """Point RCCL's INFO log (INIT and P2P subsystems only) at a per-process file
    for the transport capture, unless the user set ``NCCL_DEBUG`` (then theirs
    stands) or ``KFA_RCCL_TRANSPORT_LOG=0``.  RCCL reads these variables once per
    process, at its first call; the file keeps receiving the lazily-made
    connections' lines (the first collectives)."""
    if os.environ.get("KFA_RCCL_TRANSPORT_LOG", "1") != "1" or "NCCL_DEBUG" in os.environ:
        return None
    path = os.path.join(tempfile.gettempdir(),
                        f"kfc_rccl_{os.getpid()}_{re.sub(r'[^A-Za-z0-9]', '_', key)}.log")
    os.environ.update({"NCCL_DEBUG": "INFO", "NCCL_DEBUG_SUBSYS": "INIT,P2P", "NCCL_DEBUG_FILE": path})
    return path


def _disarm_rccl_log() -> None:
    """Drop the logging variables from this process's environment again (children
    must not inherit them); RCCL keeps the settings it already read."""
    for v in _RCCL_LOG_VARS:
        os.environ.pop(v, None)


_VIA = re.compile(r"(\d+)\[[^\]]*\]\s*->\s*(\d+)\[[^\]]*\]\s*(?:\[\w+\]\s*)?via\s+(\S+)")


def parse_rccl_transport(path: Optional[str], rank: int) -> Dict:
    """Summarise RCCL's "Channel cc/r : a[d] -> b[e] via T" lines for ``rank``."""
    if not path or not os.path.exists(path):
        return {"via": "unknown"}
    via: Dict[str, int] = {}
    peers: Dict[int, str] = {}
    with open(path, errors="replace") as f:
        for line in f:
            m = _VIA.search(line)
            if not m:
                continue
            a, b, t = int(m.group(1)), int(m.group(2)), m.group(3)
            if rank not in (a, b) or a == b:
                continue
            via[t] = via.get(t, 0) + 1
            peers.setdefault(b if a == rank else a, t)
    if not via:
        return {"via": "unknown"}
    return {"via": via, "peers": {str(k): v for k, v in sorted(peers.items())}}


class TorchComm:
    """The same interface over ``torch.distributed`` (gloo on the CPU: the test double)."""

    native = False
    backend = "torch"

    def __init__(self, process_group=None):
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(process_group) if dist.is_initialized() else 0

    @staticmethod
    def _rop(op):
        if not isinstance(op, str):
            return op
        return {"sum": dist.ReduceOp.SUM, "prod": dist.ReduceOp.PRODUCT, "max": dist.ReduceOp.MAX,
                "min": dist.ReduceOp.MIN, "avg": dist.ReduceOp.AVG}[op]

    def all_reduce(self, t, op="sum", async_op=False):
        return dist.all_reduce(t, op=self._rop(op), group=self.pg, async_op=async_op) or Work()

    def reduce_scatter_tensor(self, out, inp, op="sum", async_op=False):
        return dist.reduce_scatter_tensor(out, inp, op=self._rop(op), group=self.pg, async_op=async_op) or Work()

    def all_gather_into_tensor(self, out, inp, async_op=False):
        return dist.all_gather_into_tensor(out, inp, group=self.pg, async_op=async_op) or Work()

    def broadcast(self, t, src, async_op=False):
        return dist.broadcast(t, src, group=self.pg, async_op=async_op) or Work()

    def reduce(self, t, dst, op="sum", async_op=False):
        return dist.reduce(t, dst, op=self._rop(op), group=self.pg, async_op=async_op) or Work()

    def send(self, t, dst, async_op=False):
        if async_op:
            return dist.isend(t, dst, group=self.pg)
        dist.send(t, dst, group=self.pg)
        return Work()

    def recv(self, t, src, async_op=False):
        if async_op:
            return dist.irecv(t, src, group=self.pg)
        dist.recv(t, src, group=self.pg)
        return Work()

    def recv_any(self, t, timeout_s=None, tag: int = 0) -> int:
        return dist.recv(t, src=None, group=self.pg, tag=tag)

    def all_to_all_single(self, out, inp, out_splits, in_splits, async_op=False):
        return dist.all_to_all_single(out, inp, list(out_splits), list(in_splits), group=self.pg,
                                      async_op=async_op) or Work()

    def barrier(self):
        dist.barrier(group=self.pg)

    def check(self):
        pass

    def destroy(self, abort=False):
        pass

    def __repr__(self) -> str:
        return f"TorchComm({dist.get_backend(self.pg) if dist.is_initialized() else 'none'}, {self.world} ranks)"


class P2P:
    """Point-to-point channel of the asynchronous parameter server
    (``parallel/async_ps.py``): ``send`` / ``recv`` to one rank, ``recv_any`` from
    whichever rank sends first.  ``native``: the first-party host transport
    (:class:`Communicator`, ``backend="host"``: per-pair ordered TCP streams, so
    the protocol's tags are implied by the order of its messages); else
    ``torch.distributed`` on the default group with the tags (gloo)."""

    def __init__(self, comm=None, group=None):
        self.comm, self.group = comm, group

    @property
    def native(self) -> bool:
        return self.comm is not None

    def send(self, t: torch.Tensor, dst: int, tag: int = 0) -> None:
        if self.comm is not None:
            self.comm.send(t, dst)
        else:
            dist.send(t, dst, group=self.group, tag=tag)

    def recv(self, t: torch.Tensor, src: int, tag: int = 0) -> None:
        if self.comm is not None:
            self.comm.recv(t, src)
        else:
            dist.recv(t, src, group=self.group, tag=tag)

    def recv_any(self, t: torch.Tensor, tag: int = 0) -> int:
        if self.comm is not None:
            return self.comm.recv_any(t)
        return dist.recv(t, src=None, group=self.group, tag=tag)

    def destroy(self) -> None:
        if self.comm is not None:
            self.comm.destroy()
            self.comm = None

    def __repr__(self) -> str:
        return f"P2P({self.comm!r})" if self.comm is not None else "P2P(torch.distributed)"


def make_p2p(store=None, mode: Optional[str] = None, timeout_s: Optional[float] = None, group=None) -> P2P:
    """The async PS control / host-data channel over the default group's ranks:
    ``KFA_PS_P2P`` = ``native`` (default: the first-party host transport) | ``torch``
    (gloo; also for a sub-group).  Collective over every rank of the default group."""
    mode = (mode or os.environ.get("KFA_PS_P2P", "native")).lower()
    if mode == "torch" or not dist.is_initialized() or (group is not None and group is not dist.group.WORLD):
        return P2P(None, group)
    t = timeout_s if timeout_s is not None else float(os.environ.get("KFA_PS_P2P_TIMEOUT", "1800"))
    return P2P(Communicator.create(store or default_store(), dist.get_rank(), dist.get_world_size(),
                                   torch.device("cpu"), backend="host", key="kfc/ps_p2p", timeout_s=t))


_CONTROL_ONLY = False  # the default group is gloo for control scalars; RCCL = the native layer


def dist_backend(use_gpu: bool) -> str:
    """Backend for a job's default ``torch.distributed`` group: ``KFA_DIST_BACKEND``
    if set (gloo on GPUs = several ranks sharing one GPU, which RCCL refuses);
    else on GPUs **gloo** when the gradient traffic will run on the native
    communicator (control scalars only, see the module doc) and nccl under
    ``KFA_COMM=torch``; gloo on the CPU."""
    forced = os.environ.get("KFA_DIST_BACKEND")
    if forced:
        return forced
    if not use_gpu:
        return "gloo"
    return "nccl" if os.environ.get("KFA_COMM", "").lower() == "torch" else "gloo"


def init_default_group(rank: int, world: int, device: torch.device, timeout, store=None,
                       backend: Optional[str] = None) -> str:
    """``dist.init_process_group`` with :func:`dist_backend`; returns the backend.
    An nccl group is bound to ``device`` (eager communicator); a control-only gloo
    group on a GPU job marks this process for the native layer (:func:`comm_mode`)."""
    global _CONTROL_ONLY
    use_gpu = device.type == "cuda"
    be = backend or dist_backend(use_gpu)
    if be == "nccl":
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    kw = {"device_id": device} if (be == "nccl" and use_gpu) else {}
    if store is not None:
        kw["store"] = store
    dist.init_process_group(be, rank=rank, world_size=world, timeout=timeout, **kw)
    _CONTROL_ONLY = use_gpu and be == "gloo" and not (backend or os.environ.get("KFA_DIST_BACKEND"))
    return be


def control_device(device) -> torch.device:
    """Where a control scalar lives for a collective on the default group: the GPU
    only when that group IS torch's RCCL (``KFA_COMM=torch``), else the CPU (gloo)."""
    if device is not None and torch.device(device).type == "cuda" and dist.is_initialized() \
            and dist.get_backend() == "nccl":
        return torch.device(device)
    return torch.device("cpu")


def comm_mode(device: torch.device) -> str:
    """``KFA_COMM`` if set; else native on GPUs whose default group runs RCCL or is
    the control-only gloo group of :func:`init_default_group` — a job that forced
    gloo on GPUs (``KFA_DIST_BACKEND=gloo``: several ranks sharing one GPU, which
    RCCL refuses) keeps torch.distributed — and torch (gloo) on the CPU."""
    m = os.environ.get("KFA_COMM", "").lower()
    if m in ("native", "torch"):
        return m
    if device.type != "cuda":
        return "torch"
    if dist.is_initialized() and dist.get_backend() != "nccl" and not _CONTROL_ONLY:
        return "torch"
    return "native"


def default_store():
    """The rendezvous store of the default process group (rank 0 hosts it on the
    chief's endpoint)."""
    try:
        return dist.distributed_c10d._get_default_store()
    except Exception:  # noqa: BLE001 - older / private API: connect a client to MASTER_ADDR:PORT
        return dist.TCPStore(os.environ.get("MASTER_ADDR", "127.0.0.1"), int(os.environ["MASTER_PORT"]),
                             is_master=False)


def _probe(comm, device, world: int, rank: int, a2a: bool = False) -> str:
    """Every collective the data-parallel paths use — reduce-scatter, all-gather, fp32
    and bf16 all-reduce (sum, max), broadcast from the last rank (``a2a``: also an uneven
    all-to-all, the embedding exchange's) — over rank-distinct values, checked element by
    element: catches a wrong offset, order, op or dtype, not only a dead communicator
    ("" = good).  Integers below 2^8 keep the bf16 sums exact."""
    n = 4 * world + 3  # per-rank block, odd
    base = torch.arange(n * world, dtype=torch.float32, device=device)
    inp = base * (rank + 1) + 1000.0 * rank
    out = torch.empty(n, dtype=torch.float32, device=device)
    comm.reduce_scatter_tensor(out, inp, "sum")
    tot = sum(r + 1 for r in range(world))
    want = base[rank * n:(rank + 1) * n] * tot + 1000.0 * sum(range(world))
    if not torch.equal(out, want):
        return f"probe reduce-scatter mismatch on rank {rank}"
    mine = torch.full((n,), float(rank * 7 + 1), device=device) + torch.arange(n, dtype=torch.float32, device=device)
    g = torch.empty(n * world, dtype=torch.float32, device=device)
    comm.all_gather_into_tensor(g, mine)
    want = torch.cat([torch.full((n,), float(r * 7 + 1), device=device)
                      + torch.arange(n, dtype=torch.float32, device=device) for r in range(world)])
    if device.type == "cuda":
        torch.cuda.current_stream(device).synchronize()
    if not torch.equal(g, want):
        return f"probe all-gather mismatch on rank {rank}"
    for dt in (torch.float32, torch.bfloat16):
        a = (torch.arange(n, device=device) % 7 + rank + 1).to(dt)
        comm.all_reduce(a, "sum")
        want = (torch.arange(n, device=device) % 7 * world + sum(r + 1 for r in range(world))).to(dt)
        if device.type == "cuda":
            torch.cuda.current_stream(device).synchronize()
        if not torch.equal(a, want):
            return f"probe {dt} all-reduce mismatch on rank {rank}"
    m = torch.arange(n, dtype=torch.float32, device=device) + 100.0 * rank
    comm.all_reduce(m, "max")
    b = torch.arange(n, dtype=torch.float32, device=device) * (rank + 2)
    comm.broadcast(b, world - 1)
    if device.type == "cuda":
        torch.cuda.current_stream(device).synchronize()
    if not torch.equal(m, torch.arange(n, dtype=torch.float32, device=device) + 100.0 * (world - 1)):
        return f"probe all-reduce max mismatch on rank {rank}"
    if not torch.equal(b, torch.arange(n, dtype=torch.float32, device=device) * (world + 1)):
        return f"probe broadcast mismatch on rank {rank}"
    if a2a:  # uneven all-to-all: rank r sends (r + p + 1) values r * 100 + p to rank p
        ins = [rank + p + 1 for p in range(world)]
        outs = [p + rank + 1 for p in range(world)]
        src = torch.cat([torch.full((c,), float(rank * 100 + p), device=device) for p, c in enumerate(ins)])
        dst = torch.empty(sum(outs), device=device)
        comm.all_to_all_single(dst, src, outs, ins)
        if device.type == "cuda":
            torch.cuda.current_stream(device).synchronize()
        want = torch.cat([torch.full((c,), float(p * 100 + rank), device=device) for p, c in enumerate(outs)])
        if not torch.equal(dst, want):
            return f"probe all-to-all mismatch on rank {rank}"
    return ""


def make_comm(device: torch.device, process_group=None, store=None, mode: Optional[str] = None):
    """The communicator for a job's gradient / parameter traffic (see module doc)."""
    mode = mode or comm_mode(device)
    if not dist.is_initialized() or dist.get_world_size(process_group) == 1 or mode == "torch":
        return TorchComm(process_group)
    if process_group is not None and process_group is not dist.group.WORLD:
        raise CommError("the native communicator spans the default group's ranks only")
    t = float(os.environ.get("KFA_DIST_INIT_TIMEOUT", "300"))
    world, rank = dist.get_world_size(), dist.get_rank()
    comm, err = None, ""
    try:
        comm = Communicator.create(store or default_store(), rank, world, device, timeout_s=t)
        err = _probe(comm, device, world, rank, a2a=os.environ.get("KFA_COMM_PROBE_A2A", "0") == "1")
        ok = not err
        if ok and comm.backend == "rccl":
            comm.transport  # noqa: B018 - read the log while the probe's connections are fresh
    except Exception as e:  # noqa: BLE001 - decided collectively below
        ok, err = False, str(e)
    # every rank keeps the native layer or none does (a rank that fell back alone would
    # leave its peers waiting in collectives it never joins); the vote rides the
    # default group on the CPU (gloo) unless that group is torch's RCCL
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=control_device(device))
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if int(flag.item()) == 1:
        return comm
    if comm is not None:
        comm.destroy()
    if mode == "native" and os.environ.get("KFA_COMM", "").lower() == "native":
        raise CommError(f"native communicator unavailable: {err or 'another rank failed'}")
    print(f"[kfc comm] native communicator unavailable ({err or 'another rank failed'}): torch.distributed",
          file=sys.stderr, flush=True)
    if device.type == "cuda" and dist.get_backend() != "nccl":
        # the control-only gloo default group cannot carry GPU tensors fast: torch's
        # RCCL in a group of its own (created by every rank together, here)
        return TorchComm(dist.new_group(backend="nccl"))
    return TorchComm(process_group)
