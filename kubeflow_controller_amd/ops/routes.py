"""Per-shape kernel routing table (own kernel variant vs library, conv tile / prologue
choices), committed per GPU architecture so two boxes run the SAME kernels.

Every per-shape decision of the ops layer (``gemm.pick_fastest`` /
``gemm.prefer_own`` / ``conv._use_bnpro`` / ``conv`` tile variants) goes through
:func:`decide`:

1. ``KFA_ROUTES`` != ``off`` and the committed table (``ops/routes_<arch>.json``)
   holds the shape -> that candidate, by NAME, no timing;
2. else the candidates are timed (30 launches per sample, median of 3 samples,
   outside any graph capture), the fastest wins subject to the caller's margin,
   and rank 0's choice is applied on every rank.

``KFA_ROUTES=retune`` ignores the table (re-measures); ``KFA_ROUTES_DUMP=<path>``
writes every decision this process made (table hits included) as a table at
exit — ``tools/gpu_r5_routes.sh`` regenerates the committed file that way.
:func:`summary` (in ``bench.py``'s JSON) names the table by a content hash and
counts how many decisions came from it vs were measured, and own vs library.

Why: the round-4 tuner timed 10 launches once with a 1 % margin; own-kernel times
vary up to 16 % between boxes, so routing flipped from box to box and a measured
number did not identify a configuration.
"""
from __future__ import annotations

import atexit
import hashlib
import json
import os
import statistics
import sys
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch

ARCH = os.environ.get("KFA_ROUTES_ARCH", "gfx950")
MODE = os.environ.get("KFA_ROUTES", "on").lower()     # on | off | retune
TABLE_PATH = os.environ.get("KFA_ROUTES_FILE",
                            os.path.join(os.path.dirname(os.path.abspath(__file__)), f"routes_{ARCH}.json"))
# candidate names that run a vendor library kernel; every other pick is an own HIP
# kernel ("sep" = the separate own BatchNorm-apply pass, "igemm" / "pp" = own conv tiles)
LIBRARY_NAMES = ("hipblaslt", "library", "vendor", "miopen")

_table: Optional[Dict[str, str]] = None
_made: Dict[str, dict] = {}      # key -> {"pick": name, "times": {...} | None, "from": "table" | "timed"}


def _load() -> Dict[str, str]:
    global _table
    if _table is None:
        _table = {}
        if MODE == "on" and os.path.exists(TABLE_PATH):
            with open(TABLE_PATH) as f:
                doc = json.load(f)
            _table = dict(doc.get("routes", {}))
    return _table


def key_str(kind: str, key: Sequence) -> str:
    return kind + "|" + ",".join(str(k) for k in key)


def time_ms(fn: Callable[[], object], reps: int = 30, samples: int = 3) -> float:
    """Median over ``samples`` of the mean time of ``reps`` back-to-back launches."""
    for _ in range(3):
        fn()
    out = []
    for _ in range(samples):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        out.append(s.elapsed_time(e) / reps)
    return statistics.median(out)


def _agree_index(i: int, device) -> int:
    """Rank 0's pick on every rank of a lockstep (data-parallel) job (see ``conv._agree``)."""
    import torch.distributed as dist
    from . import conv as _c
    if not _c._LOCKSTEP or not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return i
    from ..parallel.comm import control_device  # the CPU unless the default group is torch's RCCL
    t = torch.tensor([int(i)], dtype=torch.int32, device=control_device(device))
    dist.broadcast(t, 0)
    return int(t.item())


def decide(kind: str, key: Sequence, device, candidates: List[Tuple[str, Callable[[], object]]],
           margin: float = 0.99, log: bool = False) -> int:
    """Index of the candidate to run for this shape.  ``candidates[0]`` is the
    default (library / unfused) form: any other must beat it by ``margin``
    (time < margin x its time) to be measured-picked.  Returns 0 while a graph
    capture is in progress and the shape is not in the table."""
    ks = key_str(kind, key)
    if ks in _made:
        name = _made[ks]["pick"]
        for i, (n, _) in enumerate(candidates):
            if n == name:
                return i
    names = [n for n, _ in candidates]
    tab = _load()
    if ks in tab and tab[ks] in names:
        i = names.index(tab[ks])
        _made[ks] = {"pick": tab[ks], "times": None, "from": "table"}
        return i
    if torch.cuda.is_current_stream_capturing():
        return 0
    with torch.no_grad():
        ts = [time_ms(fn) for _, fn in candidates]
    best = min(range(1, len(ts)), key=lambda i: ts[i]) if len(ts) > 1 else 0
    if best and not ts[best] < margin * ts[0]:
        best = 0
    best = _agree_index(best, device)
    _made[ks] = {"pick": names[best], "times": {n: round(t, 5) for n, t in zip(names, ts)}, "from": "timed"}
    if log or os.environ.get("KFA_ROUTES_LOG", "0") == "1":
        desc = ", ".join(f"{n} {t:.4f} ms" for n, t in zip(names, ts))
        print(f"[kfa routes] {ks}: {desc} -> {names[best]}", file=sys.stderr, flush=True)
    return best


def digest() -> str:
    tab = _load()
    if not tab:
        return "none"
    return hashlib.sha1(json.dumps(tab, sort_keys=True).encode()).hexdigest()[:12]


def summary() -> dict:
    """What this process ran: the table's hash, decisions from the table vs timed,
    own-kernel vs library picks."""
    made = list(_made.values())
    own = sum(1 for m in made if m["pick"] not in LIBRARY_NAMES)
    return {"table": os.path.basename(TABLE_PATH) if _load() else None, "table_sha": digest(), "mode": MODE,
            "decisions": len(made), "from_table": sum(1 for m in made if m["from"] == "table"),
            "timed": sum(1 for m in made if m["from"] == "timed"), "own": own, "library": len(made) - own}


def dump(path: str) -> None:
    """Write this process's decisions (merged over an existing file at ``path``)."""
    doc = {"arch": ARCH, "routes": {}, "timings_ms": {}}
    if os.path.exists(path):
        with open(path) as f:
            old = json.load(f)
        doc["routes"].update(old.get("routes", {}))
        doc["timings_ms"].update(old.get("timings_ms", {}))
    for k, m in sorted(_made.items()):
        doc["routes"][k] = m["pick"]
        if m["times"]:
            doc["timings_ms"][k] = m["times"]
    with open(path + ".tmp", "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
    os.replace(path + ".tmp", path)


if os.environ.get("KFA_ROUTES_DUMP"):
    atexit.register(lambda: dump(os.environ["KFA_ROUTES_DUMP"]))
