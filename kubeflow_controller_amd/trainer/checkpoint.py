"""Checkpoint / resume of a replica's training state.

The reference only had ``tf.train.Supervisor(logdir=tempfile.mkdtemp())``
(``mnist_replica.py:198-215``) — a pod-local temp dir, so nothing survived a
restart — and never read ``spec.modelDir``.  Here ``spec.modelDir`` reaches
every replica (env ``KFA_MODEL_DIR``, ``--model_dir``) and:

* every rank writes ``ckpt-<step>.rank<r>.pt``: the model ``state_dict``
  (parameters + buffers such as BN running stats), the fp32 master of each
  flat group and the optimizer state.  In the sharded (PS push/pull) layout a
  rank's optimizer state is only authoritative on the shard it owns, so each
  rank keeps its own file — the "PS shard owners write their shards" rule;
* rank 0 writes ``manifest.json`` last (atomically), naming the complete step;
* on start, a replica with a manifest resumes from it (its own rank file when
  the world size matches, else rank 0's weights with fresh optimizer state).

Files are loaded with ``torch.load(weights_only=True)`` only.
"""
from __future__ import annotations

import json
import os
from typing import Optional

import torch

MANIFEST = "manifest.json"


def _opt_state(opt) -> dict:
    st = {"step_count": int(getattr(opt, "step_count", 0))}
    for name in ("mom", "m", "v"):
        bufs = getattr(opt, name, None)
        if bufs is not None:
            st[name] = [b.detach().cpu() if b is not None else torch.empty(0) for b in bufs]
    return st


def _load_opt_state(opt, st: dict) -> None:
    opt.step_count = int(st.get("step_count", 0))
    for name in ("mom", "m", "v"):
        bufs = getattr(opt, name, None)
        if bufs is None or name not in st:
            continue
        for b, s in zip(bufs, st[name]):
            if b is not None and s.numel() == b.numel():
                b.copy_(s.to(b.device))


def save(model_dir: str, step: int, rank: int, world: int, model, groups=(), opt=None, extra: Optional[dict] = None,
         is_chief: bool = True, keep: int = 2, full_masters=None, layout: Optional[str] = None) -> str:
    """Write this rank's file.  ``full_masters`` (sharded layouts, rank 0): every
    group's full fp32 master, reassembled from the owners' shards, so a resume at
    a different world size restores exact fp32 weights."""
    os.makedirs(model_dir, exist_ok=True)
    if full_masters is not None:
        masters = [m.detach().cpu() for m in full_masters]
    else:
        masters = [g.master.detach().cpu() if g.master is not None else torch.empty(0) for g in groups]
    state = {
        "step": step,
        "world": world,
        "layout": layout or "",
        "model": {k: v.detach().cpu() for k, v in model.state_dict().items()},
        "masters": masters,
    }
    if opt is not None:
        state["opt"] = _opt_state(opt)
        state["spaces"] = [sp.w.detach().cpu() for sp in getattr(opt, "spaces", [])]
    if extra:
        state["extra"] = extra
    path = os.path.join(model_dir, f"ckpt-{step}.rank{rank}.pt")
    tmp = path + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, path)
    if is_chief:
        write_manifest(model_dir, step, world, keep)
    return path


def write_manifest(model_dir: str, step: int, world: int, keep: int = 2) -> None:
    """Publish ``step`` as the latest complete checkpoint (call after every rank saved)."""
    man = {"step": step, "world": world, "files": [f"ckpt-{step}.rank{r}.pt" for r in range(world)]}
    tmp = os.path.join(model_dir, MANIFEST + ".tmp")
    with open(tmp, "w") as f:
        json.dump(man, f)
    os.replace(tmp, os.path.join(model_dir, MANIFEST))
    _prune(model_dir, step, keep)


def _prune(model_dir: str, step: int, keep: int) -> None:
    steps = sorted({int(f.split("-")[1].split(".")[0]) for f in os.listdir(model_dir)
                    if f.startswith("ckpt-") and f.endswith(".pt")})
    for s in steps[:-keep]:
        if s == step:
            continue
        for f in os.listdir(model_dir):
            if f.startswith(f"ckpt-{s}."):
                try:
                    os.remove(os.path.join(model_dir, f))
                except FileNotFoundError:
                    pass


def latest(model_dir: str) -> Optional[dict]:
    p = os.path.join(model_dir, MANIFEST)
    if not model_dir or not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f)


def restore(model_dir: str, rank: int, world: int, model, groups=(), opt=None, layout: Optional[str] = None,
            sync=None) -> int:
    """Load the manifest's step into model/groups/opt; returns the step (0 if none).

    Same world size and layout: this rank's own file — weights, its fp32 master
    (shard) and optimizer state, exactly.  Otherwise rank 0's file: the weights
    and the FULL fp32 masters (each rank takes the part it owns through
    ``sync.load_full_master`` in the sharded layouts), fresh optimizer state."""
    man = latest(model_dir)
    if man is None:
        return 0
    own = os.path.join(model_dir, f"ckpt-{man['step']}.rank{rank}.pt")
    same_world = man.get("world") == world and os.path.exists(own)
    path = own if same_world else os.path.join(model_dir, man["files"][0])
    state = torch.load(path, map_location="cpu", weights_only=True)
    model.load_state_dict(state["model"])
    exact = (same_world and opt is not None and "opt" in state and "spaces" in state
             and (layout is None or state.get("layout", "") in ("", layout))
             and all(a.numel() == b.w.numel() for a, b in zip(state["spaces"], opt.spaces)))
    if exact:
        for sp, w in zip(opt.spaces, state["spaces"]):
            sp.w.copy_(w.to(sp.w.device))
        _load_opt_state(opt, state["opt"])
        return int(state["step"])
    chief = os.path.join(model_dir, man["files"][0])
    if path != chief:  # full masters: rank 0's file (the sharded layouts write them there only)
        state = torch.load(chief, map_location="cpu", weights_only=True)
    masters = state.get("masters", [])
    for gi, g in enumerate(groups):
        m = masters[gi] if gi < len(masters) else torch.empty(0)
        full = g.data.detach().float()
        if m.numel():  # same parameter offsets at any world size; only the tail padding differs
            k = min(m.numel(), g.numel)
            full[:k] = m[:k].to(full.device)
        if sync is not None:
            sync.load_full_master(gi, full)
        elif g.master is not None:
            g.master.copy_(full.to(g.master.device))
            g.data.copy_(g.master)
    return int(state["step"])
