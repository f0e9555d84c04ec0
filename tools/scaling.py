#!/usr/bin/env python3
"""Scaling harness: run ``bench.py`` at 1/2/4/8 GPUs of one
node back to back (one ``torchrun`` per N, one rank per GPU over RCCL/xGMI),
collect each run's JSON line and print the scaling table (whole-node value,
per-GPU value, weak-scaling efficiency vs N = 1) as markdown, optionally
writing the raw lines to a JSON file.

    python tools/scaling.py --gpus 1 2 4 8 --steps 20 --warmup 5 --out scale.json
    python tools/scaling.py --gpus 1 2 --backend gloo      # rehearsal: ranks share one GPU over gloo
    python tools/scaling.py --dry-run                       # print the commands only

Runs stop at the first failing N (a failed multi-GPU run says nothing about
the larger ones).  ``--backend gloo`` sets ``KFA_DIST_BACKEND=gloo`` (see
``trainer/engine.init_distributed``) so several ranks can share one GPU.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
from typing import Dict, List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def command(n: int, steps: int, warmup: int, port: int, extra: List[str]) -> List[str]:
    bench = os.path.join(ROOT, "bench.py")
    args = ["--gpus", str(n), "--steps", str(steps), "--warmup", str(warmup), *extra]
    if n == 1:
        return [sys.executable, bench, *args]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
            "--master-addr", "127.0.0.1", "--master-port", str(port), bench, *args]


def parse_line(out: str) -> Optional[Dict]:
    for line in reversed(out.strip().splitlines()):
        line = line.strip()
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    return None


def table(results: List[Dict]) -> str:
    base = next((r for r in results if r["n_gpus"] == 1), None)
    rows = ["| GPUs | value | per GPU | ms/step | weak-scaling efficiency |", "|---|---|---|---|---|"]
    for r in results:
        n = r["n_gpus"]
        eff = (r["value"] / (n * base["value"])) if base else None
        rows.append(f"| {n} | {r['value']:.1f} {r['unit']} | {r['value'] / n:.1f} | {r['ms_per_step']:.2f} | "
                    + (f"{eff * 100:.1f} %" if eff is not None else "—") + " |")
    return "\n".join(rows)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--port", type=int, default=29600)
    ap.add_argument("--timeout", type=int, default=900, help="seconds per run")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default=None)
    ap.add_argument("--out", default=None, help="write the raw JSON lines here")
    ap.add_argument("--dry-run", action="store_true")
    ap.add_argument("extra", nargs=argparse.REMAINDER, help="-- extra bench.py args (e.g. -- --batch 128)")
    a = ap.parse_args(argv)
    extra = a.extra[1:] if a.extra[:1] == ["--"] else a.extra
    env = dict(os.environ)
    if a.backend:
        env["KFA_DIST_BACKEND"] = a.backend
    results = []
    for i, n in enumerate(a.gpus):
        cmd = command(n, a.steps, a.warmup, a.port + i, extra)
        print("$ " + " ".join(cmd), file=sys.stderr, flush=True)
        if a.dry_run:
            continue
        p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=a.timeout)
        r = parse_line(p.stdout)
        if p.returncode != 0 or r is None:
            print(f"N={n} failed (exit {p.returncode}):\n{p.stderr[-4000:]}", file=sys.stderr)
            break
        results.append(r)
        print(json.dumps(r), flush=True)
    if results:
        print(table(results))
        if a.out:
            with open(a.out, "w") as f:
                json.dump(results, f, indent=1)
    return 0 if (a.dry_run or len(results) == len(a.gpus)) else 1


if __name__ == "__main__":
    sys.exit(main())
