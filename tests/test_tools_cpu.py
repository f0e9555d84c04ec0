"""CPU tests of the benchmark tooling: the scaling harness builds one torchrun per
N (127.0.0.1 rendezvous), parses bench.py's JSON line and computes weak-scaling
efficiency against N = 1."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

import scaling  # noqa: E402


def test_commands():
    one = scaling.command(1, 10, 2, 29600, [])
    assert one[1].endswith("bench.py") and "--gpus" in one and "1" in one
    eight = scaling.command(8, 10, 2, 29601, ["--batch", "128"])
    assert "torch.distributed.run" in eight and "--nproc-per-node" in eight
    assert eight[eight.index("--master-addr") + 1] == "127.0.0.1"
    assert eight[-2:] == ["--batch", "128"]


def test_parse_and_table():
    def line(n, v):
        return json.dumps({"metric": "images/sec", "value": v, "unit": "images/sec", "n_gpus": n,
                           "ms_per_step": 28.0})
    out = "warning: x\n" + line(2, 18000.0) + "\n"
    r = scaling.parse_line(out)
    assert r["n_gpus"] == 2 and r["value"] == 18000.0
    assert scaling.parse_line("no json here") is None
    t = scaling.table([json.loads(line(1, 9000.0)), json.loads(line(2, 18000.0)), json.loads(line(8, 68400.0))])
    assert "| 2 | 18000.0 images/sec | 9000.0 |" in t and "100.0 %" in t and "95.0 %" in t


def test_dry_run_returns_zero(capsys):
    assert scaling.main(["--dry-run", "--gpus", "1", "2"]) == 0
    err = capsys.readouterr().err
    assert err.count("$ ") == 2
