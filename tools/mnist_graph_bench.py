"""The reference's local MNIST softmax job (784->10, GD lr 0.5,
batch 100; ``examples/workdir/mnist_softmax.py``) on one GPU through the replica
runtime, eager vs the step replayed as a HIP graph — steps/s and accuracy.

    python tools/mnist_graph_bench.py [--steps 20000]
"""
import argparse
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(graph: str, steps: int, model: str, opt: str, lr: str):
    cmd = [sys.executable, "-m", "kubeflow_controller_amd.trainer.replica", "--model", model, "--optimizer", opt,
           "--learning_rate", lr, "--batch_size", "100", "--train_steps", str(steps),
           "--log_every", str(steps // 4), "--graph", graph]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=900)
    text = r.stdout + r.stderr
    if r.returncode != 0:
        raise SystemExit(text[-3000:])
    el = float(re.search(r"Training elapsed time: ([0-9.]+)", text).group(1))
    sps = float(re.search(r"Steady-state: ([0-9.]+) steps/s", text).group(1))
    acc = re.search(r"Test accuracy: ([0-9.]+)", text)
    return el, sps, float(acc.group(1)) if acc else float("nan")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20000)
    a = ap.parse_args()
    for model, opt, lr in (("mnist_softmax", "sgd", "0.5"), ("mnist_mlp", "adam", "0.01")):
        for g in ("off", "on"):
            el, sps, acc = run(g, a.steps, model, opt, lr)
            print(f"{model:14s} {opt:4s} graph={g:3s}: {a.steps} steps in {el:.2f} s, steady state {sps:,.0f} steps/s "
                  f"({sps * 100:,.0f} examples/s), test accuracy {acc:.4f}", flush=True)


if __name__ == "__main__":
    main()
