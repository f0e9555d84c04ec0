"""1-GPU rehearsal of the parameter-server modes of trainer/replica.py on
BERT-base (2 workers + 1 PS, every process on the one GPU):

* async, device transport: PS variables / Adam state / gradient mailboxes in HBM,
  pull / push as one device copy per PS run (HIP IPC), headers over gloo;
* async, host transport: the same protocol with the payloads over gloo;
* collective sync replicas (--ps_mode collective, gloo on the one GPU: RCCL
  refuses two ranks on one device), the Engine's reduce-scatter / owner-apply /
  all-gather path.

Each worker reports its steady-state examples/s; the table sums them.  The
processes share ONE GPU, so this measures the protocol's overhead relative to
the compute, not multi-GPU throughput.

    python tools/async_rehearsal.py [--steps 40] [--batch 32]
"""
import argparse
import os
import re
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run(mode, transport, steps, batch, seq, model, timeout):
    wh = f"127.0.0.1:{_port()},127.0.0.1:{_port()}"
    ph = f"127.0.0.1:{_port()}"
    env = dict(os.environ, HIP_VISIBLE_DEVICES="0", PYTHONPATH=ROOT, OMP_NUM_THREADS="4")
    if mode == "collective":
        env["KFA_DIST_BACKEND"] = "gloo"
    base = [sys.executable, "-u", "-m", "kubeflow_controller_amd.trainer.replica", "--model", model,
            "--train_steps", str(steps), "--batch_size", str(batch), "--seq_len", str(seq), "--ps_mode", mode,
            "--learning_rate", "0.0001", "--log_every", "0", "--worker_hosts=" + wh, "--ps_hosts=" + ph]
    if mode == "async":
        base += ["--ps_transport", transport]
    else:
        base += ["--sync_replicas", "--graph", "off"]
    procs, logs = [], []
    for job, idx in (("ps", 0), ("worker", 0), ("worker", 1)):
        f = open(os.path.join(ROOT, "gpurun_out", f"rehearsal_{mode}_{transport}_{job}{idx}.log"), "w+")
        logs.append(f)
        procs.append(subprocess.Popen(base + [f"--job_name={job}", f"--task_index={idx}"], env=env, stdout=f,
                                      stderr=subprocess.STDOUT, text=True))
    t0 = time.time()
    try:
        for p in procs[1:] + procs[:1]:
            p.wait(timeout=max(1.0, timeout - (time.time() - t0)))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    outs = []
    for f in logs:
        f.seek(0)
        outs.append(f.read())
        f.close()
    if any(p.returncode != 0 for p in procs):
        print("\n-----\n".join(o[-2000:] for o in outs), file=sys.stderr)
        raise SystemExit(f"{mode}/{transport}: a replica failed")
    eps = [float(m.group(1)) for o in outs[1:] for m in re.finditer(r"Steady-state: .*?, ([\d.]+) examples/s", o)]
    for o in outs[1:2]:  # worker 0's transport line (device / host per PS, and why)
        for line in o.splitlines():
            if "transport" in line:
                print(f"    worker 0: {line.strip()[:200]}", file=sys.stderr, flush=True)
                break
    return sum(eps), eps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--model", default="bert_base")
    ap.add_argument("--timeout", type=float, default=240)
    ap.add_argument("--modes", default="async:device,async:host,collective:-",
                    help="comma list of mode:transport to run")
    a = ap.parse_args()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    print(f"| mode ({a.model}, 2 workers + 1 PS on 1 GPU, batch {a.batch}/worker, seq {a.seq}) | "
          f"examples/s (sum) | per worker |", flush=True)
    print("|---|---|---|", flush=True)
    for mode, tr in (m.split(":") for m in a.modes.split(",")):
        tot, per = run(mode, tr, a.steps, a.batch, a.seq, a.model, a.timeout)
        print(f"| {mode} {tr} | {tot:.1f} | {', '.join(f'{x:.1f}' for x in per)} |", flush=True)


if __name__ == "__main__":
    main()
