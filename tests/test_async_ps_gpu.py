"""Device-resident async parameter server (parallel/async_ps.py, HIP IPC):
PS variables / Adam state / gradient mailboxes in GPU memory, pulls and pushes
as device-to-device copies, only headers over gloo.  Runs every process on the
one GPU of the box (IPC within a device works like across xGMI peers)."""
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _proc(rank, W, P, port, out, opt, agg, sig="1", nsteps=5):
    sys.path.insert(0, ROOT)
    os.environ["KFA_PS_DEVICE_SIGNAL"] = sig
    import datetime

    import torch.distributed as dist
    from kubeflow_controller_amd.parallel.async_ps import DeviceAsyncPSClient, DeviceAsyncPSServer
    torch.cuda.set_device(0)
    store = dist.TCPStore("127.0.0.1", port, W + P, rank == 0, timeout=datetime.timedelta(seconds=120))
    dist.init_process_group("gloo", store=store, rank=rank, world_size=W + P)
    m = torch.nn.Sequential(torch.nn.Linear(300, 20), torch.nn.Linear(20, 4))
    for p in m.parameters():
        torch.nn.init.constant_(p, 0.5)
    if rank >= W:
        s = DeviceAsyncPSServer(list(m.named_parameters()), W, P, rank - W, store, torch.device("cuda", 0), lr=0.25,
                                optimizer=opt, aggregate=agg)
        pushes = s.serve()
        torch.save({"vars": {k: v.cpu() for k, v in s.variables().items()}, "names": s.names, "pushes": pushes,
                    "step": s.global_step}, f"{out}.ps{rank - W}")
    else:
        m = m.cuda()
        c = DeviceAsyncPSClient(list(m.named_parameters()), W, P, rank, store)
        steps = []
        for _ in range(nsteps):
            c.pull()
            c.zero_grad()
            for p in m.parameters():   # the grads are views of the client's flat buffers
                p.grad.fill_(1.0 if opt == "adam" else float(rank + 1))
            steps.append(c.push())
        c.pull()
        final = {n: p.detach().cpu().clone() for n, p in m.named_parameters()}
        c.done()
        torch.save({"steps": steps, "final": final, "transports": c.transports}, f"{out}.w{rank}")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("sig", ["1", "0"], ids=["device_signal", "host_waits"])
@pytest.mark.parametrize("opt,agg,nsteps", [("sgd", 0, 5), ("adam", 0, 5), ("adam", 2, 5), ("sgd", 0, 40)],
                         ids=["sgd", "adam", "adam_agg2", "sgd_long"])
def test_device_async_ps_matches_host_server(tmp_path, opt, agg, sig, nsteps):
    """Every push applied once (async) or every 2 averaged (sync replicas), the
    variables equal the host PS's TF-form update on the same gradients (Adam:
    fused HIP kernel vs AsyncPSServer._apply in fp32), and every client mapped
    the PS memory (canary check passed: device transport, no host fallback).
    ``sgd_long``: 80 updates per PS, so the device-signalling event chains roll
    over five generations (ROCm's interprocess events fail after 31 records)."""
    from kubeflow_controller_amd.parallel.async_ps import AsyncPSServer
    W, P = 2, 2
    out = str(tmp_path / "dps")
    mp.start_processes(_proc, args=(W, P, _free_port(), out, opt, agg, sig, nsteps), nprocs=W + P, join=True,
                       start_method="spawn")
    names = ["0.weight", "0.bias", "1.weight", "1.bias"]
    updates = nsteps if agg else nsteps * W
    for k in range(P):
        ps = torch.load(f"{out}.ps{k}", weights_only=True)
        assert sorted(ps["names"]) == sorted(names[k::P]) and ps["pushes"] == nsteps * W and ps["step"] == updates
        for n, v in ps["vars"].items():
            if opt == "sgd":
                want = torch.full_like(v, 0.5 - 0.25 * nsteps * sum(range(1, W + 1)))
            else:  # constant gradient 1: the same update sequence whatever the arrival order
                ref = AsyncPSServer([(n, torch.full((v.numel(),), 0.5))], 1, 1, 0, lr=0.25, optimizer="adam")
                for _ in range(updates):
                    ref._apply(torch.ones(v.numel()))
                want = ref.w
            torch.testing.assert_close(v, want, rtol=1e-5, atol=1e-5)
    for w in range(W):
        got = torch.load(f"{out}.w{w}", weights_only=True)
        assert got["transports"] == ["device"] * P
        if opt == "sgd":
            for n, t in got["final"].items():   # the last pull (after every push) sees the final PS values
                assert t.min().item() >= 0.5 - 0.25 * nsteps * sum(range(1, W + 1)) - 1e-5
    steps = sorted(s for w in range(W) for s in torch.load(f"{out}.w{w}", weights_only=True)["steps"])
    if agg:
        assert steps == sorted(list(range(1, nsteps + 1)) * W)
    else:
        assert steps == list(range(1, nsteps * W + 1))


def test_replica_async_bert_tiny_device_transport(tmp_path):
    """trainer/replica.py --ps_mode async with a GPU PS: bert_tiny, 2 workers + 1 PS."""
    port = _free_port()
    wh = f"127.0.0.1:{port},127.0.0.1:{_free_port()}"
    ph = f"127.0.0.1:{_free_port()}"
    env = dict(os.environ, HIP_VISIBLE_DEVICES="0", PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    base = [sys.executable, "-m", "kubeflow_controller_amd.trainer.replica", "--model", "bert_tiny", "--train_steps",
            "8", "--batch_size", "8", "--seq_len", "64", "--ps_mode", "async", "--ps_transport", "device",
            "--learning_rate", "0.002", "--worker_hosts=" + wh, "--ps_hosts=" + ph]
    logs = [open(tmp_path / f"r{i}.log", "w+") for i in range(3)]
    procs = [subprocess.Popen(base + ["--job_name=ps", "--task_index=0"], env=env, stdout=logs[0],
                              stderr=subprocess.STDOUT, text=True)]
    for i in range(2):
        procs.append(subprocess.Popen(base + ["--job_name=worker", f"--task_index={i}"], env=env,
                                      stdout=logs[i + 1], stderr=subprocess.STDOUT, text=True))
    try:
        for p in procs[1:] + procs[:1]:
            p.wait(timeout=100)
    except subprocess.TimeoutExpired:
        pass
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    outs = [(tmp_path / f"r{i}.log").read_text() for i in range(3)]
    assert all(p.returncode == 0 for p in procs), "\n-----\n".join(o[-3000:] for o in outs)
    assert "device-resident" in outs[0] and "GPU HBM" in outs[0]
    assert "device transport" in outs[1] and "Final loss" in outs[1]
