"""Whole-step HIP graph replay (Engine.capture) vs the eager step it records."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _engine(model):
    from kubeflow_controller_amd.ops.loss import cross_entropy
    from kubeflow_controller_amd.trainer.engine import DistInfo, Engine
    return Engine(model, lambda m, x, y: cross_entropy(m(x), y), optimizer="sgd", lr=0.05,
                  dist_info=DistInfo(device=torch.device("cuda")))


def test_graph_replay_matches_eager_steps():
    """4 executed steps either way (graph engine: 1 eager + capture's side-stream
    warm-up step + 2 replays); the fp32 masters must agree to BN-atomics noise,
    and the replayed loss must be refreshed on every replay."""
    from kubeflow_controller_amd.models.resnet import ResNet
    from kubeflow_controller_amd.ops import _lib
    _lib.lib()
    torch.manual_seed(0)
    base = ResNet(layers=(1, 1, 1, 1), num_classes=10, width=64)
    ea, eg = _engine(copy.deepcopy(base)), _engine(copy.deepcopy(base))
    d = torch.device("cuda")
    x = torch.randn(8, 3, 64, 64, device=d, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device=d)
    eager = [float(ea.train_step(x, y)) for _ in range(4)]

    assert eg.graph_ok() is not None  # no eager step yet
    l0 = float(eg.train_step(x, y))
    assert eg.graph_ok() is None
    eg.capture(x, y)
    l2 = float(eg.train_step(x, y))
    l3 = float(eg.train_step(x, y))
    torch.cuda.synchronize()
    assert eg.steps == ea.steps and eg.opt.step_count == ea.opt.step_count
    assert abs(l0 - eager[0]) < 1e-3 * max(1.0, abs(eager[0]))
    assert l2 != l3, "replayed loss buffer not refreshed"
    assert abs(l3 - eager[3]) < 2e-2 * max(1.0, abs(eager[3])), (eager, [l0, l2, l3])
    for ga, gg in zip(ea.groups, eg.groups):
        torch.testing.assert_close(gg.master, ga.master, atol=2e-3, rtol=2e-2)


def test_graph_replay_copies_new_batch():
    """A batch passed in new tensors is copied into the captured inputs: replaying
    on batch B must give B's loss, not the captured batch A's."""
    from kubeflow_controller_amd.models.resnet import ResNet
    torch.manual_seed(1)
    base = ResNet(layers=(1, 1, 1, 1), num_classes=10, width=64)
    eg = _engine(copy.deepcopy(base))
    d = torch.device("cuda")
    xa = torch.randn(8, 3, 64, 64, device=d, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ya = torch.randint(0, 10, (8,), device=d)
    eg.train_step(xa, ya)
    eg.capture(xa.clone(), ya.clone())
    xb = (xa * 3.0).contiguous(memory_format=torch.channels_last)
    yb = (ya + 1) % 10
    lb = float(eg.train_step(xb, yb))
    static_x, static_y = eg._graph[1]
    assert torch.equal(static_x, xb) and torch.equal(static_y, yb)
    la = float(eg.train_step(xa, ya))
    assert lb == lb and la == la and lb != la


def test_graph_adam_mlp_matches_eager():
    """Adam's step count / bias corrections advance on the device (kfa_adam_bc), so a
    replayed Adam step matches the eager ones (the reference's MNIST MLP, Adam)."""
    from kubeflow_controller_amd.models.mnist import MnistMLP
    from kubeflow_controller_amd.ops.loss import cross_entropy
    from kubeflow_controller_amd.trainer.engine import DistInfo, Engine
    torch.manual_seed(2)
    base = MnistMLP(100)
    d = torch.device("cuda")

    def mk():
        return Engine(copy.deepcopy(base), lambda m, x, y: cross_entropy(m(x).float(), y), optimizer="adam",
                      lr=0.01, weight_decay=0.0, compute_dtype=None, channels_last=False,
                      dist_info=DistInfo(device=d))
    ea, eg = mk(), mk()
    xs = [torch.rand(100, 784, device=d) for _ in range(6)]
    ys = [torch.randint(0, 10, (100,), device=d) for _ in range(6)]
    la = [float(ea.train_step(x, y)) for x, y in zip(xs, ys)]
    lg = [float(eg.train_step(xs[0], ys[0]))]
    lg.append(float(eg.capture(xs[1].clone(), ys[1].clone())))
    lg += [float(eg.train_step(x, y)) for x, y in zip(xs[2:], ys[2:])]
    torch.cuda.synchronize()
    assert eg.opt.step_count == ea.opt.step_count == 6
    assert int(eg.opt._t.item()) == 6
    for a, g in zip(la, lg):
        assert abs(a - g) < 1e-4 * max(1.0, abs(a)), (la, lg)
    for ga, gg in zip(ea.groups, eg.groups):
        torch.testing.assert_close(gg.master, ga.master, atol=1e-5, rtol=1e-4)


def test_graph_refuses_dropout_model():
    from kubeflow_controller_amd.models.bert import BertConfig, BertForPreTraining
    from kubeflow_controller_amd.trainer.engine import DistInfo, Engine
    cfg = BertConfig(vocab_size=1024, hidden=128, layers=1, heads=2, intermediate=512, max_position=128)
    m = BertForPreTraining(cfg)
    eng = Engine(m, lambda mm, *b: mm(*b), optimizer="adam", lr=1e-4, channels_last=False,
                 dist_info=DistInfo(device=torch.device("cuda")))
    eng.opt.step_count = 1
    assert "dropout" in eng.graph_ok()
    m.eval()
    assert eng.graph_ok() is None


def test_replica_local_mnist_softmax_graph(tmp_path):
    """The reference's local MNIST job (C20) through the replica runtime with the step
    replayed as a HIP graph: trains, and reports the same accuracy as eager."""
    import subprocess
    import sys
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = {}
    for g in ("off", "on"):
        r = subprocess.run([sys.executable, "-m", "kubeflow_controller_amd.trainer.replica", "--model", "mnist_softmax",
                            "--optimizer", "sgd", "--learning_rate", "0.5", "--train_steps", "300",
                            "--log_every", "100", "--graph", g], cwd=root, capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        acc = [l for l in r.stdout.splitlines() + r.stderr.splitlines() if "Test accuracy" in l]
        assert acc, r.stdout[-2000:]
        out[g] = float(acc[-1].split()[-1])
        if g == "on":
            assert "captured as a HIP graph" in r.stdout + r.stderr
    assert out["on"] > 0.5 and abs(out["on"] - out["off"]) < 0.02, out
