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


def test_graph_refuses_adam():
    from kubeflow_controller_amd.models.resnet import ResNet
    from kubeflow_controller_amd.ops.loss import cross_entropy
    from kubeflow_controller_amd.trainer.engine import DistInfo, Engine
    eng = Engine(ResNet(layers=(1, 1, 1, 1), num_classes=10, width=64),
                 lambda m, x, y: cross_entropy(m(x), y), optimizer="adam", lr=1e-3,
                 dist_info=DistInfo(device=torch.device("cuda")))
    assert "Adam" in eng.graph_ok()
    with pytest.raises(RuntimeError):
        eng.capture(torch.zeros(1, device="cuda"))
