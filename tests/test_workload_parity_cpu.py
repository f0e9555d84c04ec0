"""Reference-workload parity on CPU: the summed clipped cross-entropy of
``mnist_replica.py:167-168``, the dropout launch keys (seed mixing) and the
replica's flag semantics for ``--replicas_to_aggregate`` without ``--sync_replicas``
(``mnist_replica.py:172-176`` reads it only under sync)."""
import numpy as np
import pytest
import torch

from kubeflow_controller_amd.ops.loss import clipped_sum_cross_entropy
from kubeflow_controller_amd.ops.transformer import hash_key


def _tf_reference(z, y, eps=1e-10):
    """-reduce_sum(y_ * log(clip_by_value(softmax(z), eps, 1))) with one-hot y_ (float64)."""
    z = z.double().detach().requires_grad_()
    p = torch.softmax(z, -1)
    onehot = torch.nn.functional.one_hot(y, z.shape[-1]).double()
    loss = -(onehot * torch.log(torch.clamp(p, eps, 1.0))).sum()
    loss.backward()
    return loss.detach(), z.grad


def test_clipped_sum_cross_entropy_matches_tf_semantics():
    torch.manual_seed(0)
    z = torch.randn(100, 10) * 3
    z[3, :] = torch.tensor([60.0, -60.0] + [0.0] * 8)  # label 1 below the clip: capped loss, zero gradient
    y = torch.randint(0, 10, (100,))
    y[3] = 1
    zz = z.clone().requires_grad_()
    loss = clipped_sum_cross_entropy(zz, y)
    loss.backward()
    ref, gref = _tf_reference(z, y)
    assert abs(float(loss.detach()) - float(ref)) < 1e-3 * float(ref)
    torch.testing.assert_close(zz.grad.double(), gref, atol=1e-5, rtol=1e-4)
    assert float(zz.grad[3].abs().sum()) == 0.0
    assert abs(float(-torch.log(torch.tensor(1e-10)))) > 23


def _drop_hash(key, i):
    """numpy copy of drop_hash (csrc/kernels/common.h)."""
    k0, k1 = np.uint32(key & 0xFFFFFFFF), np.uint32(key >> 32)
    with np.errstate(over="ignore"):
        x = (i.astype(np.uint32) ^ k0) + k1
        x ^= x >> np.uint32(16)
        x *= np.uint32(0x7FEB352D)
        x ^= x >> np.uint32(15)
        x *= np.uint32(0x846CA68B)
        x ^= x >> np.uint32(16)
    return x


@pytest.mark.parametrize("seed", [0, 1, 12345, 2**40])
def test_dropout_keys_of_neighbouring_seeds_are_uncorrelated(seed):
    """The kernels fold their key into the index linearly, so raw seeds s and s^1
    give index-permuted copies of one mask; the launch keys (hash_key) do not."""
    n, p = 1 << 16, 0.1
    i = np.arange(n, dtype=np.uint64)
    thr = np.uint32(int(p * 2**32))
    raw_a = _drop_hash(seed, i) >= thr
    raw_b = _drop_hash(seed ^ 1, i ^ np.uint64(1)) >= thr
    assert (raw_a == raw_b).all()  # the raw-seed defect this guards against
    a = _drop_hash(hash_key(seed), i) >= thr
    b = _drop_hash(hash_key(seed + 1), i) >= thr
    both_drop = float(np.mean(~a & ~b))
    assert abs(both_drop - p * p) < 0.004, both_drop  # independent masks: P(both dropped) = p^2
    assert hash_key(seed) != hash_key(seed + 1)


def test_replicas_to_aggregate_ignored_without_sync(monkeypatch):
    """An async-style command line that passes --replicas_to_aggregate still runs
    on the collective path (no error), as in the reference."""
    from kubeflow_controller_amd.trainer import replica
    from kubeflow_controller_amd.trainer.cluster import parse_cluster
    args = replica.build_parser().parse_args(
        ["--worker_hosts=127.0.0.1:1,127.0.0.1:2", "--job_name=worker", "--task_index=0",
         "--replicas_to_aggregate", "1", "--model", "mnist_mlp"])
    spec = parse_cluster(args)
    assert replica._aggregate(spec, args) == 0
    assert replica._async_mode(spec, args) is False
    called = {}

    def fake_init(*a, **k):
        called["timeout"] = k.get("timeout")
        raise SystemExit("stop here")

    monkeypatch.setattr(replica, "_store", lambda *a, **k: None)
    monkeypatch.setattr(replica.dist, "init_process_group", fake_init)
    args.device = "cpu"
    with pytest.raises(SystemExit, match="stop here"):
        replica.run_worker(spec, args)
    assert called["timeout"].total_seconds() == args.dist_timeout
