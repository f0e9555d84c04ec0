"""Data-parallel training on the HIP kernels (GradSync buckets fired from the direct-
gradient notifications) matches one process on the concatenated batch.

Two ranks share the box's one GPU over gloo (RCCL refuses two ranks on one device;
``KFA_COMM=torch``), so the bucket bookkeeping of the GPU path — HIP backwards that
write the flat gradient and notify — drives real all-reduces.  A bucket that fired
before its last gradient landed (the round-5 double count, ``docs/architecture.md``)
all-reduces a partial gradient and the ranks' weights leave the single-process ones.
SGD (linear in the gradient) keeps the comparison tight: the updates agree to the
bf16 rounding of the gradient buffer (each rank rounds its half-sum, one process the
whole sum), and the two ranks' weights agree exactly.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

B, S, STEPS = 4, 128, 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg():
    from kubeflow_controller_amd.models.bert import BertConfig
    return BertConfig(vocab_size=1024, hidden=256, layers=2, heads=4, intermediate=1024, max_position=128,
                      hidden_dropout=0.0, attn_dropout=0.0)


def _batch(cfg, r, d):
    from kubeflow_controller_amd.models.bert import synthetic_mlm_batch
    return synthetic_mlm_batch(cfg, B, S, torch.Generator().manual_seed(100 + r))


def _engine(model, d, info, ps=0):
    from kubeflow_controller_amd.models.bert import bert_loss
    from kubeflow_controller_amd.trainer.engine import Engine
    return Engine(model, bert_loss, optimizer="sgd", lr=0.1, momentum=0.0, weight_decay=0.0,
                  compute_dtype=torch.bfloat16, channels_last=False, bucket_mb=0.5, dist_info=info,
                  ps=ps, ps_placement="sharded")


def _to(batch, d):
    return tuple(t.to(d) if isinstance(t, torch.Tensor) else t for t in batch)


def _worker(rank, world, port, out, ps=0):
    import torch.distributed as dist
    from kubeflow_controller_amd.models.bert import BertForPreTraining
    from kubeflow_controller_amd.trainer.engine import DistInfo
    os.environ["KFA_COMM"] = "torch"
    d = torch.device("cuda", 0)
    torch.cuda.set_device(d)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    cfg = _cfg()
    torch.manual_seed(5)
    e = _engine(BertForPreTraining(cfg), d, DistInfo(rank=rank, world=world, device=d), ps)
    batch = _to(_batch(cfg, rank, d), d)
    for _ in range(STEPS):
        e.train_step(*batch)
    e.wait()
    torch.cuda.synchronize()
    torch.save([(g.data if ps else g.fp32).float().cpu() for g in e.groups], f"{out}.{rank}")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("ps", [0, 1], ids=["allreduce", "sharded_ps"])
def test_dp_two_ranks_match_single_process(tmp_path, ps):
    """ps=0: bucketed all-reduce (parallel/ddp.py), fp32 masters compared; ps=1: sharded
    owners — push, owner-side update, pull (parallel/ps.py).  The PS layouts keep the
    fp32 masters in the owners' compact shards (``ShardedGradSync.w32``) and pull the
    bf16 compute weights: those are compared, to one bf16 rounding."""
    from kubeflow_controller_amd.models.bert import BertForPreTraining
    from kubeflow_controller_amd.trainer.engine import DistInfo
    out = str(tmp_path / "w")
    mp.start_processes(_worker, args=(2, _free_port(), out, ps), nprocs=2, join=True, start_method="spawn")
    d = torch.device("cuda", 0)
    cfg = _cfg()
    torch.manual_seed(5)
    e = _engine(BertForPreTraining(cfg), d, DistInfo(device=d))
    init = [(g.data if ps else g.fp32).float().cpu().clone() for g in e.groups]
    parts = [_batch(cfg, r, d) for r in range(2)]
    ids, tt, _, flat, labels, nsp = (list(x) for x in zip(*parts))
    flat = [f + r * B * S for r, f in enumerate(flat)]  # positions index the concatenated [B*S] rows
    batch = _to((torch.cat(ids), torch.cat(tt), None, torch.cat(flat), torch.cat(labels), torch.cat(nsp)), d)
    for _ in range(STEPS):
        e.train_step(*batch)
    torch.cuda.synchronize()
    ref = [(g.data if ps else g.fp32).float().cpu() for g in e.groups]
    w0, w1 = (torch.load(f"{out}.{r}", weights_only=True) for r in range(2))
    for a, b in zip(w0, w1):  # every rank applied the same summed update
        torch.testing.assert_close(a, b, rtol=0, atol=0)
    for a, r, i in zip(w0, ref, init):
        n = r.numel()  # world 2 pads each group to a multiple of 16 elements (reduce-scatter shards)
        da, dr = a[:n] - i, r - i
        tol = 2e-2 * dr.abs() + 1e-2 * float(dr.abs().max()) + (2 ** -7 * r.abs() if ps else 0.0)
        assert bool(((da - dr).abs() <= tol).all()), float((da - dr).abs().max())


def _resnet_worker(rank, world, port, out):
    """ResNet (HIP conv / BN / wgrad backwards that write the flat gradient and notify):
    the model the driver's multi-GPU bench runs through these same bucket hooks."""
    import torch.distributed as dist
    from kubeflow_controller_amd.models.resnet import ResNet
    from kubeflow_controller_amd.ops.loss import cross_entropy
    from kubeflow_controller_amd.trainer.engine import DistInfo, Engine
    os.environ["KFA_COMM"] = "torch"
    d = torch.device("cuda", 0)
    torch.cuda.set_device(d)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    torch.manual_seed(5)
    e = Engine(ResNet(layers=(1, 1, 1, 1), num_classes=10, width=64), lambda m, x, y: cross_entropy(m(x), y),
               optimizer="sgd", lr=0.05, momentum=0.9, weight_decay=0.0, bucket_mb=0.25,
               dist_info=DistInfo(rank=rank, world=world, device=d))
    assert len(e.sync.buckets) > 4, len(e.sync.buckets)
    g = torch.Generator().manual_seed(200 + rank)
    x = torch.randn(8, 3, 64, 64, generator=g).to(d, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), generator=g).to(d)
    fired = []
    for _ in range(STEPS):
        e.train_step(x, y)
        fired.append(e.sync.comm_wait_ms() is not None)
    torch.cuda.synchronize()
    torch.save([gr.fp32.float().cpu() for gr in e.groups], f"{out}.{rank}")
    dist.barrier()
    dist.destroy_process_group()
    assert all(fired)


def test_dp_resnet_ranks_stay_identical(tmp_path):
    """Two ranks with different batches (per-rank BatchNorm statistics, so no
    single-process reference): every rank must apply the SAME summed update.  A
    bucket all-reduced before its last HIP-written gradient landed, or a gradient
    counted twice (GradSync raises on a negative pending count), makes the ranks'
    fp32 masters differ."""
    out = str(tmp_path / "w")
    mp.start_processes(_resnet_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    w0, w1 = (torch.load(f"{out}.{r}", weights_only=True) for r in range(2))
    for a, b in zip(w0, w1):
        torch.testing.assert_close(a, b, rtol=0, atol=0)
