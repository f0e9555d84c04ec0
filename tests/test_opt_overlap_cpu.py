"""Per-bucket optimizer updates issued during backward (``Engine(opt_overlap=True)``,
``trainer/engine.py``) give the weights of the one-pass optimizer step after it.

On the CPU every update runs the moment its bucket completes, so a backward that
read a weight AFTER reporting its gradient ready would see the updated weight
here and the runs would diverge: the test also pins that ordering contract.
"""
import copy

import pytest
import torch

from kubeflow_controller_amd.trainer.engine import DistInfo, Engine


def _bert():
    from kubeflow_controller_amd.models.bert import BertConfig, BertForPreTraining, bert_loss, synthetic_mlm_batch
    cfg = BertConfig.tiny()
    torch.manual_seed(7)
    m = BertForPreTraining(cfg)
    batches = [synthetic_mlm_batch(cfg, 2, 16, generator=torch.Generator().manual_seed(i)) for i in range(3)]
    return m, bert_loss, batches, "adam"


def _resnet():
    from kubeflow_controller_amd.models.resnet import resnet_tiny
    from kubeflow_controller_amd.ops.loss import cross_entropy
    torch.manual_seed(7)
    m = resnet_tiny(10)
    g = torch.Generator().manual_seed(3)
    batches = [(torch.randn(2, 3, 32, 32, generator=g), torch.randint(0, 10, (2,), generator=g)) for _ in range(3)]
    return m, (lambda mm, x, y: cross_entropy(mm(x), y)), batches, "sgd"


@pytest.mark.parametrize("make", [_bert, _resnet], ids=["bert_adam", "resnet_sgd"])
def test_overlapped_optimizer_matches_one_pass(make):
    m, loss, batches, opt = make()
    engines = [Engine(copy.deepcopy(m), loss, optimizer=opt, lr=1e-3, compute_dtype=torch.bfloat16,
                      channels_last=False, bucket_mb=0.05, dist_info=DistInfo(), opt_overlap=ov)
               for ov in (False, True)]
    ref, ovl = engines
    assert ovl.opt_overlap and not ref.opt_overlap
    assert len(ovl.sync.buckets) > 3  # the step really is cut into several updates
    seen = []
    inner = ovl.opt.update
    ovl.opt.update = lambda si, a, b, *r: (seen.append((si, a, b)), inner(si, a, b, *r))[1]
    for b in batches:
        la, lb = ref.train_step(*b), ovl.train_step(*b)
        torch.testing.assert_close(lb, la, rtol=1e-5, atol=1e-6)
        # every bucket updated exactly once in its step
        assert sorted(seen) == sorted((k.group, k.start, k.end) for k in ovl.sync.buckets)
        seen.clear()
    assert ovl.opt.step_count == ref.opt.step_count == len(batches)
    for ga, gb in zip(ref.groups, ovl.groups):
        torch.testing.assert_close(gb.fp32, ga.fp32, rtol=1e-6, atol=1e-7)
    assert ovl.graph_ok() is not None  # eager-only


def test_opt_overlap_is_single_process_only():
    m, loss, _, opt = _bert()
    e = Engine(m, loss, optimizer=opt, channels_last=False, dist_info=DistInfo(), opt_overlap=None)
    assert not e.opt_overlap  # env default off (and CPU)


def test_tied_word_embedding_uses_survive_deepcopy():
    """The tied word embedding reports its gradient twice per backward (decoder +
    embedding); a deep-copied model must still expect both, or its bucket would
    complete after the first."""
    from kubeflow_controller_amd.models.bert import BertConfig, BertForPreTraining, bert_loss
    m = copy.deepcopy(BertForPreTraining(BertConfig.tiny()))
    e = Engine(m, bert_loss, optimizer="adam", channels_last=False, dist_info=DistInfo(), opt_overlap=True,
               bucket_mb=0.05)
    gi, pi = next((gi, pi) for gi, g in enumerate(e.groups) for pi, p in enumerate(g.params) if p is m.word_emb)
    assert max(b.total for b in e.sync._of_param[(gi, pi)]) >= 2


def test_direct_notification_counts_once():
    """A parameter whose gradient a HIP backward wrote directly (flat.notify_grad_ready,
    backward returns None) is reported once, although autograd's post-accumulate hook
    also fires for it."""
    from kubeflow_controller_amd.parallel.flat import notify_grad_ready, register_ready_hook
    w = torch.nn.Parameter(torch.ones(4))
    x = torch.nn.Parameter(torch.ones(4))
    seen = []
    for p in (w, x):
        register_ready_hook(p, lambda q: seen.append(q))

    class Direct(torch.autograd.Function):
        @staticmethod
        def forward(ctx, a, wt):
            return a * wt

        @staticmethod
        def backward(ctx, g):
            notify_grad_ready(w)
            return g, None
    for _ in range(2):
        seen.clear()
        Direct.apply(x, w).sum().backward()
        assert [id(q) for q in seen].count(id(w)) == 1 and [id(q) for q in seen].count(id(x)) == 1, seen


def test_bucket_overcount_raises():
    """A gradient reported ready more often than its bucket counts (an undeclared
    tied parameter delivered by two direct backwards) must not silently start the
    bucket's collective / update early: the second notification after completion
    raises."""
    import pytest
    from kubeflow_controller_amd.parallel import flat
    from kubeflow_controller_amd.parallel.ddp import GradSync
    model = torch.nn.Sequential(torch.nn.Linear(8, 8), torch.nn.Linear(8, 4))
    groups = flat.split_params(model, None)
    sync = GradSync(groups, bucket_mb=1.0)
    done = []
    sync.on_bucket_ready(done.append)
    p = groups[0].params[0]
    for g in groups:
        for q in g.params:
            flat.notify_grad_ready(q)
    assert len(done) == len(sync.buckets)
    with pytest.raises(RuntimeError, match="ready notifications"):
        flat.notify_grad_ready(p)
    assert sync.comm_wait_ms() is None  # world 1 / CPU: nothing timed
