"""Count, per parameter, the gradient-ready notifications one backward delivers to the
bucket bookkeeping (parallel/ddp.py): direct ones (flat.notify_grad_ready from a HIP
backward) and autograd's post-accumulate hooks.  Every parameter must report exactly
its `_kfa_uses` once per backward, else its bucket completes early or never."""
import collections
import os
import sys

import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.parallel import flat  # noqa: E402
from kubeflow_controller_amd.trainer.engine import DistInfo, Engine  # noqa: E402


def count(model, loss, batch, **kw):
    e = Engine(model, loss, dist_info=DistInfo(device=torch.device("cuda")), channels_last=False, opt_overlap=True, **kw)
    names = {id(p): n for n, p in model.named_parameters()}
    direct, acc = collections.Counter(), collections.Counter()
    for n, p in model.named_parameters():
        cb = flat._READY_CB.get(id(p))
        if cb is not None:
            flat._READY_CB[id(p)] = (lambda cb, n: (lambda q: (direct.update([n]), cb(q))))(cb, n)
        p.register_post_accumulate_grad_hook((lambda n: (lambda q: acc.update([n])))(n))
    e.train_step(*batch)
    torch.cuda.synchronize()
    bad = []
    for n, p in model.named_parameters():
        want = int(getattr(p, "_kfa_uses", 1))
        if direct[n] + acc[n] != want:
            bad.append((n, direct[n], acc[n], want))
    return bad, names


if __name__ == "__main__":
    from kubeflow_controller_amd.models.bert import BertConfig, BertForPreTraining, bert_loss, synthetic_mlm_batch
    d = torch.device("cuda")
    cfg = BertConfig(vocab_size=1024, hidden=256, layers=2, heads=4, intermediate=1024, max_position=128)
    torch.manual_seed(11)
    m = BertForPreTraining(cfg)
    batch = tuple(t.to(d) if isinstance(t, torch.Tensor) else t
                  for t in synthetic_mlm_batch(cfg, 8, 128, generator=torch.Generator().manual_seed(0)))
    bad, _ = count(m, bert_loss, batch, optimizer="adam", compute_dtype=torch.bfloat16, bucket_mb=0.5)
    print("BERT params with a wrong ready count (name, direct, autograd, expected):")
    for b in bad:
        print("  ", b)
    from kubeflow_controller_amd.models.resnet import resnet_tiny
    from kubeflow_controller_amd.ops.loss import cross_entropy
    torch.manual_seed(1)
    r = resnet_tiny(10)
    x = torch.randn(4, 3, 32, 32, device=d)
    y = torch.randint(0, 10, (4,), device=d)
    bad, _ = count(r, lambda mm, a, b: cross_entropy(mm(a), b), (x, y), optimizer="sgd", compute_dtype=torch.bfloat16,
                   bucket_mb=0.05)
    print("ResNet params with a wrong ready count (name, direct, autograd, expected):")
    for b in bad:
        print("  ", b)
