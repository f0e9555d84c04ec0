"""Which parameters differ after ONE step with the overlapped optimizer (Engine(opt_overlap=True))
vs the one-pass step, with the updates on the side stream and on the main stream, plus the
bucket completion order (param that completed each bucket)."""
import copy
import os
import sys

import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.models.bert import BertConfig, BertForPreTraining, bert_loss, synthetic_mlm_batch  # noqa
from kubeflow_controller_amd.trainer.engine import DistInfo, Engine  # noqa

d = torch.device("cuda")
cfg = BertConfig(vocab_size=1024, hidden=256, layers=2, heads=4, intermediate=1024, max_position=128)
torch.manual_seed(11)
base = BertForPreTraining(cfg)
batch = tuple(t.to(d) if isinstance(t, torch.Tensor) else t
              for t in synthetic_mlm_batch(cfg, 8, 128, generator=torch.Generator().manual_seed(0)))
names = {id(p): n for n, p in base.named_parameters()}


def mk(ov):
    m = copy.deepcopy(base)
    e = Engine(m, bert_loss, optimizer="adam", lr=1e-3, compute_dtype=torch.bfloat16, channels_last=False,
               bucket_mb=0.5, dist_info=DistInfo(device=d), opt_overlap=ov)
    return m, e


mr, ref = mk(False)
ref.train_step(*batch)
pn = {n: p for n, p in mr.named_parameters()}
for mode in ("side", "main"):
    mo, ovl = mk(True)
    on = {id(p): n for n, p in mo.named_parameters()}
    order = []
    if mode == "main":
        def upd(b, e=ovl):
            if not e._opt_open:
                e.opt.begin_step()
                e._opt_open = True
            e.opt.update(b.group, b.start, b.end)
        ovl.sync._on_ready = lambda b: (order.append(b.index), upd(b))
    else:
        inner = ovl.sync._on_ready
        ovl.sync._on_ready = lambda b: (order.append(b.index), inner(b))
    ovl.train_step(*batch)
    torch.cuda.synchronize()
    print(f"[{mode}] bucket completion order: {order}")
    for b in ovl.sync.buckets:
        ps = [on.get(id(ovl.groups[b.group].params[i]), "?") for i in b.params] if isinstance(b.params[0], int) \
            else [on.get(id(p), "?") for p in b.params]
        print(f"  bucket {b.index} (group {b.group}, [{b.start}, {b.end}), total {b.total}): {ps[:4]}{' ...' if len(ps) > 4 else ''}")
    bad = []
    for n, p in mo.named_parameters():
        dd = float((p.detach().float() - pn[n].detach().float()).abs().max())
        if dd > 0:
            bad.append((dd, n))
    print(f"[{mode}] params that differ after one step: {len(bad)}")
    for dd, n in sorted(bad, reverse=True)[:20]:
        print(f"   {dd:.3e}  {n}")
