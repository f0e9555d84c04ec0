"""Wide&Deep input assembly kernels (csrc/kernels/widedeep.hip) vs the PyTorch ops they replace."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,F,E,Dp", [(1000, 26, 64, 16), (37, 3, 16, 8), (4096, 8, 32, 24)])
def test_wd_input_fwd_bwd_matches_torch(B, F, E, Dp):
    from kubeflow_controller_amd.models.wide_deep import _WDInputFn
    torch.manual_seed(0)
    d = torch.device("cuda")
    rows = torch.randn(B * F, E + 8, device=d).to(torch.bfloat16).requires_grad_()
    dense = torch.randn(B, Dp, device=d)
    x, wide = _WDInputFn.apply(rows, dense, B, F, E)
    r = rows.detach().float().view(B, F, E + 8).requires_grad_()
    xr = torch.cat([dense.to(torch.bfloat16).float(), r[:, :, :E].reshape(B, F * E)], 1)
    wr = r[:, :, E].sum(1)
    assert torch.equal(x.float(), xr)
    torch.testing.assert_close(wide, wr, atol=1e-4, rtol=1e-5)
    gx = torch.randn_like(xr).to(torch.bfloat16)
    gw = torch.randn(B, device=d)
    (x.float() * gx.float()).sum().add_((wide * gw).sum()).backward()
    (xr * gx.float()).sum().add_((wr * gw).sum()).backward()
    ref = r.grad.view(B * F, E + 8).to(torch.bfloat16)
    assert torch.equal(rows.grad, ref)


def test_wide_deep_step_fused_input_matches_unfused(monkeypatch):
    """Same tiny W&D training steps with the fused input / head kernels and with the PyTorch chain."""
    import copy
    from kubeflow_controller_amd.models import wide_deep as WD
    from kubeflow_controller_amd.trainer.engine import DistInfo, Engine
    d = torch.device("cuda")
    cfg = WD.WideDeepConfig.tiny()
    torch.manual_seed(0)
    base = WD.WideDeep(cfg, device=d)
    g = torch.Generator().manual_seed(1)
    batch = WD.prepare_batch(base, *WD.synthetic_batch(cfg, 512, g, "cpu"), d)
    losses = {}
    for fused in (True, False):
        monkeypatch.setattr(WD, "FUSED_INPUT", fused)
        monkeypatch.setattr(WD, "FUSED_HEAD", fused)
        eng = Engine(copy.deepcopy(base), WD.wide_deep_loss, optimizer="adam", lr=1e-2, channels_last=False,
                     dist_info=DistInfo(device=d))
        losses[fused] = [float(eng.train_step(*batch)) for _ in range(4)]
    for a, b in zip(losses[True], losses[False]):
        assert abs(a - b) < 2e-3 * max(1.0, abs(b)), losses


@pytest.mark.parametrize("B,H,Dp", [(65536, 256, 16), (1000, 32, 8), (37, 512, 64), (8, 256, 0)])
def test_wd_head_matches_fp32_reference(B, H, Dp):
    """Fused output head + sigmoid cross-entropy (kfa_wd_head_fwd / _bwd) vs the plain
    fp32 PyTorch chain it replaces: loss and every gradient."""
    from kubeflow_controller_amd.models.wide_deep import _WDHeadFn
    import torch.nn.functional as F
    torch.manual_seed(B + H)
    d = torch.device("cuda")
    x = (torch.randn(B, H, device=d) * 0.5).to(torch.bfloat16).requires_grad_()
    w = (torch.randn(1, H, device=d) * H ** -0.5).requires_grad_()
    b = torch.randn(1, device=d).requires_grad_()
    wide = torch.randn(B, device=d).requires_grad_()
    dpad = torch.randn(B, Dp, device=d)
    wd = (torch.randn(1, Dp, device=d) * 0.1).requires_grad_()
    y = (torch.rand(B, device=d) < 0.3).float()
    loss = _WDHeadFn.apply(x, w, b, wide, dpad, wd, y)
    (loss * 3.0).backward()
    xr = x.detach().float().requires_grad_()
    wr, br, wider, wdr = (t.detach().clone().requires_grad_() for t in (w, b, wide, wd))
    z = (xr @ wr.t()).squeeze(1) + br + wider + (dpad @ wdr.t()).squeeze(1)
    ref = F.binary_cross_entropy_with_logits(z, y)
    (ref * 3.0).backward()
    torch.testing.assert_close(loss, ref, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=1e-6, rtol=1e-2)
    torch.testing.assert_close(w.grad, wr.grad, atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(b.grad, br.grad, atol=1e-6, rtol=1e-4)
    torch.testing.assert_close(wide.grad, wider.grad, atol=1e-7, rtol=1e-5)
    if Dp:
        torch.testing.assert_close(wd.grad, wdr.grad, atol=1e-5, rtol=1e-4)
    # deterministic: a second run gives bit-identical loss and gradients
    g1 = (w.grad.clone(), x.grad.clone())
    w.grad = None
    x.grad = None
    loss2 = _WDHeadFn.apply(x, w, b, wide, dpad, wd, y)
    (loss2 * 3.0).backward()
    assert torch.equal(loss2, loss) and torch.equal(w.grad, g1[0]) and torch.equal(x.grad, g1[1])


@pytest.mark.parametrize("B,H,Dn,Dp", [(65536, 256, 13, 16), (1000, 64, 5, 8)])
def test_wd_head_flat_bf16_params_direct_grads(B, H, Dn, Dp):
    """The training-time head: bf16 out_w / wide_dense and fp32 out_b living in flat
    gradient buffers, raw [B, Dn] dense features (Dn < Dp, zero pad columns), int64
    labels.  The backward ADDS the three parameter gradients into the flat buffers
    (no casts, no autograd accumulate) and reports each parameter ready exactly once;
    loss and gradients vs the fp32 PyTorch chain."""
    from kubeflow_controller_amd.models.wide_deep import _WDHeadFn
    from kubeflow_controller_amd.parallel.flat import FlatGroup, register_ready_hook
    import torch.nn.functional as F
    torch.manual_seed(B + Dn)
    d = torch.device("cuda")
    x = (torch.randn(B, H, device=d) * 0.5).to(torch.bfloat16).requires_grad_()
    out_w = torch.nn.Parameter((torch.randn(1, H, device=d) * H ** -0.5).to(torch.bfloat16))
    wide_dense = torch.nn.Parameter((torch.randn(1, Dp, device=d) * 0.1).to(torch.bfloat16))
    out_b = torch.nn.Parameter(torch.randn(1, device=d))
    gbf = FlatGroup([out_w, wide_dense])
    g32 = FlatGroup([out_b])
    prior = 0.25  # gradients already accumulated this step: the head must add to them
    gbf.grad.fill_(prior)
    g32.grad.fill_(prior)
    seen = []
    hooks = [register_ready_hook(p, lambda q: seen.append(id(q))) for p in (out_w, out_b, wide_dense)]
    wide = torch.randn(B, device=d).requires_grad_()
    dense = torch.randn(B, Dn, device=d)
    y = (torch.rand(B, device=d) < 0.3).long()
    loss = _WDHeadFn.apply(x, out_w, out_b, wide, dense, wide_dense, y)
    (loss * 3.0).backward()
    for h in hooks:
        h.remove()
    assert sorted(seen) == sorted(id(p) for p in (out_w, out_b, wide_dense))
    xr = x.detach().float().requires_grad_()
    wr = out_w.detach().float().requires_grad_()
    wdr = wide_dense.detach().float().requires_grad_()
    br = out_b.detach().clone().requires_grad_()
    wider = wide.detach().clone().requires_grad_()
    dpad = F.pad(dense, (0, Dp - Dn))
    z = (xr @ wr.t()).squeeze(1) + br + wider + (dpad @ wdr.t()).squeeze(1)
    ref = F.binary_cross_entropy_with_logits(z, y.float())
    (ref * 3.0).backward()
    torch.testing.assert_close(loss, ref, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=1e-6, rtol=1e-2)
    torch.testing.assert_close(wide.grad, wider.grad, atol=1e-7, rtol=1e-5)
    # the flat gradient views: prior + gradient, rounded once to bf16 (fp32 for out_b)
    torch.testing.assert_close(out_w.grad.float(), (prior + wr.grad).to(torch.bfloat16).float(), atol=1e-3, rtol=1e-2)
    torch.testing.assert_close(wide_dense.grad[:, :Dn].float(), (prior + wdr.grad[:, :Dn]).to(torch.bfloat16).float(),
                               atol=1e-3, rtol=1e-2)
    assert torch.all(wide_dense.grad[:, Dn:].float() == prior)  # pad columns: nothing added
    torch.testing.assert_close(out_b.grad, prior + br.grad, atol=1e-6, rtol=1e-4)
    assert out_w.grad.data_ptr() == gbf.grad.data_ptr() + gbf.offsets[0] * 2  # still the flat view


def test_wd_fused_lookup_matches_lookup_then_assembly(monkeypatch):
    """World 1: the table gather straight into the MLP input (kfa_wd_gather_fwd) vs the
    lookup kernel + the assembly kernel — the same loss, and the table's sparse optimizer
    receives bit-identical ids and row gradients either way (the update itself is the
    same segment-reduce Adam call; its fp32 segment sums are not order-deterministic)."""
    import copy
    from kubeflow_controller_amd.models import wide_deep as WD
    from kubeflow_controller_amd.parallel.embedding import ShardedEmbedding
    d = torch.device("cuda")
    cfg = WD.WideDeepConfig(cardinalities=(5000, 300, 40, 7) * 3, embed_dim=32, mlp=(64, 32))
    torch.manual_seed(0)
    base = WD.WideDeep(cfg, device=d).to(d)
    for p in base.weights:
        p.data = p.data.to(torch.bfloat16)
    g = torch.Generator().manual_seed(3)
    dense, ids, labels = WD.synthetic_batch(cfg, 3000, g, d)
    orig_asm, orig_apply = WD.WideDeep._assemble, ShardedEmbedding.apply_sparse
    seen = {}

    def spy_asm(self, *a, **k):  # the lookup + assembly pair ran
        seen["unfused"] = True
        return orig_asm(self, *a, **k)

    def spy_apply(self, local, grad, prep=None, wd_src=None):
        if wd_src is not None:  # the rows the segment update reads out of dx / dwide, materialised
            dx, dwide, F, E, Dp = wd_src
            nb = dx.shape[0]
            tail = torch.zeros(nb * F, 8, dtype=torch.bfloat16, device=dx.device)
            tail[:, 0] = dwide.to(torch.bfloat16).repeat_interleave(F)
            grad_eq = torch.cat([dx[:, Dp:Dp + F * E].reshape(nb * F, E), tail], 1)
        seen["sparse"] = (local.clone(), (grad if wd_src is None else grad_eq).clone())
        return orig_apply(self, local, grad, prep=prep, wd_src=wd_src)
    monkeypatch.setattr(WD.WideDeep, "_assemble", spy_asm)
    monkeypatch.setattr(ShardedEmbedding, "apply_sparse", spy_apply)
    out = {}
    for fused in (True, False):
        monkeypatch.setattr(WD, "FUSED_LOOKUP", fused)
        m = copy.deepcopy(base)
        gids = (ids + m.offsets.view(1, -1)).reshape(-1)
        assert WD.lookup_fusable(m.tables, gids, cfg.embed_dim) is fused
        seen.clear()
        loss = m(dense, ids, labels)
        loss.backward()
        torch.cuda.synchronize()
        assert seen.get("unfused", False) is (not fused) and "sparse" in seen
        local, grad = seen["sparse"]
        if fused:  # per-table ids (the sort adds the table offsets itself): as global rows
            local = (local.view(-1, len(cfg.cardinalities)) + m.offsets.view(1, -1)).reshape(-1)
        out[fused] = (float(loss.detach()), local, grad)
    assert out[True][0] == out[False][0]
    assert torch.equal(out[True][1], out[False][1]) and torch.equal(out[True][2], out[False][2])


def test_seg_apply_reads_wd_gradient_in_place():
    """kfa_seg_apply_wd (the table's segment Adam reading each row's gradient straight out
    of the MLP input gradient dx / dwide, on a sort whose key pass added the per-table
    offsets: kfa_seg_prepare_off) vs kfa_seg_apply on the materialised rows
    (kfa_wd_input_bwd) sorted by global row: the same table, moments and step afterwards."""
    import copy
    from kubeflow_controller_amd.models.wide_deep import _lib as L
    from kubeflow_controller_amd.parallel.embedding import ShardedEmbedding
    d = torch.device("cuda")
    torch.manual_seed(7)
    B, F, E, Dp = 4000, 13, 32, 16
    emb = ShardedEmbedding(20000, E + 8, lr=1e-2, device=d)
    # per-table ids of 13 tables of 1500 rows (hot rows, long segments); global row = id + offset
    ids = (torch.rand(B * F, device=d) ** 3 * 1500).long().clamp_(0, 1499)
    offs = torch.arange(F, device=d, dtype=torch.int64) * 1500
    gids = (ids.view(B, F) + offs.view(1, F)).reshape(-1)
    dx = torch.randn(B, Dp + F * E, device=d).to(torch.bfloat16)
    dwide = torch.randn(B, device=d)
    e2 = copy.deepcopy(emb)
    prep = emb.prepare_sparse(ids, offsets=offs, F=F)   # the sort's key pass adds the offsets
    assert emb.can_apply_wd(ids, prep)
    emb.apply_sparse(ids, None, prep=prep, wd_src=(dx, dwide, F, E, Dp))
    drows = torch.empty(B * F, E + 8, dtype=torch.bfloat16, device=d)
    L.call("kfa_wd_input_bwd", L.ptr(dx), L.ptr(dwide), L.ptr(drows), B, F, E, Dp, L.stream())
    e2.apply_sparse(gids, drows, prep=e2.prepare_sparse(gids))
    torch.cuda.synchronize()
    assert emb.t == e2.t == 1
    # chunk-crossing segments meet in fp32 atomics: equal up to summation order
    torch.testing.assert_close(emb.weight, e2.weight, atol=1e-6, rtol=0)
    torch.testing.assert_close(emb.exp_avg, e2.exp_avg, atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(emb.exp_avg_sq, e2.exp_avg_sq, atol=1e-8, rtol=1e-4)
