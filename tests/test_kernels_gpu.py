"""Numerics of the hand-written HIP kernels vs plain PyTorch fp32 references."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev():
    return torch.device("cuda")


def _native_loaded():
    from kubeflow_controller_amd.ops import _lib
    lib = _lib.lib()
    assert lib is not None
    return lib


@pytest.mark.parametrize("N,C,H,W", [(4, 64, 14, 14), (2, 256, 7, 7), (3, 2048, 2, 3), (8, 24, 5, 5), (1, 4096, 1, 3)])
@pytest.mark.parametrize("relu,res", [(True, False), (True, True), (False, False)])
def test_bn_act_fwd_bwd(N, C, H, W, relu, res):
    _native_loaded()
    from kubeflow_controller_amd.ops.batchnorm import bn_act
    torch.manual_seed(0)
    d = _dev()
    x = (torch.randn(N, C, H, W, device=d) * 2 + 3).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(x) if res else None
    g = (torch.rand(C, device=d) + 0.5).requires_grad_()
    b = torch.randn(C, device=d).requires_grad_()
    rm, rv = torch.zeros(C, device=d), torch.ones(C, device=d)
    xr = x.detach().clone().requires_grad_()
    rr = r.detach().clone().requires_grad_() if res else None
    y = bn_act(xr, g, b, rm, rv, rr, True, 0.1, 1e-5, relu)
    # fp32 reference
    xf = x.float().detach().requires_grad_()
    rf = r.float().detach().requires_grad_() if res else None
    g2, b2 = g.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    rm2, rv2 = torch.zeros(C, device=d), torch.ones(C, device=d)
    yf = torch.nn.functional.batch_norm(xf, rm2, rv2, g2, b2, True, 0.1, 1e-5)
    if res:
        yf = yf + rf
    if relu:
        yf = torch.relu(yf)
    assert (y.float() - yf).abs().max().item() < 0.05 * max(1.0, yf.abs().max().item() / 8)
    torch.testing.assert_close(rm, rm2, atol=2e-3, rtol=2e-3)
    torch.testing.assert_close(rv, rv2, atol=2e-3, rtol=2e-3)
    dy = torch.randn_like(y)
    y.backward(dy)
    yf.backward(dy.float())
    # the kernel's ReLU mask comes from the bf16 output; compare where the masks agree
    assert (xr.grad.float() - xf.grad).abs().max().item() < 0.05 * max(1.0, xf.grad.abs().max().item())
    torch.testing.assert_close(g.grad, g2.grad, atol=0.05 * max(1.0, g2.grad.abs().max().item()), rtol=0.02)
    torch.testing.assert_close(b.grad, b2.grad, atol=0.05 * max(1.0, b2.grad.abs().max().item()), rtol=0.02)
    if res:
        assert (rr.grad.float() - rf.grad).abs().max().item() < 0.02 * max(1.0, rf.grad.abs().max().item())


@pytest.mark.parametrize("res", [False, True])
@pytest.mark.parametrize("N,C,H,W", [(4, 64, 14, 14), (3, 2048, 2, 3), (8, 24, 5, 5)])
def test_bn_relu_mask_from_input_matches_output_mask(N, C, H, W, res, monkeypatch):
    """BN+ReLU recomputes the backward ReLU mask from x and the saved scale/shift
    (no residual) or reads the forward's bit mask (residual); both must reproduce
    the output-mask backward bit for bit."""
    from kubeflow_controller_amd.ops import batchnorm as bnmod
    torch.manual_seed(1)
    d = _dev()
    x = (torch.randn(N, C, H, W, device=d) * 2).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.randn_like(x)
    r = torch.randn_like(x) if res else None
    outs = []
    for from_x in (True, False):
        monkeypatch.setattr(bnmod, "MASK_FROM_X", from_x)
        g = (torch.rand(C, device=d, generator=torch.Generator(d).manual_seed(2)) + 0.5).requires_grad_()
        b = torch.randn(C, device=d, generator=torch.Generator(d).manual_seed(3)).requires_grad_()
        xr = x.detach().clone().requires_grad_()
        rr = r.detach().clone().requires_grad_() if res else None
        y = bnmod.bn_act(xr, g, b, torch.zeros(C, device=d), torch.ones(C, device=d), rr, True, 0.1, 1e-5, True)
        y.backward(dy)
        outs.append((y, xr.grad, g.grad, b.grad) + ((rr.grad,) if res else ()))
    for a, b_ in zip(*outs):
        assert torch.equal(a, b_)


def test_bn_act_eval():
    from kubeflow_controller_amd.ops.batchnorm import bn_act
    d = _dev()
    C = 128
    x = torch.randn(2, C, 9, 9, device=d).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g, b = torch.rand(C, device=d) + 0.5, torch.randn(C, device=d)
    rm, rv = torch.randn(C, device=d), torch.rand(C, device=d) + 0.5
    y = bn_act(x, g, b, rm, rv, None, False, 0.1, 1e-5, True)
    yf = torch.relu(torch.nn.functional.batch_norm(x.float(), rm, rv, g, b, False, 0.1, 1e-5))
    assert (y.float() - yf).abs().max().item() < 0.05


@pytest.mark.parametrize("rows,V,dtype", [(64, 1000, torch.bfloat16), (7, 10, torch.float32), (5, 30522, torch.bfloat16),
                                          (16, 1000, torch.float32)])
@pytest.mark.parametrize("smoothing", [0.0, 0.1])
def test_softmax_xent(rows, V, dtype, smoothing):
    from kubeflow_controller_amd.ops.loss import argmax, cross_entropy
    d = _dev()
    torch.manual_seed(1)
    z = (torch.randn(rows, V, device=d) * 3).to(dtype).requires_grad_()
    y = torch.randint(0, V, (rows,), device=d)
    y[0] = -100  # ignored row
    loss = cross_entropy(z, y, smoothing)
    zf = z.detach().float().requires_grad_()
    valid = (y >= 0)
    ref = torch.nn.functional.cross_entropy(zf, y.clamp(min=0), reduction="none", label_smoothing=smoothing)
    ref = (ref * valid).sum() / rows
    torch.testing.assert_close(loss, ref, atol=2e-3, rtol=2e-3)
    loss.backward()
    ref.backward()
    torch.testing.assert_close(z.grad.float(), zf.grad, atol=3e-3 / 1, rtol=0.05)
    am = argmax(z.detach())
    torch.testing.assert_close(am, z.detach().float().argmax(-1))


@pytest.mark.parametrize("nesterov", [False, True])
def test_fused_sgd_matches_torch(nesterov):
    from kubeflow_controller_amd.ops.optim import FusedSGD
    from kubeflow_controller_amd.parallel.flat import FlatGroup
    d = _dev()
    torch.manual_seed(2)
    ps = [torch.nn.Parameter(torch.randn(37, 5, device=d)), torch.nn.Parameter(torch.randn(11, device=d))]
    ref = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    g = FlatGroup(ps, name="weights")
    opt = FusedSGD([g], lr=0.05, momentum=0.9, weight_decay=0.01, nesterov=nesterov)
    topt = torch.optim.SGD(ref, lr=0.05, momentum=0.9, weight_decay=0.01, nesterov=nesterov)
    for _ in range(3):
        grads = [torch.randn_like(p) for p in ps]
        g.zero_grad()
        for p, gr in zip(ps, grads):
            p.grad.copy_(gr)
        for p, gr in zip(ref, grads):
            p.grad = gr.clone()
        opt.step()
        topt.step()
    for p, r in zip(ps, ref):
        torch.testing.assert_close(p.detach(), r.detach(), atol=1e-5, rtol=1e-5)


def test_fused_adam_bf16_master():
    from kubeflow_controller_amd.ops.optim import FusedAdam
    from kubeflow_controller_amd.parallel.flat import FlatGroup
    d = _dev()
    torch.manual_seed(3)
    p0 = torch.randn(64, 33, device=d)
    ps = [torch.nn.Parameter(p0.to(torch.bfloat16))]
    ref = torch.nn.Parameter(ps[0].detach().float().clone())
    g = FlatGroup(ps, name="weights")
    opt = FusedAdam([g], lr=1e-2, weight_decay=0.1)
    topt = torch.optim.AdamW([ref], lr=1e-2, weight_decay=0.1)
    for _ in range(4):
        gr = torch.randn(64, 33, device=d).to(torch.bfloat16)
        g.zero_grad()
        ps[0].grad.copy_(gr)
        ref.grad = gr.float()
        opt.step()
        topt.step()
    torch.testing.assert_close(g.master[:64 * 33].view(64, 33), ref.detach(), atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(ps[0].detach().float(), ref.detach(), atol=2e-2, rtol=1e-2)


def test_resnet_tiny_step_runs_native():
    """One full engine step on a tiny ResNet: every HIP op on the path runs."""
    from kubeflow_controller_amd.models.resnet import resnet_tiny
    from kubeflow_controller_amd.ops.loss import cross_entropy
    from kubeflow_controller_amd.trainer.engine import DistInfo, Engine
    d = _dev()
    m = resnet_tiny(10)
    eng = Engine(m, lambda mm, x, y: cross_entropy(mm(x), y), lr=0.05,
                 dist_info=DistInfo(device=d))
    x = torch.randn(8, 3, 32, 32, device=d, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device=d)
    losses = [float(eng.train_step(x, y)) for _ in range(8)]
    assert all(l == l for l in losses)
    assert losses[-1] < losses[0]


@pytest.mark.parametrize("k,s,p", [(3, 2, 1), (3, 2, 0), (2, 2, 0), (3, 1, 1)])
@pytest.mark.parametrize("N,C,H,W", [(2, 64, 112, 112), (3, 16, 9, 7)])
def test_maxpool_fwd_bwd(N, C, H, W, k, s, p):
    """3x3/s2 takes the batched-load fast path; other windows the generic kernels."""
    from kubeflow_controller_amd.ops.pool import max_pool2d
    d = _dev()
    torch.manual_seed(4)
    x = torch.randn(N, C, H, W, device=d).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xr = x.detach().clone().requires_grad_()
    y = max_pool2d(xr, k, s, p)
    xf = x.float().detach().requires_grad_()
    yf = torch.nn.functional.max_pool2d(xf, k, s, p)
    torch.testing.assert_close(y.float(), yf)
    dy = torch.randn_like(y)
    y.backward(dy)
    yf.backward(dy.float())
    torch.testing.assert_close(xr.grad.float(), xf.grad, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("N,C,H,W", [(4, 256, 14, 14), (2, 2048, 7, 7), (8, 24, 5, 5)])
@pytest.mark.parametrize("conv_stats", [False, True])
def test_bn_act_dual_downsample_pair_matches_fp32(N, C, H, W, conv_stats):
    """relu(bn(x) + bn_r(r)) in one apply pass each way (ops.batchnorm.bn_act_dual)
    vs two fp32 batch_norms: output, running stats, dx, dr, both BNs' dgamma /
    dbeta.  conv_stats: x / r come from convs whose epilogues accumulated the
    statistics (x into the shared slots, r into DS_SLOTS).  Both slot
    workspaces must be clean (all zero) afterwards."""
    _native_loaded()
    from kubeflow_controller_amd.ops import conv as CV
    from kubeflow_controller_amd.ops.batchnorm import DS_SLOTS, BatchNorm2dAct, bn_act_dual, bn_slot_workspace
    torch.manual_seed(3)
    d = _dev()
    cl = torch.channels_last
    bn, bnr = BatchNorm2dAct(C, relu=True).to(d), BatchNorm2dAct(C, relu=False).to(d)
    for m in (bn, bnr):
        with torch.no_grad():
            m.weight.copy_(torch.rand(C, device=d) + 0.5)
            m.bias.copy_(torch.randn(C, device=d) * 0.3)
    if conv_stats and C % 64 == 0:
        xin = (torch.randn(N, 64, H, W, device=d)).to(torch.bfloat16).contiguous(memory_format=cl)
        w1 = (torch.randn(C, 64, 1, 1, device=d) * 0.2).to(torch.bfloat16).contiguous(memory_format=cl)
        w2 = (torch.randn(C, 64, 1, 1, device=d) * 0.2).to(torch.bfloat16).contiguous(memory_format=cl)
        with torch.no_grad():
            r0 = CV.conv2d(xin, w2, bn_stats=DS_SLOTS)
            x0 = CV.conv2d(xin, w1, bn_stats=True)
        assert getattr(x0, "_kfa_prestats", False) and getattr(r0, "_kfa_prestats_tag", None) == DS_SLOTS
    else:
        x0 = (torch.randn(N, C, H, W, device=d) * 2 + 1).to(torch.bfloat16).contiguous(memory_format=cl)
        r0 = (torch.randn(N, C, H, W, device=d) - 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
    x = x0.detach().requires_grad_()
    r = r0.detach().requires_grad_()
    for t, t0 in ((x, x0), (r, r0)):  # keep the conv's statistics tags on the leaf copies
        for a in ("_kfa_prestats", "_kfa_prestats_tag"):
            if hasattr(t0, a):
                setattr(t, a, getattr(t0, a))
    y = bn_act_dual(bn, x, bnr, r)
    xf, rf = x0.float().detach().requires_grad_(), r0.float().detach().requires_grad_()
    g1, b1 = bn.weight.detach().clone().requires_grad_(), bn.bias.detach().clone().requires_grad_()
    g2, b2 = bnr.weight.detach().clone().requires_grad_(), bnr.bias.detach().clone().requires_grad_()
    rm1, rv1, rm2, rv2 = (torch.zeros(C, device=d), torch.ones(C, device=d), torch.zeros(C, device=d),
                          torch.ones(C, device=d))
    F = torch.nn.functional
    yf = torch.relu(F.batch_norm(xf, rm1, rv1, g1, b1, True, 0.1, 1e-5) + F.batch_norm(rf, rm2, rv2, g2, b2, True, 0.1,
                                                                                         1e-5))
    assert (y.float() - yf).abs().max().item() < 0.05 * max(1.0, yf.abs().max().item() / 8)
    for a, b_ in ((bn.running_mean, rm1), (bn.running_var, rv1), (bnr.running_mean, rm2), (bnr.running_var, rv2)):
        torch.testing.assert_close(a, b_, atol=3e-3, rtol=3e-3)
    dy = torch.randn_like(y)
    y.backward(dy)
    yf.backward(dy.float())
    for got, want in ((x.grad, xf.grad), (r.grad, rf.grad)):
        assert (got.float() - want).abs().max().item() < 0.05 * max(1.0, want.abs().max().item())
    for got, want in ((bn.weight.grad, g1.grad), (bn.bias.grad, b1.grad), (bnr.weight.grad, g2.grad),
                      (bnr.bias.grad, b2.grad)):
        torch.testing.assert_close(got, want, atol=0.05 * max(1.0, want.abs().max().item()), rtol=0.02)
    torch.cuda.synchronize()
    for tag in ("bn_slots", DS_SLOTS):
        assert bn_slot_workspace(C, d, tag).abs().max().item() == 0, f"{tag} left dirty"


@pytest.mark.parametrize("N,C,H,W", [(4, 64, 112, 112), (2, 16, 9, 7)])
def test_bn_relu_maxpool_fused_matches_fp32(N, C, H, W):
    """Stem BN + ReLU + 3x3/s2 max pool in one pass (ops.batchnorm.bn_relu_maxpool)
    vs fp32 batch_norm -> relu -> max_pool2d: output, running stats, dx, dgamma,
    dbeta."""
    _native_loaded()
    from kubeflow_controller_amd.ops.batchnorm import BatchNorm2dAct, bn_relu_maxpool
    torch.manual_seed(9)
    d = _dev()
    bn = BatchNorm2dAct(C, relu=True).to(d)
    with torch.no_grad():
        bn.weight.copy_(torch.rand(C, device=d) + 0.5)
        bn.bias.copy_(torch.randn(C, device=d) * 0.3)
    x0 = (torch.randn(N, C, H, W, device=d) * 2 + 0.5).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x = x0.detach().requires_grad_()
    y = bn_relu_maxpool(bn, x)
    xf = x0.float().detach().requires_grad_()
    g, b = bn.weight.detach().clone().requires_grad_(), bn.bias.detach().clone().requires_grad_()
    rm, rv = torch.zeros(C, device=d), torch.ones(C, device=d)
    F = torch.nn.functional
    yf = F.max_pool2d(torch.relu(F.batch_norm(xf, rm, rv, g, b, True, 0.1, 1e-5)), 3, 2, 1)
    assert y.shape == yf.shape
    assert (y.float() - yf).abs().max().item() < 0.02 * max(1.0, yf.abs().max().item())
    torch.testing.assert_close(bn.running_mean, rm, atol=2e-3, rtol=2e-3)
    torch.testing.assert_close(bn.running_var, rv, atol=2e-3, rtol=2e-3)
    dy = torch.randn_like(y)
    y.backward(dy)
    yf.backward(dy.float())
    # argmax ties between bf16-rounded window values may route a gradient to a different tap
    err = (x.grad.float() - xf.grad).abs()
    assert (err > 0.05 * max(1.0, xf.grad.abs().max().item())).float().mean().item() < 1e-3
    torch.testing.assert_close(bn.weight.grad, g.grad, atol=0.05 * max(1.0, g.grad.abs().max().item()), rtol=0.03)
    torch.testing.assert_close(bn.bias.grad, b.grad, atol=0.05 * max(1.0, b.grad.abs().max().item()), rtol=0.03)


@pytest.mark.parametrize("N,C,H,W", [(256, 2048, 7, 7), (3, 16, 5, 3)])
def test_global_avg_pool_fwd_bwd(N, C, H, W):
    """ops.pool.global_avg_pool (kfa_gap_fwd / kfa_gap_bwd) vs fp32 mean."""
    _native_loaded()
    from kubeflow_controller_amd.ops.pool import global_avg_pool
    torch.manual_seed(2)
    d = _dev()
    x0 = torch.randn(N, C, H, W, device=d).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x = x0.detach().requires_grad_()
    y = global_avg_pool(x)
    xf = x0.float().detach().requires_grad_()
    yf = xf.mean((2, 3))
    torch.testing.assert_close(y.float(), yf, atol=1e-2, rtol=1e-2)
    dy = torch.randn(N, C, device=d).to(torch.bfloat16)
    y.backward(dy)
    yf.backward(dy.float())
    assert x.grad.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(x.grad.float(), xf.grad, atol=1e-3, rtol=1e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_clipped_sum_xent_matches_fp32(dtype):
    """mnist_replica.py:168's summed clipped cross-entropy on the fused xent kernel:
    loss and gradient vs the float64 TensorFlow-semantics reference (clip_by_value
    passes no gradient where the label probability is below 1e-10)."""
    from kubeflow_controller_amd.ops.loss import clipped_sum_cross_entropy
    torch.manual_seed(3)
    z = (torch.randn(100, 10, device="cuda") * 3)
    z[5] = torch.tensor([80.0, -80.0] + [0.0] * 8, device="cuda")
    y = torch.randint(0, 10, (100,), device="cuda")
    y[5] = 1
    zz = z.to(dtype).clone().requires_grad_()
    loss = clipped_sum_cross_entropy(zz, y)
    loss.backward()
    zr = z.to(dtype).detach().double().cpu().requires_grad_()
    p = torch.softmax(zr, -1)
    ref = -(torch.nn.functional.one_hot(y.cpu(), 10).double() * torch.log(p.clamp(1e-10, 1.0))).sum()
    ref.backward()
    assert abs(float(loss.detach()) - float(ref)) <= 2e-3 * float(ref)
    torch.testing.assert_close(zz.grad.double().cpu(), zr.grad, atol=2e-2 if dtype == torch.bfloat16 else 1e-5,
                               rtol=2e-2 if dtype == torch.bfloat16 else 1e-4)
    assert float(zz.grad[5].float().abs().sum()) == 0.0


@pytest.mark.parametrize("B,H,C", [(256, 768, 2), (37, 64, 5), (1000, 512, 8), (3, 8, 1), (64, 1024, 2)])
def test_classifier_head_xent_matches_fp32(B, H, C):
    """Fused small-classifier head + softmax CE (kfa_cls_head_fwd / _bwd, BERT's NSP)
    vs the plain fp32 PyTorch chain: loss, dx, dW, db; bit-identical on a rerun."""
    import torch.nn.functional as F
    from kubeflow_controller_amd.ops.loss import classifier_xent
    torch.manual_seed(B + H + C)
    d = torch.device("cuda")
    x = torch.randn(B, H, device=d).to(torch.bfloat16).requires_grad_()
    w = (torch.randn(C, H, device=d) * H ** -0.5).to(torch.bfloat16).requires_grad_()
    b = torch.randn(C, device=d).requires_grad_()
    y = torch.randint(0, C, (B,), device=d)
    loss = classifier_xent(x, w, b, y)
    (loss * 2.0).backward()
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    ref = F.cross_entropy(xr @ wr.t() + br, y)
    (ref * 2.0).backward()
    torch.testing.assert_close(loss, ref, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=1e-5, rtol=1e-2)
    torch.testing.assert_close(w.grad.float(), wr.grad, atol=1e-3, rtol=1e-2)
    torch.testing.assert_close(b.grad, br.grad, atol=1e-5, rtol=1e-4)
    g1 = (x.grad.clone(), w.grad.clone(), b.grad.clone())
    x.grad = w.grad = b.grad = None
    loss2 = classifier_xent(x, w, b, y)
    (loss2 * 2.0).backward()
    assert torch.equal(loss2, loss) and torch.equal(x.grad, g1[0]) and torch.equal(w.grad, g1[1])
