"""Implicit-GEMM conv (csrc/kernels/conv_igemm.hip) vs PyTorch fp32 reference."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _no_forward_tuner(monkeypatch):
    """These tests check the implicit GEMM itself: keep the forward tuner from
    routing a shape to the vendor forward (test_conv_forward_tuner covers it)."""
    from kubeflow_controller_amd.ops import conv as convmod
    monkeypatch.setattr(convmod, "TUNE", False)

SHAPES = [
    # N, Cin, H, W, Cout, k, stride, pad
    (2, 64, 14, 14, 64, 1, 1, 0),
    (2, 64, 14, 14, 256, 1, 1, 0),
    (2, 128, 15, 13, 128, 3, 1, 1),
    (2, 256, 14, 14, 512, 1, 2, 0),
    (2, 128, 14, 14, 128, 3, 2, 1),
    (3, 64, 9, 9, 192, 3, 2, 1),
    (1, 512, 7, 7, 2048, 1, 1, 0),
    (5, 64, 8, 8, 64, 3, 1, 1),
    # 256x256 8-wave tiles (Cout / Cin multiples of 256, K >= 256), incl. M tails
    (3, 256, 9, 11, 256, 3, 1, 1),
    (2, 256, 16, 16, 512, 3, 2, 1),
]


@pytest.mark.parametrize("big", [False, True, "pp", "pp512"])
@pytest.mark.parametrize("N,Cin,H,W,Cout,k,stride,pad", SHAPES)
def test_conv_igemm_fwd_dgrad(N, Cin, H, W, Cout, k, stride, pad, big, monkeypatch):
    """fwd + dgrad (+ the wgrad) of the implicit GEMM vs fp32 PyTorch; big = the
    8-wave 256x256 tile, "pp" = the ping-pong 256x256 kernel (conv_pp_kernel) on
    every launch with >= 64 output channels (tails in M and N included), "pp512" = its
    512x128 form (two wave-rows per group)."""
    from kubeflow_controller_amd.ops import conv as convmod
    from kubeflow_controller_amd.ops.conv import conv2d
    if big is True and not (Cout % 256 == 0 or Cin % 256 == 0):
        pytest.skip("256x256 tiles only for 256-multiple channel counts")
    if big in ("pp", "pp512"):
        monkeypatch.setattr(convmod, "PP", "1" if big == "pp" else "512")
        monkeypatch.setattr(convmod, "PP_MIN_N", 64)
    else:
        monkeypatch.setattr(convmod, "BIG", big)
    torch.manual_seed(0)
    d = torch.device("cuda")
    x = torch.randn(N, Cin, H, W, device=d).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, k, k, device=d) / (Cin * k * k) ** 0.5).to(torch.bfloat16)
    w = w.contiguous(memory_format=torch.channels_last)
    xr, wr = x.clone().requires_grad_(), w.clone().requires_grad_()
    y = conv2d(xr, wr, stride, pad)
    xf, wf = x.float().requires_grad_(), w.float().requires_grad_()
    yf = torch.nn.functional.conv2d(xf, wf, None, stride, pad)
    assert y.shape == yf.shape
    err = (y.float() - yf).abs().max().item()
    assert err < 2e-2 * max(1.0, yf.abs().max().item()), err
    dy = torch.randn_like(yf)
    y.backward(dy.to(torch.bfloat16))
    yf.backward(dy)
    gx = (xr.grad.float() - xf.grad).abs().max().item()
    assert gx < 2e-2 * max(1.0, xf.grad.abs().max().item()), gx
    gw = (wr.grad.float() - wf.grad).abs().max().item()
    assert gw < 3e-2 * max(1.0, wf.grad.abs().max().item()), gw


def _stack_grads(enabled, join, x, m):
    from kubeflow_controller_amd.ops import conv as convmod
    convmod.ENABLED = enabled
    orig = convmod.GradJoin.branch
    if not join:
        convmod.GradJoin.branch = lambda self, t: t
    try:
        m.zero_grad(set_to_none=True)
        xr = x.clone().requires_grad_()
        m(xr).float().square().mean().backward()
        return [xr.grad.float()] + [p.grad.float() for p in m.parameters()]
    finally:
        convmod.GradJoin.branch = orig
        convmod.ENABLED = True


def _fp32_reference_grads(x, m):
    """Same network in fp32 on the CPU with plain PyTorch ops (conv2d/batch_norm/relu)."""
    import copy
    ref = copy.deepcopy(m).cpu().float()
    xr = x.detach().float().cpu().contiguous().requires_grad_()
    ref(xr).float().square().mean().backward()
    return [xr.grad] + [p.grad for p in ref.parameters()]


def test_resnet_block_grads_igemm_vs_vendor():
    """Bottleneck stack incl. the fused residual-gradient joins (GradJoin): the HIP
    conv path must be as close to an fp32 reference as the vendor bf16 convs are."""
    from kubeflow_controller_amd.models.resnet import ResNet
    d = torch.device("cuda")
    torch.manual_seed(0)
    m = ResNet((2, 1, 1, 1), num_classes=10, width=64).to(d).to(memory_format=torch.channels_last)
    for p in m.parameters():
        if p.dim() >= 2:
            p.data = p.data.to(torch.bfloat16)
    for mod in m.modules():  # non-zero residual scale so every branch carries gradient
        if hasattr(mod, "bn3"):
            torch.nn.init.uniform_(mod.bn3.weight, 0.5, 1.5)
    x = torch.randn(8, 3, 128, 128, device=d).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ref = _fp32_reference_grads(x, m)
    fused = _stack_grads(True, True, x, m)
    unfused = _stack_grads(True, False, x, m)
    vendor = _stack_grads(False, False, x, m)
    names = ["input"] + [n for n, _ in m.named_parameters()]
    bad = []
    for n, f, u, v, r in zip(names, fused, unfused, vendor, ref):
        r = r.to(f.device).float()
        if r.dim() == 4:
            r = r.contiguous(memory_format=torch.channels_last)
        # relative Frobenius error: the max-abs error of a tiny, rounding-dominated
        # gradient (e.g. the last stage's conv3 weight at 4x4 pixels) varies run to
        # run with the order of the BN-statistics atomics
        rn = max(1e-12, r.norm().item())
        e_f, e_u, e_v = ((t.float() - r).norm().item() / rn for t in (f, u, v))
        if e_f > 1.5 * e_v + 0.01 or e_u > 1.5 * e_v + 0.01:
            bad.append((n, e_f, e_u, e_v))
    assert not bad, bad


@pytest.mark.parametrize("rows,out_f,in_f", [(8192, 2304, 768), (4096, 768, 3072), (1000, 64, 136),
                                             # 64x256 tiles (Co <= 64, N % 256 == 0), split-K, tail rows
                                             (20000, 64, 256), (3001, 48, 512),
                                             # ping-pong pointwise 256x256 (wgrad_pp_kernel): BERT shapes,
                                             # a tail k-tile, edge tiles in both dims, a 1x1 conv's pixels
                                             (32768, 768, 768), (32768, 768, 3072), (12001, 512, 256),
                                             (9000, 768, 1280), (12544, 1024, 256),
                                             (20000, 1024, 1680), (17000, 776, 1000),  # edge tiles: N % 256 != 0
                                             # small weights, hundreds of pixel splits: the reduce's
                                             # 64 / 16 split-lanes per element
                                             (200000, 64, 64), (60000, 128, 72)])
def test_wgrad_dense_shapes(rows, out_f, in_f):
    """dW = dYᵀ·X through the wgrad kernel as a 1x1 conv over `rows` pixels."""
    from kubeflow_controller_amd.ops.conv import wgrad_into
    torch.manual_seed(0)
    d = torch.device("cuda")
    x = torch.randn(rows, in_f, device=d).to(torch.bfloat16)
    dy = torch.randn(rows, out_f, device=d).to(torch.bfloat16)
    ref = dy.float().t() @ x.float()
    out = torch.full((out_f, in_f), 0.5, device=d)  # fp32 target, accumulate
    wgrad_into(x, dy, out, 1, 1, rows, in_f, 1, rows, out_f, 1, 1, 1, 0, accumulate=True)
    err = (out - 0.5 - ref).abs().max().item()
    assert err < 1e-2 * ref.abs().max().item(), err
    outb = torch.zeros(out_f, in_f, device=d, dtype=torch.bfloat16)
    wgrad_into(x, dy, outb, 1, 1, rows, in_f, 1, rows, out_f, 1, 1, 1, 0, accumulate=False)
    err = (outb.float() - ref).abs().max().item()
    assert err < 2e-2 * ref.abs().max().item(), err


@pytest.mark.parametrize("N,Cin,H,W,Cout,k,stride,pad", [
    (8, 256, 32, 32, 256, 3, 1, 1),    # 14x14-stage-like 3x3: 8192 pixels, Co = 256, N = 2304
    (5, 256, 33, 31, 512, 3, 2, 1),    # strided 3x3, odd sizes: a tail k-tile, taps off both edges
    (24, 512, 14, 14, 512, 3, 2, 1),   # ResNet stage-4 entry shape, tail k-tile
    (9, 512, 30, 30, 1024, 1, 2, 0),   # strided 1x1 (downsample): gathered, not pointwise
    (2, 512, 64, 64, 256, 3, 1, 1),    # 18 weight tiles -> pixel split-K partials of the gathered kernel
])
def test_wgrad_gathered_pingpong(N, Cin, H, W, Cout, k, stride, pad):
    """Gathered (3x3 / strided) big weight gradients on wgrad_pp_kernel<true> (Co % 256 == 0,
    N % 256 == 0, >= 8192 pixels) vs the fp32 PyTorch weight gradient, fp32 accumulate
    and bf16 overwrite."""
    from kubeflow_controller_amd.ops.conv import wgrad_into
    torch.manual_seed(1)
    d = torch.device("cuda")
    x = torch.randn(N, Cin, H, W, device=d).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    P_ = (H + 2 * pad - k) // stride + 1
    Q_ = (W + 2 * pad - k) // stride + 1
    dy = torch.randn(N, Cout, P_, Q_, device=d).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ref = torch.ops.aten.convolution_backward(dy.float(), x.float(), torch.empty(Cout, Cin, k, k, device=d), None,
                                              [stride, stride], [pad, pad], [1, 1], False, [0, 0], 1,
                                              [False, True, False])[1]
    ref = ref.permute(0, 2, 3, 1).contiguous()  # [Co][R][S][Ci]
    out = torch.full((Cout, k, k, Cin), 0.25, device=d)
    wgrad_into(x, dy, out, N, H, W, Cin, P_, Q_, Cout, k, k, stride, pad, accumulate=True)
    err = (out - 0.25 - ref).abs().max().item()
    assert err < 1e-2 * ref.abs().max().item(), err
    outb = torch.zeros(Cout, k, k, Cin, device=d, dtype=torch.bfloat16)
    wgrad_into(x, dy, outb, N, H, W, Cin, P_, Q_, Cout, k, k, stride, pad, accumulate=False)
    err = (outb.float() - ref).abs().max().item()
    assert err < 2e-2 * ref.abs().max().item(), err


@pytest.mark.parametrize("wide", ["1", "0", "any"])
def test_wgrad_co64_gathered_taps(wide, monkeypatch):
    """Co = 64 weight gradients (1x1, gathered 3x3 / strided taps; N = R*S*Ci a
    multiple of 256) on the 64x256 tile and on the 64x128 one, both vs fp32.
    Own process per setting: the tile choice is read once from the env."""
    import subprocess, sys, os
    code = (
        "import torch, torch.nn.functional as F\n"
        "from kubeflow_controller_amd.ops.conv import wgrad_into\n"
        "torch.manual_seed(0); d = torch.device('cuda')\n"
        "for (N, Ci, H, k, s, p) in [(4, 256, 14, 1, 1, 0), (3, 256, 13, 3, 2, 1), (2, 512, 9, 3, 1, 1),\n"
        "                            (4, 64, 20, 3, 1, 1)]:  # N = 576: a quarter-full last 256-wide tile\n"
        "    x = torch.randn(N, Ci, H, H, device=d).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)\n"
        "    w = torch.randn(64, Ci, k, k, device=d)\n"
        "    y = F.conv2d(x.float(), w, None, s, p)\n"
        "    dy = torch.randn_like(y).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)\n"
        "    ref = torch.ops.aten.convolution_backward(dy.float(), x.float(), w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1, [False, True, False])[1]\n"
        "    P, Q = y.shape[2], y.shape[3]\n"
        "    out = torch.zeros(64, k, k, Ci, device=d)\n"
        "    wgrad_into(x, dy, out, N, H, H, Ci, P, Q, 64, k, k, s, p, accumulate=False)\n"
        "    err = (out.permute(0, 3, 1, 2) - ref).abs().max().item()\n"
        "    assert err < 1e-2 * ref.abs().max().item(), (N, Ci, H, k, s, err)\n"
        "print('ok')\n")
    env = dict(os.environ, KFA_WGRAD_WIDE64="0" if wide == "0" else "1", KFA_WGRAD_WIDE64_ANY="1" if wide == "any" else "0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-3000:]


@pytest.mark.parametrize("vendor", [False, True])
def test_wgrad_direct_into_flat_buffer(vendor, monkeypatch):
    """Direct-gradient protocol on both wgrad routes the tuner can pick: the HIP
    split-K wgrad accumulates into the flat view; the vendor's dW is added into it."""
    from kubeflow_controller_amd.ops import conv as convmod
    from kubeflow_controller_amd.ops.conv import Conv2d
    if vendor:
        monkeypatch.setattr(convmod, "TUNE", True)
        monkeypatch.setattr(convmod, "_use_vendor_wgrad", lambda *a: True)
    from kubeflow_controller_amd.parallel.flat import FlatGroup, set_ready_callback
    d = torch.device("cuda")
    torch.manual_seed(0)
    conv = Conv2d(64, 128, 3, stride=2, padding=1).to(d)
    conv.weight.data = conv.weight.data.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g = FlatGroup([conv.weight])
    seen = []
    set_ready_callback(conv.weight, lambda p: seen.append(p))
    x = torch.randn(4, 64, 28, 28, device=d).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = conv(x)
    dy = torch.randn_like(y)
    y.backward(dy)
    xf = x.float().requires_grad_()
    wf = conv.weight.detach().float().requires_grad_()
    torch.nn.functional.conv2d(xf, wf, None, 2, 1).backward(dy.float())
    assert len(seen) == 1 and conv.weight.grad.data_ptr() == g.grad.data_ptr()
    err = (conv.weight.grad.float() - wf.grad).abs().max().item()
    assert err < 3e-2 * wf.grad.abs().max().item(), err


@pytest.mark.parametrize("pp", [False, True, "512"])
@pytest.mark.parametrize("Cin,Cout,k,stride", [(64, 256, 1, 1), (128, 128, 3, 2), (64, 64, 3, 1), (256, 256, 3, 1)])
def test_bn_stats_fused_into_conv_epilogue(Cin, Cout, k, stride, pp, monkeypatch):
    """conv(bn_stats=True) accumulates the BN statistics in its epilogue; the BN
    then skips its stats pass — same outputs / running stats as the unfused pair,
    and the self-cleaning slot workspace is left zeroed (pp: the ping-pong kernel's epilogue)."""
    from kubeflow_controller_amd.ops import conv as convmod
    from kubeflow_controller_amd.ops.batchnorm import BatchNorm2dAct, bn_slot_workspace
    from kubeflow_controller_amd.ops.conv import Conv2d
    monkeypatch.setattr(convmod, "BIG", Cout % 256 == 0)  # the 256x256 tiles' epilogue too
    if pp:
        monkeypatch.setattr(convmod, "PP", "1" if pp is True else "512")
        monkeypatch.setattr(convmod, "PP_MIN_N", 64)
    d = torch.device("cuda")
    torch.manual_seed(0)
    conv = Conv2d(Cin, Cout, k, stride=stride, padding=k // 2).to(d)
    conv.weight.data = conv.weight.data.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    bn_a, bn_b = BatchNorm2dAct(Cout).to(d), BatchNorm2dAct(Cout).to(d)
    x = (torch.randn(6, Cin, 30, 30, device=d) + 0.5).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y1 = conv(x, bn_stats=True)
    assert getattr(y1, "_kfa_prestats", False)
    out_a = bn_a(y1)
    y2 = conv(x)
    out_b = bn_b(y2)
    assert torch.equal(y1, y2)
    assert (out_a.float() - out_b.float()).abs().max().item() < 3e-2
    torch.testing.assert_close(bn_a.running_mean, bn_b.running_mean, atol=1e-3, rtol=1e-3)
    torch.testing.assert_close(bn_a.running_var, bn_b.running_var, atol=1e-3, rtol=1e-3)
    torch.cuda.synchronize()
    assert bn_slot_workspace(Cout, d).abs().max().item() == 0


@pytest.mark.parametrize("pp", [False, True, "512"])
@pytest.mark.parametrize("C,Cout,k,stride", [(64, 64, 3, 1), (128, 128, 3, 2), (64, 256, 1, 1), (256, 256, 3, 1)])
def test_bn_bwd_stats_fused_into_dgrad_epilogue(C, Cout, k, stride, pp, monkeypatch):
    """BN(+ReLU) -> conv: the conv's dgrad epilogue accumulates the BN's backward
    statistics (BnBwdLink); gradients match the unfused pair and the slots end clean
    (pp: the ping-pong kernel's dgrad epilogue)."""
    from kubeflow_controller_amd.ops import conv as convmod
    from kubeflow_controller_amd.ops.batchnorm import BatchNorm2dAct, bn_slot_workspace
    from kubeflow_controller_amd.ops.conv import Conv2d
    monkeypatch.setattr(convmod, "BIG", C % 256 == 0)
    if pp:
        monkeypatch.setattr(convmod, "PP", "1" if pp is True else "512")
        monkeypatch.setattr(convmod, "PP_MIN_N", 64)
    d = torch.device("cuda")
    torch.manual_seed(0)
    bn = BatchNorm2dAct(C).to(d)
    torch.nn.init.uniform_(bn.weight, 0.5, 1.5)
    torch.nn.init.uniform_(bn.bias, -0.2, 0.2)
    conv = Conv2d(C, Cout, k, stride=stride, padding=k // 2).to(d)
    conv.weight.data = conv.weight.data.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x = torch.randn(4, C, 28, 28, device=d).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = None
    grads = []
    for link in (True, False):
        xr = x.clone().requires_grad_()
        for p in list(bn.parameters()) + list(conv.parameters()):
            p.grad = None
        y = conv(bn(xr, bwd_link=link))
        if dy is None:
            dy = torch.randn_like(y)
        y.backward(dy)
        grads.append([xr.grad.float(), bn.weight.grad.clone(), bn.bias.grad.clone(), conv.weight.grad.float()])
    for a, b in zip(*grads):
        scale = max(1e-3, b.abs().max().item())
        assert (a - b).abs().max().item() < 2e-2 * scale, ((a - b).abs().max().item(), scale)
    torch.cuda.synchronize()
    assert bn_slot_workspace(C, d).abs().max().item() == 0


def test_conv_forward_tuner(monkeypatch):
    """The per-shape forward tuner: timing both forwards records a decision; a
    vendor-forward layer leaves the BN statistics to the BN (no prestats tag, slots
    clean) and matches the fused path's outputs and gradients (the backward stays on
    the implicit-GEMM dgrad / wgrad)."""
    from kubeflow_controller_amd.ops import conv as convmod
    from kubeflow_controller_amd.ops.batchnorm import BatchNorm2dAct, bn_slot_workspace
    from kubeflow_controller_amd.ops.conv import Conv2d
    d = torch.device("cuda")
    torch.manual_seed(0)
    conv = Conv2d(128, 128, 3, stride=1, padding=1).to(d)
    conv.weight.data = conv.weight.data.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x = torch.randn(4, 128, 20, 20, device=d).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    monkeypatch.setattr(convmod, "TUNE", True)
    monkeypatch.setattr(convmod, "_fwd_plan", {})
    key = (tuple(x.shape), tuple(conv.weight.shape), 1, 1, True)
    choice = convmod._use_vendor_fwd(x, conv.weight, 1, 1, bn_slot_workspace(128, d))
    assert convmod._fwd_plan[key] is choice
    torch.cuda.synchronize()
    assert bn_slot_workspace(128, d).abs().max().item() == 0  # tuning used its own scratch slots
    outs, grads = [], []
    for vendor in (True, False):
        convmod._fwd_plan[key] = vendor
        bn = BatchNorm2dAct(128).to(d)
        xr = x.clone().requires_grad_()
        conv.weight.grad = None
        y = conv(xr, bn_stats=True)
        assert getattr(y, "_kfa_prestats", False) is (not vendor)
        out = bn(y)
        out.float().square().sum().backward()
        outs.append(out.float())
        grads.append((xr.grad.float(), conv.weight.grad.float(), bn.running_mean.clone()))
    torch.cuda.synchronize()
    assert bn_slot_workspace(128, d).abs().max().item() == 0
    assert (outs[0] - outs[1]).abs().max().item() < 5e-2
    for a, b in zip(grads[0], grads[1]):
        assert (a - b).abs().max().item() < 5e-2 * max(1.0, b.abs().max().item())


@pytest.mark.parametrize("N,C,H,W,Co,k,stride,pad", [(2, 64, 14, 14, 256, 1, 1, 0), (2, 128, 14, 14, 64, 3, 2, 1),
                                                     (3, 64, 9, 9, 128, 3, 1, 1)])
def test_dgrad_masked_addend(N, C, H, W, Co, k, stride, pad):
    """Residual gradient formed in the dgrad epilogue: dx = dgrad(dy) + g * bits
    (the bits of a BN + residual + ReLU output) equals dgrad(dy) + (g * mask)."""
    from kubeflow_controller_amd.ops.conv import apply_bit_mask, conv_dgrad
    torch.manual_seed(0)
    d = torch.device("cuda")
    cl = torch.channels_last
    P = (H + 2 * pad - k) // stride + 1
    Q = (W + 2 * pad - k) // stride + 1
    dy = torch.randn(N, Co, P, Q, device=d).to(torch.bfloat16).contiguous(memory_format=cl)
    w = (torch.randn(Co, C, k, k, device=d) / (C * k * k) ** 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
    g = torch.randn(N, C, H, W, device=d).to(torch.bfloat16).contiguous(memory_format=cl)
    bits = torch.randint(0, 256, (N * C * H * W // 8,), device=d, dtype=torch.uint8)
    got = conv_dgrad(dy, w, (N, C, H, W), stride, pad, g, None, bits)
    want = conv_dgrad(dy, w, (N, C, H, W), stride, pad, apply_bit_mask(g, bits).contiguous(memory_format=cl))
    assert torch.equal(got, want)
    keep = apply_bit_mask(g, bits) != 0
    assert 0.3 < keep.float().mean().item() < 0.7  # the mask really drops elements


def test_resnet_masked_residual_gradient():
    """Identity blocks hand conv1's dgrad epilogue the raw gradient + ReLU bits
    (GradJoin.deposit_masked) instead of a written residual gradient: every
    identity block takes that path, and the gradients are as close to the fp32
    reference as with the written residual gradient.  (Not bitwise: the fp32
    BatchNorm statistics atomics make each run's order differ, and small-batch BN
    backward amplifies that.)"""
    from kubeflow_controller_amd.models.resnet import ResNet
    from kubeflow_controller_amd.ops import conv as convmod
    d = torch.device("cuda")
    torch.manual_seed(0)
    m = ResNet((3, 2, 1, 1), num_classes=10, width=64).to(d).to(memory_format=torch.channels_last)
    for p in m.parameters():
        if p.dim() >= 2:
            p.data = p.data.to(torch.bfloat16)
    for mod in m.modules():
        if hasattr(mod, "bn3"):
            torch.nn.init.uniform_(mod.bn3.weight, 0.5, 1.5)
    x = torch.randn(8, 3, 128, 128, device=d).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ref = _fp32_reference_grads(x, m)
    calls = []
    orig = convmod.GradJoin.deposit_masked

    def counting(self, grad, mask):
        ok = orig(self, grad, mask)
        calls.append(ok)
        return ok

    convmod.GradJoin.deposit_masked = counting
    try:
        masked = _stack_grads(True, True, x, m)
    finally:
        convmod.GradJoin.deposit_masked = orig
    assert len(calls) == 3 and all(calls), calls  # 2 identity blocks in layer1, 1 in layer2
    convmod.GradJoin.deposit_masked = lambda self, grad, mask: False
    try:
        plain = _stack_grads(True, True, x, m)
    finally:
        convmod.GradJoin.deposit_masked = orig
    names = ["input"] + [n for n, _ in m.named_parameters()]
    bad = []
    for n, a, b, r in zip(names, masked, plain, ref):
        r = r.to(a.device).float()
        if r.dim() == 4:
            r = r.contiguous(memory_format=torch.channels_last)
        scale = max(1e-4, r.abs().max().item())
        e_m, e_p = (a - r).abs().max().item(), (b - r).abs().max().item()
        if e_m > 2.0 * e_p + 0.02 * scale:
            bad.append((n, e_m, e_p, scale))
    assert not bad, bad


@pytest.mark.parametrize("N,H,W,C", [(2, 224, 224, 3), (3, 32, 18, 3), (2, 20, 20, 1)])
def test_stem_space_to_depth_fwd_wgrad(N, H, W, C):
    """7x7/s2/p3 few-channel stem as a 4x4 stride-1 conv over the space-to-depth
    input (stem.hip + conv_igemm C=16 + wgrad C=16 + fold) vs fp32 PyTorch;
    also its fused BatchNorm statistics."""
    from kubeflow_controller_amd.ops import _lib
    from kubeflow_controller_amd.ops.conv import conv2d, stem_ok
    torch.manual_seed(0)
    d = torch.device("cuda")
    x = torch.randn(N, C, H, W, device=d).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(64, C, 7, 7, device=d) / (C * 49) ** 0.5).to(torch.bfloat16)
    w = w.contiguous(memory_format=torch.channels_last)
    assert stem_ok(x, w, 2, 3)
    wr = w.clone().requires_grad_()
    y = conv2d(x, wr, 2, 3)
    wf = w.float().requires_grad_()
    yf = torch.nn.functional.conv2d(x.float(), wf, None, 2, 3)
    assert y.shape == yf.shape and y.is_contiguous(memory_format=torch.channels_last)
    err = (y.float() - yf).abs().max().item()
    assert err < 2e-2 * max(1.0, yf.abs().max().item()), err
    dy = torch.randn_like(yf)
    y.backward(dy.to(torch.bfloat16))
    yf.backward(dy)
    gw = (wr.grad.float() - wf.grad).abs().max().item()
    assert gw < 3e-2 * max(1.0, wf.grad.abs().max().item()), gw
    # fused BatchNorm statistics (sum, sum of squares per channel) land in the BN slots
    from kubeflow_controller_amd.ops.batchnorm import bn_slot_workspace
    ws = bn_slot_workspace(64, x.device)
    ws = ws.view(torch.float32) if ws.dtype != torch.float32 else ws
    torch.cuda.synchronize()
    ws.zero_()
    y2 = conv2d(x, w, 2, 3, bn_stats=True)
    torch.cuda.synchronize()
    slots = ws[: _lib.lib().kfa_bn_slot_floats(64)].view(-1, 2, 64).sum(0)
    yb = y2.float().permute(0, 2, 3, 1).reshape(-1, 64)
    torch.testing.assert_close(slots[0], yb.sum(0), rtol=1e-3, atol=1e-1)
    torch.testing.assert_close(slots[1], (yb * yb).sum(0), rtol=1e-3, atol=1e-1)
    ws.zero_()


def test_batched_dgrad_weight_transpose_tracks_weight_updates(monkeypatch):
    """The per-step batched dgrad weight transpose (one launch for every conv,
    refreshed after each forward) gives bit-identical training to per-call
    transposes while the optimizer changes the weights every step."""
    from kubeflow_controller_amd.ops import conv as convmod
    from kubeflow_controller_amd.ops.conv import Conv2d
    from kubeflow_controller_amd.trainer.engine import DistInfo, Engine

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = Conv2d(64, 64, 3, 1, 1)
            self.b = Conv2d(64, 128, 3, 2, 1)
            self.c = Conv2d(128, 128, 1, 2, 0)

        def forward(self, x):
            return self.c(torch.relu(self.b(torch.relu(self.a(x)))))

    def run(batched):
        monkeypatch.setattr(convmod, "BATCHED_TRANSPOSE", batched)
        convmod._tcache = convmod._TransposeCache()
        torch.manual_seed(0)
        d = torch.device("cuda")
        eng = Engine(Net(), lambda m, x: m(x).float().pow(2).mean(), optimizer="sgd", lr=0.5, momentum=0.0,
                     weight_decay=0.0, dist_info=DistInfo(device=d))
        x = torch.randn(4, 64, 16, 16, device=d).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        x.requires_grad_()
        out = []
        for _ in range(4):
            x.grad = None
            out.append(float(eng.train_step(x)))
            out.append(x.grad.float().sum().item())
        return out, [g.grad.clone() for g in eng.groups]

    a, ga = run(False)
    b, gb = run(True)
    assert a == b
    for u, v in zip(ga, gb):
        assert torch.equal(u, v)
    assert len(convmod._tcache.entries) == 6  # a: 1; b (3x3/s2): 4 parity classes; c (1x1/s2): 1 class with taps


@pytest.mark.parametrize("big", [False, True])
@pytest.mark.parametrize("N,C,H,W,Co,k", [(4, 64, 14, 14, 64, 3), (2, 128, 14, 14, 256, 1), (3, 128, 7, 9, 128, 3),
                                          (2, 64, 20, 20, 256, 1), (2, 256, 9, 11, 256, 3), (5, 64, 8, 8, 512, 1)])
@pytest.mark.parametrize("with_y", [True, False])
def test_conv_bn_apply_prologue(N, C, H, W, Co, k, big, with_y, monkeypatch):
    """conv_fwd_bnpro(x, [scale|shift]) == conv_fwd(relu(x*scale+shift)) bit for bit
    (same MFMA operands, same tile order), the fused BN statistics match, padding
    taps stay zero (relu(shift) > 0 would leak there), and the side output is
    exactly the bf16 activation bn_apply writes.  Also vs an fp32 PyTorch conv."""
    from kubeflow_controller_amd.ops import _lib
    from kubeflow_controller_amd.ops import conv as convmod
    if big and Co % 256:
        pytest.skip("256x256 tiles only for 256-multiple Cout")
    monkeypatch.setattr(convmod, "BIG", big)
    torch.manual_seed(1)
    d = torch.device("cuda")
    pad = k // 2
    x = (torch.randn(N, C, H, W, device=d) * 2).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Co, C, k, k, device=d) / (C * k * k) ** 0.5).to(torch.bfloat16)
    w = w.contiguous(memory_format=torch.channels_last)
    # the reference activation is bn_apply's own output (eval-mode BN + ReLU), ss its [scale | shift]
    gamma, beta = torch.rand(C, device=d) + 0.25, torch.randn(C, device=d) * 0.5 + 0.3  # relu(shift) > 0 mostly
    rm, rv = torch.randn(C, device=d) * 0.1, torch.rand(C, device=d) + 0.5
    coef = torch.empty(3 * C, dtype=torch.float32, device=d)
    yref = torch.empty_like(x)
    _lib.call("kfa_bn_fwd_eval", _lib.ptr(x), None, _lib.ptr(yref), _lib.ptr(gamma), _lib.ptr(beta), _lib.ptr(rm),
              _lib.ptr(rv), _lib.ptr(coef), N * H * W, C, 1e-5, 1, _lib.stream())
    ss = coef[:2 * C]
    sc, sh = ss[:C], ss[C:]
    yf = torch.relu(x.float() * sc.view(1, C, 1, 1) + sh.view(1, C, 1, 1))
    assert (yref.float() - yf).abs().max().item() <= 1e-2 * yf.abs().max().item()
    nslot = _lib.lib().kfa_bn_slot_floats(Co)
    st_a = torch.zeros(nslot, dtype=torch.float32, device=d)
    st_b = torch.zeros(nslot, dtype=torch.float32, device=d)
    y_out = torch.empty_like(x) if with_y else None
    if y_out is not None:
        y_out.fill_(float("nan"))
    out = convmod.conv_fwd_bnpro(x, ss, w, 1, pad, st_a, y_out)
    ref = convmod.conv_fwd(yref, w, 1, pad, st_b)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    if y_out is not None:
        assert torch.equal(y_out, yref)
    sa, sb = st_a.view(-1, 2 * Co).sum(0), st_b.view(-1, 2 * Co).sum(0)
    torch.testing.assert_close(sa, sb, rtol=1e-4, atol=1e-2)
    f32 = torch.nn.functional.conv2d(yref.float(), w.float(), None, 1, pad)
    assert (out.float() - f32).abs().max().item() < 2e-2 * max(1.0, f32.abs().max().item())


@pytest.mark.parametrize("cin,mid,stride", [(256, 64, 1), (128, 64, 2)])
def test_resnet_block_lazy_bn2_fused_into_conv3(cin, mid, stride, monkeypatch):
    """bn2 -> conv3 with the BN-apply folded into conv3's operand load (lazy bn2 output,
    conv_fwd_bnpro) vs the apply pass + conv: same block output and gradients, the lazy
    output is filled for the weight gradient, and the BN slot workspace ends clean."""
    import copy
    from kubeflow_controller_amd.models import resnet as R
    from kubeflow_controller_amd.ops import conv as convmod
    from kubeflow_controller_amd.ops.batchnorm import bn_slot_workspace
    torch.manual_seed(0)
    d = torch.device("cuda")
    blk = R.Bottleneck(cin, mid, stride).to(d)
    for m in blk.modules():
        if isinstance(m, convmod.Conv2d):
            m.weight.data = m.weight.data.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    for m in blk.modules():  # non-trivial BN parameters (bn3 is zero-initialised)
        if hasattr(m, "running_var"):
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.5, 0.5)
    blk2 = copy.deepcopy(blk)
    x = (torch.randn(4, cin, 20, 20, device=d)).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    calls = {"pro": 0}
    real = convmod.conv_fwd_bnpro

    def counting(*a, **k):
        calls["pro"] += 1
        return real(*a, **k)

    outs = []
    g = None
    for fused, b in ((True, blk), (False, blk2)):
        monkeypatch.setattr(convmod, "_use_bnpro", lambda *a, f=fused, **k: f)
        monkeypatch.setattr(convmod, "conv_fwd_bnpro", counting)
        xr = x.clone().requires_grad_()
        y = b(xr)
        if g is None:  # ONE output gradient for both runs
            g = torch.randn(y.shape, device=d).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y.backward(g)
        torch.cuda.synchronize()
        outs.append((y.float(), xr.grad.float(), [p.grad.float().clone() for p in b.parameters()]))
    assert calls["pro"] == 1
    (ya, ga, pa), (yb, gb, pb) = outs
    assert (ya - yb).abs().max().item() <= 2e-2 * max(1.0, yb.abs().max().item())
    assert (ga - gb).abs().max().item() <= 3e-2 * max(1.0, gb.abs().max().item())
    for u, v in zip(pa, pb):
        assert (u - v).abs().max().item() <= 3e-2 * max(1.0, v.abs().max().item())
    for C in (mid, 4 * mid):
        assert bn_slot_workspace(C, d).abs().max().item() == 0


def test_batched_weight_transpose_matches_permute():
    """The per-backward batched transpose (weight_transpose_multi, 64 x 64 vector tiles
    with an element-wise path for partial tiles / odd channel counts) over a mix of
    BERT dense weights, 3x3 conv weights with stride-2 tap subsets and odd shapes:
    exact against torch's permute after the weights change."""
    from kubeflow_controller_amd.ops.conv import _TransposeCache
    torch.manual_seed(0)
    d = torch.device("cuda")
    shapes = [((3072, 768, 1, 1), (0, 1, 1, 0, 1, 1)), ((768, 2304, 1, 1), (0, 1, 1, 0, 1, 1)),
              ((256, 128, 3, 3), (0, 1, 3, 0, 1, 3)), ((256, 128, 3, 3), (1, 2, 1, 0, 2, 2)),
              ((100, 200, 1, 1), (0, 1, 1, 0, 1, 1)), ((10, 3, 3, 3), (0, 1, 3, 0, 1, 3)),
              ((72, 136, 3, 3), (0, 2, 2, 1, 2, 1))]
    ws = [torch.randn(*s, device=d).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
          for s, _ in shapes]
    cache = _TransposeCache()
    for w, (_, a) in zip(ws, shapes):
        cache.get(w, *a)  # first use: the single-weight kernel; joins the batch after
    for w in ws:
        w.copy_(torch.randn_like(w))
    cache.mark_stale()
    for w, (shp, (r0, dr, Rs, s0, ds, Ss)) in zip(ws, shapes):
        got = cache.get(w, r0, dr, Rs, s0, ds, Ss)  # refreshed by ONE batched launch
        sub = w[:, :, r0::dr, s0::ds][:, :, :Rs, :Ss]          # [Co, Ci, Rs, Ss]
        ref = sub.permute(1, 2, 3, 0).contiguous()              # [Ci, Rs, Ss, Co]
        assert torch.equal(got.reshape(ref.shape), ref), shp


@pytest.mark.parametrize("want", ["igemm", "igemm256x64"])
def test_narrow_conv_tiles_match_fp32(want, monkeypatch):
    """The N = 64 launches on each narrow tile the router can pick — 128 x 64 ("igemm")
    and 256 x 64 ("igemm256x64", conv_igemm_kernel<4,1,4,4>): a 64-channel 3x3 conv
    forward / data / weight gradient, and the space-to-depth stem (C = 16 multi-tap
    slices), vs fp32 PyTorch."""
    import torch.nn.functional as F
    from kubeflow_controller_amd.ops import routes
    from kubeflow_controller_amd.ops.conv import Conv2d
    seen = []

    def decide(kind, key, dev, cands, margin=0.99, log=False):
        names = [n for n, _ in cands]
        seen.append(names)
        return names.index(want) if want in names else 0
    monkeypatch.setattr(routes, "decide", decide)
    d = torch.device("cuda")
    torch.manual_seed(6)
    for cin, k, stride, pad, hw in [(64, 3, 1, 1, 28), (3, 7, 2, 3, 64)]:
        conv = Conv2d(cin, 64, k, stride=stride, padding=pad).to(d)
        conv.weight.data = conv.weight.data.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        x = torch.randn(2, cin, hw, hw, device=d).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        x.requires_grad_(cin != 3)
        y = conv(x)
        dy = torch.randn_like(y)
        y.backward(dy)
        xf = x.detach().float().requires_grad_(cin != 3)
        wf = conv.weight.detach().float().requires_grad_()
        yr = F.conv2d(xf, wf, None, stride, pad)
        yr.backward(dy.float())
        for name, a, r in [("y", y, yr), ("dw", conv.weight.grad, wf.grad)] + ([("dx", x.grad, xf.grad)] if cin != 3 else []):
            err = (a.float() - r).abs().max().item()
            assert err < 3e-2 * max(1.0, r.abs().max().item()), (cin, name, err)
    assert any(want in n for n in seen), seen
