"""Hand-written MFMA dense GEMM + fused epilogues (csrc/kernels/gemm.hip) vs plain PyTorch fp32."""
import pytest
import torch

pytestmark = pytest.mark.gpu

D = torch.device("cuda")


def _close(a, b, tol, what=""):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    scale = max(1.0, b.abs().max().item())
    assert err <= tol * scale, f"{what}: err {err} scale {scale}"


def _bf(*shape, s=1.0):
    return (torch.randn(*shape, device=D) * s).to(torch.bfloat16)


@pytest.fixture(params=[1, 0, 2, 3, 5, 6], ids=["persistent", "per_tile", "four_wave", "two_per_cu", "pingpong",
                                          "pingpong_nt"], autouse=True)
def _persistent(request, monkeypatch):
    """Every test runs on every GEMM kernel: the persistent tile-sweeping one,
    the one-8-wave-block-per-tile one, the 4-wave 128 x 128-wave-tile one, the
    two-blocks-per-CU 256 x 128 one and the 256 x 256 ping-pong one, with plain
    and non-temporal stores (both fall back to variant 4 when K % 64 != 0)."""
    from kubeflow_controller_amd.ops import gemm as G
    monkeypatch.setattr(G, "PERSISTENT", request.param)
    return request.param


@pytest.mark.parametrize("M,N,K,bn", [(32768, 768, 768, 256), (20000, 2048, 64, 256), (9000, 1152, 96, 128),
                                      (65536, 256, 128, 128)])
def test_gemm_nt_many_tiles_per_block(M, N, K, bn):
    """More tiles than CUs: the persistent kernel carries its LDS ring across
    tiles (K = 64 / 96: an epilogue every 2 / 3 k-steps inside the vmcnt window)."""
    from kubeflow_controller_amd.ops import gemm as G
    torch.manual_seed(5)
    a, b = _bf(M, K), _bf(N, K, s=0.05)
    bias = torch.randn(N, device=D)
    c, z = G.gemm_nt(a, b, bn=bn, bias=bias, act="gelu", want_z=True)
    zr = a.float() @ b.float().t() + bias
    _close(z, zr, 1e-2, f"Z {M}x{N}x{K}")
    _close(c, torch.nn.functional.gelu(zr), 1e-2, f"C {M}x{N}x{K}")


@pytest.mark.parametrize("M,N,K,bn", [(256, 256, 32, 256), (256, 128, 64, 128), (1000, 776, 96, 128),
                                      (333, 2304, 768, 0), (4096, 768, 3072, 128), (2048, 3072, 768, 256),
                                      (513, 136, 1680, 0), (40, 8, 8, 0)])
def test_gemm_nt_plain(M, N, K, bn):
    from kubeflow_controller_amd.ops import gemm as G
    torch.manual_seed(0)
    a, b = _bf(M, K), _bf(N, K, s=0.05)
    c, z = G.gemm_nt(a, b, bn=bn)
    assert z is None
    _close(c, a.float() @ b.float().t(), 1e-2, f"C {M}x{N}x{K}")


def test_gemm_nt_strided_operands():
    from kubeflow_controller_amd.ops import gemm as G
    torch.manual_seed(1)
    big = _bf(700, 1024)
    a = big[:, 128:128 + 512]           # lda = 1024
    b = _bf(384, 768, s=0.05)[:, 256:]  # ldb = 768, K = 512
    c, _ = G.gemm_nt(a, b)
    _close(c, a.float() @ b.float().t(), 1e-2, "strided")


@pytest.mark.parametrize("act", ["gelu", "relu", "tanh"])
def test_gemm_bias_act_and_preactivation(act):
    from kubeflow_controller_amd.ops import gemm as G
    torch.manual_seed(2)
    M, N, K = 777, 1024, 256
    a, b = _bf(M, K), _bf(N, K, s=0.05)
    bias = torch.randn(N, device=D)
    y, z = G.gemm_nt(a, b, bias=bias, act=act, want_z=True)
    yr, zr = G.gemm_reference(a, b, bias=bias, act=act)
    _close(z, zr, 1e-2, "Z")
    _close(y, yr, 1e-2, "Y")


def test_gemm_dgrad_with_activation_backward_and_dbias():
    """dgrad of a GELU layer: C = (dy · W) * gelu'(z), db += colsum(C); plus the addend join."""
    from kubeflow_controller_amd.ops import gemm as G
    torch.manual_seed(3)
    M, Nout, Kin = 1111, 768, 3072
    dy, w = _bf(M, Nout), _bf(Nout, Kin, s=0.05)
    wt = G.transpose(w)
    assert torch.equal(wt, w.t().contiguous())
    z = _bf(M, Kin)
    db = torch.zeros(Kin, device=D)
    c, _ = G.gemm_nt(dy, wt, zin=z, dact="gelu", dbias=db)
    ref, _ = G.gemm_reference(dy, wt, zin=z, dact="gelu")
    _close(c, ref, 1e-2, "dgrad*gelu'")
    _close(db, c.float().sum(0), 1e-3, "dbias")
    e = _bf(M, Kin)
    c2, _ = G.gemm_nt(dy, wt, addend=e)
    _close(c2, dy.float() @ w.float() + e.float(), 1e-2, "addend")


def test_dense_layer_uses_fused_gemm_and_matches_reference(monkeypatch):
    from kubeflow_controller_amd.ops import gemm as G
    from kubeflow_controller_amd.ops import transformer as T
    monkeypatch.setattr(G, "ROUTE_LAYERS", True)
    torch.manual_seed(4)
    x = _bf(512, 768).requires_grad_()
    w = _bf(768, 768, s=0.05).requires_grad_()
    b = (torch.randn(768, device=D) * 0.1).requires_grad_()
    y = T.dense(x, w, b, "gelu")
    dy = torch.randn(512, 768, device=D)
    y.backward(dy.to(torch.bfloat16))
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = T.dense_reference(xr, wr, br, "gelu")
    yr.backward(dy)
    _close(y, yr, 2e-2, "y")
    _close(x.grad, xr.grad, 3e-2, "dx")
    _close(w.grad, wr.grad, 3e-2, "dw")
    _close(b.grad, br.grad, 3e-2, "db")


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (300, 520, 128), (4096, 4096, 3072), (33000, 776, 768),
                                   (777, 2304, 192), (32768, 3072, 768)])
@pytest.mark.parametrize("variant", [5, 6])
def test_gemm_pingpong_shapes(M, N, K, variant, _persistent):
    """Ping-pong kernel: one k-tile (prologue + tail only), M / N tails (rows
    past the operand read as zero by the buffer range check), deep K (many
    steady-state k-tiles), BERT shapes; bias + GELU + pre-activation epilogue."""
    from kubeflow_controller_amd.ops import gemm as G
    torch.manual_seed(7)
    a, b = _bf(M, K), _bf(N, K, s=0.05)
    bias = torch.randn(N, device=D)
    if _persistent != 0:
        pytest.skip("shape sweep runs once (explicit variant)")
    c, z = G.gemm_nt(a, b, bias=bias, act="gelu", want_z=True, persistent=variant)
    zr = a.float() @ b.float().t() + bias
    _close(z, zr, 1e-2, f"Z {M}x{N}x{K}")
    _close(c, torch.nn.functional.gelu(zr), 1e-2, f"C {M}x{N}x{K}")


@pytest.mark.parametrize("route", [False, True])
def test_linear_module_runs_hip_dense_and_matches_fp32(route, monkeypatch, _persistent):
    """ops.linear.Linear (ResNet FC, MNIST hidden layer) on bf16 CUDA input goes
    through DenseFn: own GEMM + fused bias epilogue (route) or library GEMM +
    the fused bias pass; dW by wgrad_kernel, db by column sums — vs fp32."""
    if _persistent != 0:
        pytest.skip("runs once")
    from kubeflow_controller_amd.ops import gemm as G
    from kubeflow_controller_amd.ops.linear import Linear
    monkeypatch.setattr(G, "ROUTE_LAYERS", route)
    torch.manual_seed(11)
    lin = Linear(2048, 1000).to(D)
    x = _bf(256, 2048).requires_grad_()
    y = lin(x)
    assert y.dtype == torch.bfloat16 and y.shape == (256, 1000)
    dy = torch.randn(256, 1000, device=D)
    y.backward(dy.to(torch.bfloat16))
    xr = x.detach().float().requires_grad_()
    wr = lin.weight.detach().to(torch.bfloat16).float().requires_grad_()
    br = lin.bias.detach().float().requires_grad_()
    yr = torch.nn.functional.linear(xr, wr, br)
    yr.backward(dy)
    _close(y, yr, 2e-2, "y")
    _close(x.grad, xr.grad, 3e-2, "dx")
    _close(lin.weight.grad, wr.grad, 3e-2, "dw")
    _close(lin.bias.grad, br.grad, 3e-2, "db")


def test_dense_auto_route_matches_fp32(monkeypatch):
    """KFA_GEMM=auto: a Linear layer times its candidates (hipBLASLt, the fused-epilogue
    GEMM, the persistent GEMM variants) once per shape, forward and dgrad, records the
    choice, and its outputs / gradients match fp32 whichever wins."""
    from kubeflow_controller_amd.ops import gemm as G
    from kubeflow_controller_amd.ops.linear import Linear
    monkeypatch.setattr(G, "ROUTE_AUTO", True)
    monkeypatch.setattr(G, "ROUTE_LAYERS", False)
    monkeypatch.setattr(G, "ROUTE_FUSED", False)
    monkeypatch.setattr(G, "_choice", {})
    torch.manual_seed(0)
    d = torch.device("cuda")
    lin = Linear(512, 1024).to(d)  # dgrad K = 1024: a persistent-GEMM candidate too
    x = torch.randn(256, 512, device=d).to(torch.bfloat16).requires_grad_()
    y = lin(x)
    y.float().pow(2).mean().backward()
    kinds = {k[0] for k in G._choice}
    assert kinds == {"dense_fwd", "dense_dgrad"}, G._choice
    xr = x.detach().float().requires_grad_()
    wr = lin.weight.detach().to(torch.bfloat16).float().requires_grad_()
    br = lin.bias.detach().float().requires_grad_()
    yr = xr @ wr.t() + br
    yr.pow(2).mean().backward()
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=2e-2)
    err = (x.grad.float() - xr.grad).abs().max().item() / xr.grad.abs().max().item()
    assert err < 3e-2, err


@pytest.mark.parametrize("pick", [0, 1, 2, 3, 4, 99])  # 99: the last candidate (skinny)
def test_dense_every_route_matches_fp32(monkeypatch, pick):
    """Each DenseFn forward candidate (hipBLASLt + bias/act pass, fused-epilogue GEMM,
    persistent GEMM variants + bias/act pass) and each dgrad candidate, forced."""
    from kubeflow_controller_amd.ops import gemm as G
    from kubeflow_controller_amd.ops import transformer as T
    monkeypatch.setattr(G, "ROUTE_AUTO", True)
    monkeypatch.setattr(G, "ROUTE_LAYERS", False)
    monkeypatch.setattr(G, "ROUTE_FUSED", False)
    monkeypatch.setattr(G, "_choice", {})
    monkeypatch.setattr(G, "pick_fastest", lambda kind, key, dev, c: min(pick, len(c) - 1))
    torch.manual_seed(pick)
    d = torch.device("cuda")
    x = torch.randn(1000, 768, device=d).to(torch.bfloat16).requires_grad_()
    w = (torch.randn(1536, 768, device=d) * 0.03).to(torch.bfloat16).requires_grad_()
    b = torch.randn(1536, device=d).requires_grad_()
    y = T.dense(x, w, b, "gelu")
    dy = torch.randn_like(y)
    y.backward(dy)
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = torch.nn.functional.gelu(xr @ wr.t() + br)
    yr.backward(dy.float())
    _close(y, yr, 2e-2, "y")
    _close(x.grad, xr.grad, 3e-2, "dx")
    _close(w.grad, wr.grad, 3e-2, "dw")
    _close(b.grad, br.grad, 3e-2, "db")
