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
    """Same tiny W&D training steps with the fused input kernels and with the PyTorch chain."""
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
        eng = Engine(copy.deepcopy(base), WD.wide_deep_loss, optimizer="adam", lr=1e-2, channels_last=False,
                     dist_info=DistInfo(device=d))
        losses[fused] = [float(eng.train_step(*batch)) for _ in range(4)]
    for a, b in zip(losses[True], losses[False]):
        assert abs(a - b) < 2e-3 * max(1.0, abs(b)), losses
