"""Persistent ping-pong GEMM (csrc/kernels/gemm_ppp.hip) vs plain PyTorch fp32:
tile boundaries inside one block's k-tile stream (C of tile i written during
tile i+1's first k-tile), partial tiles at the M / N edges, one and two
k-tiles per tile, and grids capped so blocks run many (and uneven) tile counts."""
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


@pytest.mark.parametrize("M,N,K,blocks", [
    (256, 256, 128, 0),       # one tile, two k-tiles
    (512, 512, 128, 1),       # 4 tiles on one block, two k-tiles each (every k-tile a boundary one)
    (1000, 776, 192, 3),      # edge tiles in M and N, uneven tile counts per block
    (4096, 4096, 768, 0),     # one tile per CU
    (8192, 2304, 768, 0),     # 4.5 tiles per CU
    (32768, 768, 768, 0),     # BERT out-projection: 1.5 tiles per CU
    (32768, 3072, 768, 0),    # BERT FFN-up: 6 tiles per CU
    (2048, 768, 3072, 5),     # long k-loop, many tiles per block
    (1024, 1024, 4096, 64),   # grid capped at the 16 tiles, 64 k-tiles each
    (300, 8, 128, 0),         # N = 8
    (512, 512, 128, 2),       # two k-tiles per tile: every other k-tile a boundary one
])
def test_gemm_ppp_matches_fp32(M, N, K, blocks):
    from kubeflow_controller_amd.ops import gemm as G
    torch.manual_seed(M + N + K)
    a, b = _bf(M, K), _bf(N, K, s=0.05)
    c = G.gemm_ppp(a, b, blocks=blocks)
    _close(c, a.float() @ b.float().t(), 1e-2, f"C {M}x{N}x{K} blocks={blocks}")


@pytest.mark.parametrize("M,N,K,blocks", [
    (256, 192, 128, 0),       # one 256 x 192 tile, two k-tiles
    (512, 384, 128, 1),       # 4 tiles on one block: every k-tile a boundary one
    (1000, 776, 192, 3),      # edge tiles in M and N (N = 776: last tile 8 columns wide), uneven tile counts
    (32768, 768, 768, 0),     # BERT out-projection: 512 tiles = two per CU
    (32768, 768, 3072, 0),    # BERT FFN-down
    (2048, 1536, 2304, 5),    # long k-loop, many tiles per block
    (300, 200, 128, 0),       # partial nh = 1 half (columns 192..199)
])
@pytest.mark.parametrize("probe", [7, 0], ids=["four_phase", "three_phase"])
def test_gemm_ppp_bn192_matches_fp32(M, N, K, blocks, probe):
    """192-wide tiles (one-block nh = 1 halves, 8-B stores, 7 DMAs per k-tile), with the
    four-phase (probe 7) and the default three-phase k-tile schedules."""
    from kubeflow_controller_amd.ops import gemm as G
    torch.manual_seed(M + N + K + 1)
    a, b = _bf(M, K), _bf(N, K, s=0.05)
    c = G.gemm_ppp(a, b, blocks=blocks, bn=192, probe=probe)
    _close(c, a.float() @ b.float().t(), 1e-2, f"C {M}x{N}x{K} bn=192 blocks={blocks} probe={probe}")


@pytest.mark.parametrize("M,N,K,blocks,bn", [
    (32768, 768, 768, 0, 256),   # 384 tiles on 256 CUs: 128 leftover tiles in 2 k-ranges each
    (1024, 1024, 1024, 12, 256), # 16 tiles on 12 blocks: 4 leftover tiles in 3 uneven k-ranges
    (256, 512, 2048, 0, 256),    # no full round: 2 tiles x 8 k-ranges
    (256, 1000, 2048, 0, 256),   # ResNet-50 FC shape (partial last tile in N)
    (300, 200, 4096, 0, 192),    # 192-wide tiles, partial tiles in M and N, 8 k-ranges
    (5120, 768, 30528 // 64 * 64, 0, 256),  # MLM-decoder dgrad shape: 60 tiles x 4 k-ranges
])
def test_gemm_ppp_split_matches_fp32(M, N, K, blocks, bn):
    """Split remainder: partial accumulators of k-ranges combined in-kernel; run
    twice so the self-cleaning unit counters are exercised."""
    from kubeflow_controller_amd.ops import gemm as G
    torch.manual_seed(M + N + K + 2)
    a, b = _bf(M, K), _bf(N, K, s=0.05)
    ref = a.float() @ b.float().t()
    c1 = G.gemm_ppp(a, b, blocks=blocks, bn=bn)
    c2 = G.gemm_ppp(a, b, blocks=blocks, bn=bn)
    _close(c1, ref, 1e-2, f"split C {M}x{N}x{K} bn={bn}")
    assert torch.equal(c1, c2)
    c3 = G.gemm_ppp(a, b, blocks=blocks, bn=bn, split=False)
    _close(c3, ref, 1e-2, f"unsplit C {M}x{N}x{K} bn={bn}")


def test_gemm_ppp_strided_a_and_repeatable():
    """Row stride > K on A (a column slice); two launches give identical bits."""
    from kubeflow_controller_amd.ops import gemm as G
    torch.manual_seed(1)
    big = _bf(3000, 1024)
    a = big[:, 128:128 + 640]
    b = _bf(1000, 640, s=0.05)
    c1 = G.gemm_ppp(a, b, blocks=7)
    c2 = G.gemm_ppp(a, b, blocks=7)
    assert torch.equal(c1, c2)
    _close(c1, a.float() @ b.float().t(), 1e-2, "strided")


@pytest.mark.parametrize("probe", [2, 3, 4], ids=["writeback_stores", "row_pairs", "row_pairs_nt"])
def test_gemm_ppp_store_policies(probe):
    """The store-policy builds (non-temporal C stores, whole-row store phases) write the same C."""
    from kubeflow_controller_amd.ops import gemm as G
    torch.manual_seed(probe)
    a, b = _bf(1000, 640), _bf(776, 640, s=0.05)
    c = G.gemm_ppp(a, b, blocks=3, probe=probe)
    _close(c, a.float() @ b.float().t(), 1e-2, f"probe {probe}")


def test_gemm_ppp_split_under_cu_hog():
    """Forward progress without co-residency: a diagnostic kernel holds all but 32
    CUs for 1 s on another stream while the split-remainder shapes run.  With the
    last-arriver combine no block waits for another, so the GEMMs finish on the CUs
    that are left, before the hog ends, bit-identical to the unloaded runs."""
    from kubeflow_controller_amd.ops import _lib
    from kubeflow_controller_amd.ops import gemm as G
    _lib.register("kfa_cu_hog", [_lib.I, _lib.L, _lib.P, _lib.P])
    shapes = [(32768, 768, 768), (256, 1000, 2048), (1024, 1024, 1024), (5120, 768, 30528 // 64 * 64)]
    torch.manual_seed(7)
    ops = [(_bf(M, K), _bf(N, K, s=0.05)) for M, N, K in shapes]
    for (a, b), (M, N, K) in zip(ops, shapes):
        assert _lib.lib().kfa_gemm_ppp_ws_bytes(M, N, K, 256, 0) > 0, f"{M}x{N}x{K} should take the split path"
    ref = [G.gemm_ppp(a, b, bn=256) for a, b in ops]
    torch.cuda.synchronize()
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    nhog = ncu - 32
    hog_s, gemm_s = torch.cuda.Stream(), torch.cuda.Stream()
    flags = torch.zeros(nhog, dtype=torch.int32, device=D)
    with torch.cuda.stream(hog_s):
        _lib.call("kfa_cu_hog", nhog, 1_000_000, _lib.ptr(flags), _lib.stream())
        hog_done = torch.cuda.Event()
        hog_done.record(hog_s)
    with torch.cuda.stream(gemm_s):
        out = [G.gemm_ppp(a, b, bn=256) for a, b in ops]
        gemm_done = torch.cuda.Event()
        gemm_done.record(gemm_s)
    gemm_done.synchronize()
    finished_under_hog = not hog_done.query()
    hog_done.synchronize()
    torch.cuda.synchronize()
    assert (flags.cpu() == (torch.arange(nhog) * 7 % 64 + 1).int()).all(), "hog kernel did not run to completion"
    for r, o, s in zip(ref, out, shapes):
        assert torch.equal(r, o), f"split GEMM {s} under load differs from the unloaded run"
    assert finished_under_hog, "split GEMMs waited for the hog kernel to release its CUs"


@pytest.mark.parametrize("M,N,K,splits,bias", [
    (256, 1000, 2048, 0, True),    # ResNet-50 FC forward (bias fused)
    (256, 2048, 1000, 0, False),   # its data gradient: K = 1000, a partial last k-step
    (256, 1000, 2048, 1, True),    # one slice: no partial exchange
    (100, 64, 520, 3, False),      # M < 256, uneven slices, k tail
    (256, 4, 8, 0, True),          # tiny
    (200, 1024, 4096, 16, False),  # many slices
    (5120, 768, 768, 0, True),     # BERT MLM transform: 20 row bands x 12 tiles, no split
    (1000, 200, 2048, 0, False),   # 4 bands (partial last), split slices over bands
    (777, 96, 3000, 2, True),      # partial band, partial tile, k tail, 2 slices
])
def test_gemm_skinny_matches_fp32(M, N, K, splits, bias):
    """Split-K skinny GEMM (csrc/kernels/gemm_skinny.hip): partials of K slices summed by
    the last-arriving slice in slice order (bit-identical run to run), bias fused;
    M > 256 as several 256-row bands."""
    from kubeflow_controller_amd.ops import gemm as G
    torch.manual_seed(M + N + K)
    a, b = _bf(M, K), _bf(N, K, s=0.05)
    bv = torch.randn(N, device=D) if bias else None
    ref = a.float() @ b.float().t() + (bv if bias else 0)
    c1 = G.gemm_skinny(a, b, bv, splits=splits)
    c2 = G.gemm_skinny(a, b, bv, splits=splits)
    _close(c1, ref, 1e-2, f"skinny {M}x{N}x{K} s={splits}")
    assert torch.equal(c1, c2)


def test_dense_layer_small_batch_routes_own():
    """The ResNet-50 FC shape through Linear: the per-shape tuner times the skinny
    kernel against hipBLASLt; forward and both gradients match fp32 either way."""
    from kubeflow_controller_amd.ops.linear import Linear
    torch.manual_seed(0)
    lin = Linear(2048, 1000).cuda()
    x = torch.randn(256, 2048, device=D).to(torch.bfloat16).requires_grad_()
    w = lin.weight.detach().to(torch.bfloat16)
    lin.weight.data = w
    y = lin(x)
    g = torch.randn_like(y)
    y.backward(g)
    xr = x.detach().float().requires_grad_()
    wr = w.float().requires_grad_()
    br = lin.bias.detach().float().requires_grad_()
    yr = xr @ wr.t() + br
    yr.backward(g.float())
    _close(y, yr, 2e-2, "fc fwd")
    _close(x.grad, xr.grad, 2e-2, "fc dgrad")
    _close(lin.bias.grad, br.grad, 2e-2, "fc dbias")


@pytest.mark.parametrize("M,N,K,blocks", [
    (256, 256, 128, 0),       # one tile: only the after-loop stores
    (512, 512, 128, 1),       # 4 tiles on one block, every k-tile a boundary one (hand-off each phase)
    (1000, 776, 192, 3),      # edge tiles in M and N, uneven tile counts per block
    (8192, 2304, 768, 0),     # 4.5 tiles per CU
    (32768, 3072, 768, 0),    # BERT FFN-up: 6 tiles per CU
    (2048, 768, 3072, 5),     # long k-loop, many tiles per block
    (300, 8, 128, 0),         # N = 8
])
@pytest.mark.parametrize("probe", [9, 10], ids=["ppw", "ppw_nt"])
def test_gemm_ppw_matches_fp32(M, N, K, blocks, probe):
    """Wave-specialised persistent GEMM (gemm_ppw_kernel): group 0 issues every LDS-DMA
    piece and hands its C quadrants to group 1 through LDS, group 1 issues every C store."""
    from kubeflow_controller_amd.ops import gemm as G
    torch.manual_seed(M + N + K + 3)
    a, b = _bf(M, K), _bf(N, K, s=0.05)
    c = G.gemm_ppp(a, b, blocks=blocks, probe=probe, split=False)
    _close(c, a.float() @ b.float().t(), 1e-2, f"ppw {M}x{N}x{K} blocks={blocks} probe={probe}")
    c2 = G.gemm_ppp(a, b, blocks=blocks, probe=probe, split=False)
    assert torch.equal(c, c2)


@pytest.mark.parametrize("M,N,K", [
    (65536, 1024, 1680),   # W&D MLP layer 1 forward: K = 26.25 k-tiles
    (1000, 776, 200),      # partial k-tile of 8 columns + edge tiles in M and N
    (512, 512, 136),       # two k-tiles, the second one 8 deep
    (256, 512, 2056),      # split units whose last range ends in the partial k-tile
])
@pytest.mark.parametrize("form", ["ppp256", "ppp192", "split", "ppw", "ppw_nt"])
def test_gemm_ppp_k_tail_matches_fp32(M, N, K, form):
    """K % 64 != 0: the last k-tile's chunks past K are read as zeros on every kernel
    form.  A and B are row-packed (lda = ldb = K), so what lies past K in a row is the
    next row's data: reading it instead of zeros would show in C."""
    from kubeflow_controller_amd.ops import gemm as G
    torch.manual_seed(M + N + K + 9)
    a, b = _bf(M, K), _bf(N, K, s=0.05)
    kw = {"ppp256": dict(bn=256, split=False), "ppp192": dict(bn=192), "split": dict(bn=256),
          "ppw": dict(probe=9, split=False), "ppw_nt": dict(probe=10, split=False)}[form]
    c = G.gemm_ppp(a, b, **kw)
    _close(c, a.float() @ b.float().t(), 1e-2, f"K-tail C {M}x{N}x{K} {form}")


@pytest.mark.parametrize("M,N,K", [
    (32768, 3072, 768),    # BERT-base FFN-up: 6 tiles per CU
    (1000, 776, 200),      # edge tiles in M and N, K tail
    (512, 512, 128),       # 4 tiles, two k-tiles each (every other k-tile a boundary one)
    (300, 8192, 256),      # the widest bias the LDS stage holds
])
def test_gemm_ppp_gelu_epilogue_matches_fp32(M, N, K):
    """Persistent GEMM with the bias + GELU epilogue (8 stores per phase in the counted
    retire waits): z = A·Bᵀ + bias and y = gelu(z) vs fp32; y is GELU of the stored bf16 z."""
    import torch.nn.functional as F
    from kubeflow_controller_amd.ops import gemm as G
    torch.manual_seed(M + N + K + 11)
    a, b = _bf(M, K), _bf(N, K, s=0.05)
    bias = torch.randn(N, device=D)
    y, z = G.gemm_ppp_gelu(a, b, bias)
    zr = a.float() @ b.float().t() + bias
    _close(z, zr, 1e-2, f"z {M}x{N}x{K}")
    _close(y, F.gelu(z.float()), 1e-2, f"y {M}x{N}x{K}")
    y2, z2 = G.gemm_ppp_gelu(a, b, bias)
    assert torch.equal(y, y2) and torch.equal(z, z2)


@pytest.mark.parametrize("M,N,K", [
    (65536, 512, 1024),    # W&D MLP layer 1: two tiles per CU
    (65536, 1024, 1680),   # W&D layer 0: K % 64 != 0 (a partial last k-tile)
    (1000, 776, 200),      # edge tiles in M and N, K tail
    (300, 8192, 256),      # the widest bias the LDS stage holds
])
def test_gemm_ppp_relu_epilogue_matches_fp32(M, N, K):
    """Persistent GEMM with the bias + ReLU epilogue (y only, the plain store count):
    y = relu(A·Bᵀ + bias) vs fp32, run to run bit-identical."""
    from kubeflow_controller_amd.ops import gemm as G
    torch.manual_seed(M + N + K + 13)
    a, b = _bf(M, K), _bf(N, K, s=0.05)
    bias = torch.randn(N, device=D)
    y = G.gemm_ppp_relu(a, b, bias)
    _close(y, torch.relu(a.float() @ b.float().t() + bias), 1e-2, f"y {M}x{N}x{K}")
    assert torch.equal(y, G.gemm_ppp_relu(a, b, bias))


@pytest.mark.parametrize("M,N,K", [
    (65536, 1024, 1680),   # W&D layer 0: four tiles per CU, K % 64 != 0
    (65536, 256, 512),     # W&D layer 2: one tile column
    (1000, 776, 200),      # edge tiles in M and N, K tail
])
@pytest.mark.parametrize("nt", [False, True])
def test_gemm_ppw_relu_epilogue_matches_fp32(M, N, K, nt):
    """Wave-specialised persistent GEMM with the bias + ReLU store epilogue
    (gemm_ppw_kernel<NT, false, 2>): y = relu(bf16(A·Bᵀ) + bias) vs fp32, equal to the
    plain ppw GEMM + the bias/ReLU pass (the same bf16 product), run to run bit-identical."""
    from kubeflow_controller_amd.ops import gemm as G
    torch.manual_seed(M + N + K + 17)
    a, b = _bf(M, K), _bf(N, K, s=0.05)
    bias = torch.randn(N, device=D)
    y = G.gemm_ppw_relu(a, b, bias, nt=nt)
    _close(y, torch.relu(a.float() @ b.float().t() + bias), 1e-2, f"y {M}x{N}x{K}")
    ref = torch.relu(G.gemm_ppp(a, b, probe=10 if nt else 9, split=False).float() + bias).to(torch.bfloat16)
    assert torch.equal(y, ref)
    assert torch.equal(y, G.gemm_ppw_relu(a, b, bias, nt=nt))


@pytest.mark.parametrize("route", ["ppp256-relu", "ppw256-relu", "ppw256-nt-relu"])
def test_dense_relu_epilogue_route_forward_backward(monkeypatch, route):
    """The dense layer on the ReLU-epilogue route (forced): output, and the input / weight /
    bias gradients (the backward masks by y > 0 instead of the pre-activation) vs fp32."""
    from kubeflow_controller_amd.ops import gemm as G
    from kubeflow_controller_amd.ops.transformer import dense
    monkeypatch.setattr(G, "ROUTE_AUTO", True)
    picked = []
    forced = [route]

    def pick(kind, key, device, cands):  # the forward's ReLU-epilogue candidate; library elsewhere
        names = [n for n, _ in cands]
        if kind == "dense_fwd":
            picked.append(names)
            return names.index(forced[0])
        return 0
    monkeypatch.setattr(G, "pick_fastest", pick)
    torch.manual_seed(5)
    M, N, K = 4096, 512, 1024
    x = _bf(M, K).requires_grad_()
    w = (torch.randn(N, K, device=D) * 0.03).to(torch.bfloat16).requires_grad_()
    b = torch.randn(N, device=D).requires_grad_()
    y = dense(x, w, b, act="relu")
    dy = _bf(M, N)
    y.backward(dy)
    assert picked and route in picked[0]
    if route.startswith("ppw"):
        # the store epilogue adds the bias to the bf16 product, as the plain ppw GEMM + the
        # bias/ReLU pass does: bit-equal to that route, forward and backward (vs fp32 the
        # mask differs where z rounds across 0, as for every library + pass route)
        forced[0] = route[:-len("-relu")]
        xc, wc, bc = (t.detach().clone().requires_grad_() for t in (x, w, b))
        yc = dense(xc, wc, bc, act="relu")
        yc.backward(dy)
        assert torch.equal(y, yc) and torch.equal(x.grad, xc.grad)
        assert torch.equal(w.grad, wc.grad)
        # the bias column sums: same values, the per-block partial sums may land in another order
        torch.testing.assert_close(b.grad, bc.grad, rtol=1e-5, atol=1e-4)
        return
    xf, wf, bf = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = torch.relu(xf @ wf.t() + bf)
    yr.backward(dy.float())
    _close(y, yr, 1e-2, "y")
    _close(x.grad, xf.grad, 2e-2, "dx")
    _close(w.grad, wf.grad, 2e-2, "dw")
    _close(b.grad, bf.grad, 2e-2, "db")


@pytest.mark.parametrize("M,N,K", [(4096, 3072, 768), (1000, 520, 136), (777, 256, 256), (2048, 1024, 512)])
@pytest.mark.parametrize("with_bias", [True, False])
@pytest.mark.parametrize("nt", [False, True])
def test_ppw_gelu_backward_epilogue(M, N, K, with_bias, nt):
    """gemm_ppw_dact: dz = (a @ b.T) * gelu'(z + bias) and dbias += colsum(dz), vs fp32
    PyTorch (exact-erf GELU derivative) and vs the unfused bias_act_bwd path."""
    from kubeflow_controller_amd.ops import gemm as G
    from kubeflow_controller_amd.ops.transformer import bias_act_bwd
    torch.manual_seed(3)
    d = torch.device("cuda")
    a = (torch.randn(M, K, device=d) / K ** 0.25).to(torch.bfloat16)
    b = (torch.randn(N, K, device=d) / K ** 0.25).to(torch.bfloat16)
    z = torch.randn(M, N, device=d).to(torch.bfloat16)
    bias = torch.randn(N, device=d) * 0.5 if with_bias else None
    dbias = torch.full((N,), 0.25, device=d)
    dz = G.gemm_ppw_dact(a, b, z, bias, dbias, nt=nt)
    zf = z.float() + (bias if with_bias else 0.0)
    x = zf / 2 ** 0.5
    gp = 0.5 * (1 + torch.erf(x)) + zf * torch.exp(-x * x) / (2 * torch.pi) ** 0.5
    c = (a.float() @ b.float().t()).to(torch.bfloat16).float()
    ref = c * gp
    err = (dz.float() - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item() + 1e-2, err
    dref = 0.25 + ref.sum(0)
    torch.testing.assert_close(dbias, dref, rtol=2e-3, atol=2e-2 * (M ** 0.5))
    # the unfused path (same bf16 product -> same GELU' arithmetic)
    db2 = torch.full((N,), 0.25, device=d)
    dz2 = bias_act_bwd(c.to(torch.bfloat16), z, bias, "gelu", db2)
    assert (dz.float() - dz2.float()).abs().max().item() <= 2e-2 * dz2.float().abs().max().item() + 1e-2


@pytest.mark.parametrize("M,N,K,blocks", [
    (256, 192, 128, 0),       # one tile: two k-tiles, the second LAST (2/3 of C in-loop), block 2 after
    (512, 384, 128, 1),       # 4 tiles on one block, two k-tiles each: every k-tile EPI or LAST
    (1000, 776, 192, 3),      # edge tiles in M and N (last tile 8 columns wide), uneven tile counts
    (32768, 768, 768, 0),     # BERT out-projection / 768 x 768 dgrad: 512 tiles = two per CU
    (32768, 768, 3072, 0),    # BERT FFN-down / FFN-up dgrad
    (32768, 768, 2304, 0),    # BERT QKV dgrad
    (2048, 1536, 2304, 5),    # long k-loop, many tiles per block
    (300, 200, 128, 0),       # block 2 of the second tile column past N (8 columns of 192)
    (1000, 776, 200, 0),      # K tail: a partial last k-tile of 8
])
@pytest.mark.parametrize("probe", [11, 12], ids=["ppw192", "ppw192_nt"])
def test_gemm_ppw192_matches_fp32(M, N, K, blocks, probe):
    """Wave-specialised 256 x 192 three-phase GEMM (gemm_ppw3_kernel): group 0 issues
    every LDS-DMA piece (14 in flight), group 1 every C store; rows 0-127 x blocks 0-1
    of a tile written during its own last k-tile, block 2 during the next tile's first."""
    from kubeflow_controller_amd.ops import gemm as G
    torch.manual_seed(M + N + K + 11)
    a, b = _bf(M, K), _bf(N, K, s=0.05)
    c = G.gemm_ppp(a, b, blocks=blocks, probe=probe, split=False)
    _close(c, a.float() @ b.float().t(), 1e-2, f"ppw192 {M}x{N}x{K} blocks={blocks} probe={probe}")
    c2 = G.gemm_ppp(a, b, blocks=blocks, probe=probe, split=False)
    assert torch.equal(c, c2)
