"""Owner-side sparse optimizers of ShardedEmbedding on the GPU (segment-reduce
kernels of csrc/kernels/segsparse.hip, and the scatter-add + atomic-exchange
kernels of csrc/kernels/sparse.hip) vs the plain-PyTorch fp32 reference
``ShardedEmbedding._apply_cpu``: duplicate ids, hot rows spanning hundreds of
64-entry chunks, rows never looked up, several steps."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ids(n, rows, seed):
    g = torch.Generator().manual_seed(seed)
    u = torch.rand(n, generator=g)
    ids = torch.clamp((rows ** u).long() - 1, 0, rows - 1)   # power law: id 0 ~ log2/log(rows) of the batch
    ids[: n // 4] = 3                                        # one row spanning n/4 sorted entries
    ids[n // 4: n // 4 + 7] = rows - 1                       # a short run at the very end of the key range
    return ids[torch.randperm(n, generator=g)]


@pytest.mark.parametrize("optimizer", ["adam", "sgd"])
@pytest.mark.parametrize("dim,atomic,overlap", [(72, "0", False), (72, "0", True), (16, "0", True), (72, "1", False),
                                                (12, "0", False)],
                         ids=["seg72", "seg72_side_stream_sort", "seg16_side_stream_sort", "atomic72", "fallback12"])
def test_sparse_update_matches_cpu_reference(optimizer, dim, atomic, overlap, monkeypatch):
    from kubeflow_controller_amd.parallel.embedding import ShardedEmbedding
    monkeypatch.setenv("KFA_SPARSE_ATOMIC", atomic)
    rows = 5000
    gpu = ShardedEmbedding(rows, dim, optimizer=optimizer, lr=1e-2, weight_decay=0.01, device="cuda")
    cpu = ShardedEmbedding(rows, dim, optimizer=optimizer, lr=1e-2, weight_decay=0.01, device="cpu")
    gpu.grad_scale = cpu.grad_scale = 0.5
    with torch.no_grad():
        cpu.weight.copy_(gpu.weight.cpu())
    for step, n in enumerate((40000, 63, 1, 20001)):
        ids = _ids(n, rows, step)
        g = torch.randn(n, dim).to(torch.bfloat16)
        ids_d = ids.cuda()
        prep = gpu.prepare_sparse(ids_d) if overlap else None
        assert (prep is not None) == (overlap and dim % 8 == 0)
        gpu.apply_sparse(ids_d, g.cuda(), prep=prep)
        cpu.apply_sparse(ids, g.float())
        torch.cuda.synchronize()
        torch.testing.assert_close(gpu.weight.detach().cpu(), cpu.weight.detach(), atol=2e-5, rtol=1e-4,
                                   msg=lambda m: f"step {step} n {n}: {m}")
        if optimizer == "adam":
            torch.testing.assert_close(gpu.exp_avg.cpu(), cpu.exp_avg, atol=1e-5, rtol=1e-4)
            torch.testing.assert_close(gpu.exp_avg_sq.cpu(), cpu.exp_avg_sq, atol=1e-6, rtol=1e-4)
    untouched = torch.ones(rows, dtype=torch.bool)
    for step, n in enumerate((40000, 63, 1, 20001)):
        untouched[_ids(n, rows, step)] = False
    assert untouched.any()


def test_segment_slots_are_left_zero():
    """The per-chunk slot buffer is self-cleaning: after an update every slot is 0
    again, so the next step (any batch size) starts from a zeroed buffer."""
    from kubeflow_controller_amd.ops import _lib
    from kubeflow_controller_amd.parallel.embedding import ShardedEmbedding
    emb = ShardedEmbedding(1000, 72, device="cuda")
    ids = _ids(30000, 1000, 7).cuda()
    emb.apply_sparse(ids, torch.randn(30000, 72, device="cuda").to(torch.bfloat16))
    torch.cuda.synchronize()
    slots = _lib.workspace(0, emb.weight.device, f"seg_sparse_slots{id(emb)}")
    assert int(torch.count_nonzero(slots)) == 0


@pytest.mark.parametrize("n,nbits", [(1, 5), (1000, 3), (8192, 9), (8193, 17), (100003, 25), (1_700_000, 25),
                                     (300000, 32)])
def test_own_radix_sort_pairs_matches_stable_sort(n, nbits):
    """csrc/kernels/radix_sort.h (the id sort of the segment-reduce update, replacing
    hipCUB): keys and carried values equal a stable sort on the low nbits bits."""
    from kubeflow_controller_amd.ops import _lib
    _lib.register("kfa_radix_ws_bytes", [_lib.L], restype=_lib.L)
    _lib.register("kfa_radix_sort_pairs", [_lib.P, _lib.P, _lib.L, _lib.I, _lib.P, _lib.L, _lib.P])
    g = torch.Generator().manual_seed(n + nbits)
    hi = 1 << min(nbits, 31)
    keys = torch.randint(0, hi, (n,), generator=g, dtype=torch.int64)
    keys[: n // 3] = keys[: n // 3] % 97   # many duplicates: stability matters
    if nbits == 32:
        keys = keys * 2 + 1                 # use the top bit too
    k32 = keys.to(torch.int64).bitwise_and(0xFFFFFFFF)
    ref_k, ref_i = torch.sort(k32, stable=True)
    kd = k32.to(torch.int32).cuda()  # bit pattern of the u32 keys
    vd = torch.arange(n, dtype=torch.int32, device="cuda")
    ws = torch.empty(_lib.lib().kfa_radix_ws_bytes(n), dtype=torch.uint8, device="cuda")
    _lib.call("kfa_radix_sort_pairs", kd.data_ptr(), vd.data_ptr(), n, nbits, ws.data_ptr(), ws.numel(),
              _lib.stream())
    got_k = kd.cpu().to(torch.int64).bitwise_and(0xFFFFFFFF)
    assert torch.equal(got_k, ref_k)
    assert torch.equal(vd.cpu().to(torch.int64), ref_i)


@pytest.mark.parametrize("n,nbits", [(5000, 25), (70000, 17), (4097, 10)])
def test_own_radix_sort_ignores_bits_above_nbits(n, nbits):
    """hipCUB end_bit semantics: keys carrying bits at and above nbits sort on the
    low nbits only (stable), the high bits travel with the key unchanged."""
    from kubeflow_controller_amd.ops import _lib
    _lib.register("kfa_radix_ws_bytes", [_lib.L], restype=_lib.L)
    _lib.register("kfa_radix_sort_pairs", [_lib.P, _lib.P, _lib.L, _lib.I, _lib.P, _lib.L, _lib.P])
    g = torch.Generator().manual_seed(n * 3 + nbits)
    low = torch.randint(0, 1 << nbits, (n,), generator=g, dtype=torch.int64)
    low[: n // 4] = low[: n // 4] % 13
    high = torch.randint(0, 1 << (32 - nbits), (n,), generator=g, dtype=torch.int64) << nbits
    k32 = (low | high).bitwise_and(0xFFFFFFFF)
    _, ref_i = torch.sort(low, stable=True)
    kd = k32.to(torch.int32).cuda()
    vd = torch.arange(n, dtype=torch.int32, device="cuda")
    ws = torch.empty(_lib.lib().kfa_radix_ws_bytes(n), dtype=torch.uint8, device="cuda")
    _lib.call("kfa_radix_sort_pairs", kd.data_ptr(), vd.data_ptr(), n, nbits, ws.data_ptr(), ws.numel(),
              _lib.stream())
    assert torch.equal(vd.cpu().to(torch.int64), ref_i)
    assert torch.equal(kd.cpu().to(torch.int64).bitwise_and(0xFFFFFFFF), k32[ref_i])


@pytest.mark.parametrize("n", [1, 63, 1024, 1025, 26561, 300000])
def test_scan_max_exclusive(n):
    from kubeflow_controller_amd.ops import _lib
    _lib.register("kfa_scan_max_excl", [_lib.P, _lib.L, _lib.I, _lib.P])
    g = torch.Generator().manual_seed(n)
    a = torch.randint(-1, 1 << 20, (n,), generator=g, dtype=torch.int32)
    a[torch.rand(n, generator=g) < 0.5] = -1
    ref = torch.cummax(torch.cat([torch.tensor([-1], dtype=torch.int32), a[:-1]]), 0).values
    d = a.cuda()
    _lib.call("kfa_scan_max_excl", d.data_ptr(), n, -1, _lib.stream())
    assert torch.equal(d.cpu(), ref)
