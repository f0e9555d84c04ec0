"""Statistics of the fused attention's dropout decisions (csrc/kernels/attention.hip:
one counter hash per (q, k) / (q, k + 16) score pair, 16-bit halves against
t16 = round(p·2^16)), checked on a numpy copy of the hash: keep rate, independence
of the two halves of a pair, of neighbouring keys and of neighbouring rows.
The GPU test (tests/test_attention_gpu.py) pins the kernels to this same copy."""
import numpy as np
import pytest

from test_attention_gpu import _drop_hash  # noqa: E402  (numpy copy of common.h drop_hash)


def _keeps(seed, rows, S, p):
    t16 = min(int(p * 65536.0 + 0.5), 65536)
    key = np.arange(S, dtype=np.uint64)
    idx = np.arange(rows, dtype=np.uint64)[:, None] * np.uint64(S) + (key & ~np.uint64(16))[None, :]
    h = _drop_hash(np.uint64(seed), idx)
    half = np.where((key & np.uint64(16)) != 0, h >> np.uint32(16), h & np.uint32(0xFFFF))
    return (half >= t16), t16


@pytest.mark.parametrize("p", [0.1, 0.5])
def test_pair_hash_dropout_statistics(p):
    rows, S = 4096, 128
    keep, t16 = _keeps(0x1234_5678_9ABC_DEF1, rows, S, p)
    n = keep.size
    rate = keep.mean()
    want = 1.0 - t16 / 65536.0
    assert abs(want - (1.0 - p)) < 1e-4
    sigma = np.sqrt(want * (1 - want) / n)
    assert abs(rate - want) < 5 * sigma, (rate, want)
    x = keep.astype(np.float64) - rate

    def corr(a, b):
        return float((a * b).mean() / np.sqrt((a * a).mean() * (b * b).mean()))

    lim = 5.0 / np.sqrt(n / 2)
    lo = x.reshape(rows, S // 32, 2, 16)
    assert abs(corr(lo[:, :, 0], lo[:, :, 1])) < lim  # the two halves of one hash
    assert abs(corr(x[:, :-1], x[:, 1:])) < lim        # neighbouring keys
    assert abs(corr(x[:-1], x[1:])) < lim              # neighbouring rows (queries)
    # per-key / per-row keep rates show no structure beyond binomial noise
    col = keep.mean(0)
    assert np.abs(col - want).max() < 6 * np.sqrt(want * (1 - want) / rows)


def test_pair_hash_seeds_differ():
    a, _ = _keeps(1, 256, 128, 0.1)
    b, _ = _keeps(2, 256, 128, 0.1)
    agree = (a == b).mean()
    assert abs(agree - (0.9 * 0.9 + 0.1 * 0.1)) < 0.01


def test_seed_crosses_autograd_as_signed_int64_with_the_same_masks():
    """Seeds reach torch.autograd.Function.apply as signed int64 (torch's profiler
    rejects Python ints >= 2^63 there); the mask keys must not change."""
    from kubeflow_controller_amd.ops import transformer as T
    for s in (0, 5, 2**63 - 1, 2**63, 2**63 + 12345, 2**64 - 1):
        v = T.s64(s)
        assert -(2**63) <= v < 2**63
        assert T.hash_key(v) == T.hash_key(s)
        assert T.mix_seed(v, 3) == T.mix_seed(s, 3)
