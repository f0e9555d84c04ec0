"""Time the own LSD radix sort (csrc/kernels/radix_sort.h) on W&D-shaped ids.

1.7 M keys of 25 bits, (a) uniform and (b) skewed like the W&D batch (~30 %
distinct: a Zipf-ish mix of hot ids), against torch.sort (rocPRIM) for scale.
Prints one line per case: us per sort_pairs call.
"""
import torch

from kubeflow_controller_amd.ops import _lib


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1000


def main():
    _lib.register("kfa_radix_ws_bytes", [_lib.L], restype=_lib.L)
    _lib.register("kfa_radix_sort_pairs", [_lib.P, _lib.P, _lib.L, _lib.I, _lib.P, _lib.L, _lib.P])
    n, nbits = 1_700_000, 25
    g = torch.Generator().manual_seed(0)
    uni = torch.randint(0, 1 << nbits, (n,), generator=g)
    hot = torch.randint(0, 1 << nbits, (4096,), generator=g)
    pick = (torch.rand(n, generator=g) ** 3 * 4096).long()   # skewed towards the first hot ids
    skew = torch.where(torch.rand(n, generator=g) < 0.7, hot[pick], uni)
    ws = torch.empty(_lib.lib().kfa_radix_ws_bytes(n), dtype=torch.uint8, device="cuda")
    for name, keys in (("uniform", uni), ("skewed", skew)):
        k0 = keys.to(torch.int32).cuda()
        v0 = torch.arange(n, dtype=torch.int32, device="cuda")
        k, v = k0.clone(), v0.clone()

        def own():
            k.copy_(k0)
            v.copy_(v0)
            _lib.call("kfa_radix_sort_pairs", k.data_ptr(), v.data_ptr(), n, nbits, ws.data_ptr(), ws.numel(),
                      _lib.stream())

        t_copy = timeit(lambda: (k.copy_(k0), v.copy_(v0)))
        t_own = timeit(own) - t_copy
        t_torch = timeit(lambda: torch.sort(k0, stable=True))
        own()
        ref = torch.sort(k0.long(), stable=True)
        ok = torch.equal(k.long(), ref.values) and torch.equal(v.long(), ref.indices)
        print(f"radix {name:8s} n={n}: own {t_own:7.1f} us   torch.sort {t_torch:7.1f} us   match={ok}", flush=True)


if __name__ == "__main__":
    main()
