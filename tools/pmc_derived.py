"""Derived per-kernel metrics from rocprofv3 --pmc passes (markdown table).

    python tools/pmc_derived.py gpurun_out/pmc_r4/p*/p_counter_collection.csv

Counters are summed per dispatch over the CSV rows (one row per XCD / SE
instance), then averaged over the dispatches of the pass that collected them.
On MI355X (8 XCDs x 32 CUs x 4 SIMDs) the derived columns are:

* MFMA busy  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 256 CUs x 4 SIMDs)
  (GRBM_GUI_ACTIVE sums the 8 XCDs' clocks);
* MFMA TF/s  = SQ_INSTS_MFMA x 16,384 flop (v_mfma_f32_16x16x32_bf16) / dispatch time
  — valid for the bf16 16x16x32 kernels only (every own GEMM / conv / wgrad);
* LDS conflict = SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS (extra LDS cycles per LDS-busy cycle);
* LDS-wait share = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES;
* HBM read / write = FETCH_SIZE / WRITE_SIZE (KiB counters) per dispatch, and their sum over time.
"""
import collections
import csv
import sys

CUS, SIMDS, XCDS = 256, 4, 8


def load(paths):
    vals = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    dur = collections.defaultdict(dict)
    for path in paths:
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:48]
            d = (path, r["Dispatch_Id"])
            vals[k][r["Counter_Name"]][d] += float(r["Counter_Value"])
            dur[k][d] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    out = {}
    for k, cs in vals.items():
        mean = {c: sum(v.values()) / len(v) for c, v in cs.items()}
        mean["_us"] = sum(dur[k].values()) / len(dur[k]) / 1e3
        mean["_n"] = len(dur[k])
        out[k] = mean
    return out


def fmt(v, spec):
    return "—" if v is None else format(v, spec)


def main(paths, keep=("gemm", "wgrad", "conv", "seg_", "radix", "scan_max", "bn_", "attn", "ln_", "bias_act",
                      "maxpool", "pool", "stem", "sgd", "adam", "xent", "gap_")):
    rows = load(paths)
    print("| kernel | dispatches | mean us | MFMA busy | MFMA TF/s | LDS conflict | LDS-wait share | "
          "HBM read MB | HBM write MB | HBM TB/s |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for k, m in sorted(rows.items(), key=lambda kv: -kv[1]["_us"] * kv[1]["_n"]):
        if not any(s in k for s in keep):
            continue
        us = m["_us"]
        g = m.get("GRBM_GUI_ACTIVE")
        busy = m.get("SQ_VALU_MFMA_BUSY_CYCLES")
        mb = busy / (g / XCDS * CUS * SIMDS) if g and busy is not None else None
        mf = m.get("SQ_INSTS_MFMA")
        tf = mf * 16384 / (us * 1e-6) / 1e12 if mf else None
        lds = m.get("SQ_ACTIVE_INST_LDS")
        conf = m["SQ_LDS_BANK_CONFLICT"] / lds if lds else None
        wl = m["SQ_WAIT_INST_LDS"] / m["SQ_WAVE_CYCLES"] if m.get("SQ_WAVE_CYCLES") and "SQ_WAIT_INST_LDS" in m else None
        rd = m["FETCH_SIZE"] / 1024 if "FETCH_SIZE" in m else None
        wr = m["WRITE_SIZE"] / 1024 if "WRITE_SIZE" in m else None
        bw = (rd or 0) + (wr or 0)
        tbs = bw * 1e6 / (us * 1e-6) / 1e12 if rd is not None or wr is not None else None
        print(f"| `{k}` | {m['_n']} | {us:.1f} | {fmt(mb and mb * 100, '.0f')}% | {fmt(tf, '.0f')} | "
              f"{fmt(conf and conf * 100, '.0f')}% | {fmt(wl and wl * 100, '.1f')}% | {fmt(rd, '.1f')} | "
              f"{fmt(wr, '.1f')} | {fmt(tbs, '.2f')} |")


def issue(paths, keep=("attn", "gemm", "wgrad", "conv", "ln_", "bias_act")):
    """Per-wave issue mix (passes with SQ_INSTS_* and SQ_WAVES): instructions per wave
    and the share of wave cycles spent issuing VALU / waiting."""
    rows = load(paths)
    print("| kernel | dispatches | mean us | VALU / wave | SALU / wave | MFMA / wave | LDS / wave | "
          "VALU-active share | wait-any share |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|")
    for k, m in sorted(rows.items(), key=lambda kv: -kv[1]["_us"] * kv[1]["_n"]):
        w = m.get("SQ_WAVES")
        if not any(s in k for s in keep) or not w or "SQ_INSTS_VALU" not in m:
            continue
        per = lambda c: fmt(m[c] / w if c in m else None, ".0f")  # noqa: E731
        wc = m.get("SQ_WAVE_CYCLES")
        va = m["SQ_ACTIVE_INST_VALU"] / wc if wc and "SQ_ACTIVE_INST_VALU" in m else None
        wa = m["SQ_WAIT_ANY"] / wc if wc and "SQ_WAIT_ANY" in m else None
        print(f"| `{k}` | {m['_n']} | {m['_us']:.1f} | {per('SQ_INSTS_VALU')} | {per('SQ_INSTS_SALU')} | "
              f"{per('SQ_INSTS_MFMA')} | {per('SQ_INSTS_LDS')} | {fmt(va and va * 100, '.0f')}% | "
              f"{fmt(wa and wa * 100, '.0f')}% |")


if __name__ == "__main__":
    if sys.argv[1:2] == ["--issue"]:
        issue(sys.argv[2:])
    else:
        main(sys.argv[1:])
