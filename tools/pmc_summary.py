"""Summarise a rocprofv3 `--pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES [GRBM_GUI_ACTIVE]`
pass per kernel: the top-N kernels by total time, with

  mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (active cycles x 1024 SIMDs)

where active cycles = GRBM_GUI_ACTIVE / 8 (the counter sums the 8 XCDs) when it was collected, else the kernel's
duration x the clock given by --clock-ghz.  SQ_VALU_MFMA_BUSY_CYCLES counts SIMD cycles (32 per 32x32x16 bf16 MFMA,
MI355X_MICROARCH.md), so mfma_util is the fraction of the chip's MFMA issue capacity the kernel used.  Also
printed: the raw ratio SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CYCLES and the mean waves per launch.

usage: python tools/pmc_summary.py gpurun_out/sqpmc/run_counter_collection.csv [--top 6] [--clock-ghz 2.4]
"""
import argparse
import collections
import csv
import re


def short(name):
    name = re.sub(r"\(.*$", "", name)           # drop the argument list
    return name.replace("void ", "")[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=6)
    ap.add_argument("--clock-ghz", type=float, default=2.4)
    a = ap.parse_args()
    disp = {}
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            d = disp.setdefault(r["Dispatch_Id"], {"name": r["Kernel_Name"],
                                                   "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
            d[r["Counter_Name"]] = float(r["Counter_Value"])
    agg = collections.defaultdict(lambda: collections.Counter())
    for d in disp.values():
        k = agg[short(d["name"])]
        k["n"] += 1
        for key in ("ns", "SQ_BUSY_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_WAVES", "GRBM_GUI_ACTIVE"):
            k[key] += d.get(key, 0.0)
    total_ns = sum(k["ns"] for k in agg.values())
    rows = sorted(agg.items(), key=lambda kv: -kv[1]["ns"])[:a.top]
    print(f"# {a.csv}: {len(disp)} dispatches, {total_ns / 1e6:.2f} ms total kernel time")
    print("| kernel | launches | avg us | % time | MFMA busy / SQ busy | mfma_util | waves/launch |")
    print("|---|---|---|---|---|---|---|")
    for name, k in rows:
        if k["GRBM_GUI_ACTIVE"]:
            active = k["GRBM_GUI_ACTIVE"] / 8.0
        else:
            active = k["ns"] * a.clock_ghz
        util = k["SQ_VALU_MFMA_BUSY_CYCLES"] / (active * 1024.0) if active else 0.0
        raw = k["SQ_VALU_MFMA_BUSY_CYCLES"] / k["SQ_BUSY_CYCLES"] if k["SQ_BUSY_CYCLES"] else 0.0
        print(f"| `{name}` | {int(k['n'])} | {k['ns'] / k['n'] / 1e3:.1f} | {100 * k['ns'] / total_ns:.1f} | "
              f"{raw:.2f} | {util:.3f} | {k['SQ_WAVES'] / k['n']:.0f} |")


if __name__ == "__main__":
    main()
