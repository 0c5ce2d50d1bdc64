"""Per-kernel averages of every counter in rocprofv3 `--pmc` counter-collection CSVs.

usage: python tools/pmc_dump.py gpurun_out/x/run_counter_collection.csv [more.csv ...] [--match REGEX]
Prints, per kernel: launches, mean duration, and each counter's mean per dispatch; SQ_WAVE_CYCLES-relative
fractions of the SQ_WAIT_* / SQ_ACTIVE_* buckets when present (quad-cycle counters, MI355X_MICROARCH.md)."""
import argparse
import collections
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for path in a.csv:
        disp = {}
        with open(path) as f:
            for r in csv.DictReader(f):
                if a.match and not re.search(a.match, r["Kernel_Name"]):
                    continue
                d = disp.setdefault(r["Dispatch_Id"], {"name": re.sub(r"\(.*$", "", r["Kernel_Name"]).replace("void ", ""),
                                                       "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                                       "c": {}})
                d["c"][r["Counter_Name"]] = float(r["Counter_Value"])
        for d in disp.values():
            k = agg[d["name"]]
            k["_n_" + path] += 1
            k["_ns"] += d["ns"]
            k["_n"] += 1
            for c, v in d["c"].items():
                k[c] += v
                k["_cnt_" + c] += 1
    for name, k in sorted(agg.items(), key=lambda kv: -kv[1]["_ns"]):
        print(f"## {name}: {int(k['_n'])} dispatches, {k['_ns'] / k['_n'] / 1e3:.1f} us avg")
        cs = sorted(c for c in k if not c.startswith("_"))
        means = {c: k[c] / k["_cnt_" + c] for c in cs}
        for c in cs:
            print(f"   {c:32s} {means[c]:16.4g}")
        wc = means.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_MISC", "SQ_ACTIVE_INST_SCA"):
                if c in means:
                    print(f"   frac {c:27s} {means[c] / wc:8.3f}")


if __name__ == "__main__":
    main()
