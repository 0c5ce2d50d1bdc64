"""Per-kernel HBM traffic and bandwidth from two rocprofv3 counter passes (FETCH_SIZE alone, WRITE_SIZE alone: their
TCC counters do not fit one pass), following MI355X_MICROARCH.md's HBM recipe: bytes = FETCH_SIZE x 2 (gfx950
tallies 128-B requests at 64 B) x 1024 + WRITE_SIZE x 1024 (both counters in KB); time = the dispatch's own
Start/End timestamps in the FETCH pass (counter passes serialise dispatches, so this is each kernel alone).
GB/s is against ~8 TB/s peak HBM3E.
usage: python tools/hbm_summary.py FETCH.csv WRITE.csv [--top 16] [--steps N]"""
import argparse
import collections
import csv
import re


def short(name):
    return re.sub(r"\(.*$", "", name).replace("void ", "")[:80]


def load(path, counter):
    vals, durs = collections.defaultdict(list), collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = short(r["Kernel_Name"])
        vals[k].append(float(r["Counter_Value"]))
        durs[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return vals, durs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--top", type=int, default=16)
    ap.add_argument("--steps", type=int, default=3, help="profiled steps (warm-up included) for the per-step column")
    a = ap.parse_args()
    fv, fd = load(a.fetch, "FETCH_SIZE")
    wv, _ = load(a.write, "WRITE_SIZE")
    rows = []
    for k in fv:
        n = len(fv[k])
        fb = sum(fv[k]) * 2 * 1024 / n
        wb = sum(wv.get(k, [0.0])) * 1024 / max(1, len(wv.get(k, [0.0])))
        t = sum(fd[k]) / n
        rows.append((sum(fd[k]), k, n, fb, wb, t))
    rows.sort(reverse=True)
    print(f"# HBM traffic per kernel (FETCH_SIZE x2 + WRITE_SIZE), `{a.fetch}` / `{a.write}`\n")
    print("| kernel | launches | avg us (counter pass) | fetch MB / launch | write MB / launch | GB/s | fraction of 8 TB/s |")
    print("|---|---|---|---|---|---|---|")
    for tot, k, n, fb, wb, t in rows[:a.top]:
        gbs = (fb + wb) / t / 1e9 if t > 0 else 0.0
        print(f"| `{k}` | {n} | {t * 1e6:.1f} | {fb / 1e6:.1f} | {wb / 1e6:.1f} | {gbs:.0f} | {gbs / 8000:.3f} |")


if __name__ == "__main__":
    main()
