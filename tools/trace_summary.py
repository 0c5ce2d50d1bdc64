"""Per-step kernel time table from a rocprofv3 kernel trace (grouped by kernel + grid).
usage: python tools/trace_summary.py <run_kernel_trace.csv> <steps_profiled> [top]"""
import collections
import csv
import sys


def main():
    path, steps = sys.argv[1], int(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    agg = collections.defaultdict(lambda: [0, 0])
    for r in csv.DictReader(open(path)):
        key = (r["Kernel_Name"][:80], r["Grid_Size_X"], r["Grid_Size_Y"], r["Workgroup_Size_X"])
        agg[key][0] += 1
        agg[key][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    tot = sum(v[1] for v in agg.values())
    print(f"total kernel ms/step: {tot / 1e6 / steps:.2f}")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{v[1] / 1e6 / steps:7.2f} ms {v[0] / steps:6.1f}x {v[1] / v[0] / 1e3:8.1f}us  {k[0]}  grid={k[1]}x{k[2]} wg={k[3]}")


if __name__ == "__main__":
    main()
