"""Kernel statistics (the rocprofv3 --stats table: name, calls, total / average ns, share) from a rocpd
SQLite database (rocprofv3's default output on ROCm 7.2), written as CSV."""
import csv
import sqlite3
import sys

db, out = sys.argv[1], sys.argv[2]
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name_col = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else None)
rows = c.execute(f"select {name_col}, start, end from kernels").fetchall()
agg = {}
for n, s, e in rows:
    d = e - s
    t = agg.setdefault(n, [0, 0, None, 0])
    t[0] += 1
    t[1] += d
    t[2] = d if t[2] is None else min(t[2], d)
    t[3] = max(t[3], d)
tot = sum(v[1] for v in agg.values())
with open(out, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for n, (k, s, mn, mx) in sorted(agg.items(), key=lambda x: -x[1][1]):
        w.writerow([n, k, s, round(s / k, 1), round(100.0 * s / tot, 3), mn, mx])
print("kernels", len(rows), "total ms", tot / 1e6)
