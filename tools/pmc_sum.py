"""Average each PMC counter over the dispatches of kernels whose name contains a substring.
usage: python tools/pmc_sum.py run_counter_collection.csv <substring> [label]"""
import collections
import csv
import sys

agg = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r["Kernel_Name"]:
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[3] if len(sys.argv) > 3 else "", {k: f"{sum(v) / len(v):.4g}" for k, v in sorted(agg.items())}, flush=True)
