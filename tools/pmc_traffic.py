"""Per-launch HBM traffic of one kernel from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE in separate runs, MI355X_MICROARCH.md §HBM):
bytes = 2 * FETCH_SIZE[KB] * 1024 (gfx950 reports half of a wide coalesced read)
      +     WRITE_SIZE[KB] * 1024.
usage: python tools/pmc_traffic.py <fetch_csv> <write_csv> <kernel-substring> <out.json>"""
import csv
import json
import statistics
import sys


def med(path, counter, sub):
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
         if r["Counter_Name"] == counter and sub in r["Kernel_Name"]]
    return statistics.median(v), len(v)


if __name__ == "__main__":
    fetch_csv, write_csv, sub, out = sys.argv[1:5]
    f, nf = med(fetch_csv, "FETCH_SIZE", sub)
    w, nw = med(write_csv, "WRITE_SIZE", sub)
    res = {"kernel": sub, "fetch_size_kb_median": f, "write_size_kb_median": w, "launches": [nf, nw],
           "fetch_bytes_corrected": 2 * f * 1024, "write_bytes": w * 1024,
           "traffic_bytes_per_launch": 2 * f * 1024 + w * 1024,
           "correction": "FETCH_SIZE x2 (gfx950 tallies 128-B requests at 64 B); WRITE_SIZE exact for 16-B stores"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))
