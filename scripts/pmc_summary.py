#!/usr/bin/env python3
"""Condense rocprofv3 counter collections (run_counter_collection.csv, one
row per dispatch x counter) into per-kernel averages per dispatch: one CSV row
per (kernel, counter) with the dispatch count.  Used to keep the committed
profiles/ summaries small.

  python scripts/pmc_summary.py out.csv dir1/run_counter_collection.csv [dir2/... ...]
"""

import collections
import csv
import sys


def main():
    out, files = sys.argv[1], sys.argv[2:]
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for f in files:
        for r in csv.DictReader(open(f)):
            if "at::native" in r["Kernel_Name"]:  # torch's own kernels (tensor setup)
                continue
            key = (r["Kernel_Name"], r["Counter_Name"])
            tot[key] += float(r["Counter_Value"])
            disp[key].add((f, r["Dispatch_Id"]))
    with open(out, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Kernel_Name", "Counter_Name", "Dispatches", "Average_Per_Dispatch"])
        for (k, c), v in sorted(tot.items()):
            n = len(disp[(k, c)])
            w.writerow([k, c, n, v / n])


if __name__ == "__main__":
    main()
