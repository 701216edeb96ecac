"""Averages rocprofv3 --pmc counter_collection CSVs per (kernel, grid): python tools/pmc_summary.py dir1 [dir2 ...]"""
import csv
import glob
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = (r["Kernel_Name"][:70], r.get("Grid_Size", r.get("Grid_Size_X", "")))
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    print("   " + "  ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(cs.items())))
